"""Decode engine vs per-layer launches vs the CPU reference, single rows at positions around the
engine's context limit (medium test model). usage: python scripts/diag_pde_positions.py"""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402
from distributed_llama_multiusers_amd.models.synthetic import make_test_assets  # noqa: E402
from distributed_llama_multiusers_amd.utils.mfile import FloatType  # noqa: E402

C = dl.native()
d = tempfile.mkdtemp()
m, _, _ = make_test_assets(d, "tiny", FloatType.Q40, seq_len=512, seed=3, dim=1024, hidden_dim=12288, n_heads=8,
                           n_kv_heads=2, n_layers=2, vocab_size=2048)
rng = np.random.default_rng(1)
toks = [int(t) for t in rng.integers(0, 2048, 300)]
cpu = C.cpu_backend(m, "q80", 8)
os.environ["DL_DECODE_ENGINE"] = "0"
ref = C.HipEngine(m, "q80", kv_bf16=True, max_batch=256)
os.environ["DL_ATTN_BLOCK"] = "0"
sep = C.HipEngine(m, "q80", kv_bf16=True, max_batch=256)
del os.environ["DL_DECODE_ENGINE"], os.environ["DL_ATTN_BLOCK"]
got = C.HipEngine(m, "q80", kv_bf16=True, max_batch=256)
print("engines: pde", got.decode_engine, "block(ref)", ref.attn_block)
rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
for p, t in enumerate(toks):
    c = cpu.forward([t], [p], [0])[0]
    r = ref.forward([t], [p], [0])[0]
    s = sep.forward([t], [p], [0])[0]
    g = got.forward([t], [p], [0])[0]
    if p % 16 == 0 or 250 <= p <= 262:
        print(f"pos {p:3d}: pde/cpu {rel(g, c):.4f}  block/cpu {rel(r, c):.4f}  sep/cpu {rel(s, c):.4f}", flush=True)
