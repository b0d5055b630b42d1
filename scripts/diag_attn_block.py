"""Diagnose the fused attention block on small models: which configurations hand off correctly."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import distributed_llama_multiusers_amd as dl
from distributed_llama_multiusers_amd.models.synthetic import make_test_assets
from distributed_llama_multiusers_amd.utils.mfile import FloatType

C = dl.native()
d = tempfile.mkdtemp()
tiny, _, _ = make_test_assets(d, "tiny", FloatType.Q40, seq_len=128, seed=1)
med, _, _ = make_test_assets(d + "/m", "tiny", FloatType.Q40, seq_len=512, seed=3, dim=1024, hidden_dim=12288,
                             n_heads=8, n_kv_heads=2, n_layers=2, vocab_size=2048)
for name, m in (("tiny", tiny), ("medium", med)):
    for bf16 in (True, False):
        for mb in (8, 32):
            try:
                e = C.HipEngine(m, "q80", kv_bf16=bf16, max_batch=mb)
                lg = e.forward([3], [0], [0])
                lg2 = e.forward([17], [1], [0])
                print(name, "bf16" if bf16 else "f32", "mb", mb, "block", e.attn_block, "ok", np.isfinite(lg2).all(), flush=True)
            except Exception as ex:  # noqa: BLE001
                print(name, "bf16" if bf16 else "f32", "mb", mb, "ERROR", ex, flush=True)
