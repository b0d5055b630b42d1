"""Fused FFN block (w13 -> w2 in one launch) diagnostics, 8B decode shapes, TP1: the standalone
w13 / w2 GEMV times at the passes the block uses, then the block's per-role timeline (median and
spread of workgroup entry / ready / first step / wait done / exit, us from the earliest entry).
usage: python scripts/trace_ffn_block.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
for p in (2, 4):
    print(f"w13 GEMV 28672x4096 resnorm->act_q80 passes {p}: {C.bench_gemv_q40(28672, 4096, 1, 3, 1, 0, p):.2f} us", flush=True)
for p in (1, 2):
    print(f"w2  GEMV 4096x14336 global->store passes {p}: {C.bench_gemv_q40(4096, 14336, 0, 0, 1, 0, p):.2f} us", flush=True)
pos = 100
h = dict(dim=4096, hidden_dim=14336, n_layers=4, n_heads=32, n_kv_heads=8, vocab_size=128256, seq_len=pos + 64,
         rope_theta=500000, weight_type=2)
eng = C.HipEngine("", "q80", synthetic=h, max_seq_len=pos + 64)
print("ffn block:", eng.ffn_block, "attn block:", eng.attn_block, flush=True)
if not eng.ffn_block:
    sys.exit(0)
eng.forward_argmax([1] * 32, list(range(32)), [0] * 32)
for rep in range(3):
    t = eng.trace_attn_block(7, 40 + rep, 0, 2, ffn=True)
g13, _, g2 = t[:3]
tr = np.array(t[3:], dtype=np.int64).reshape(-1, 8)
t0 = tr[:, 0][tr[:, 0] > 0].min()
us = lambda v: (v - t0) / 100.0  # s_memrealtime: 100 MHz
print(f"g13 {g13} g2 {g2}")
for name, idx in (("w13", np.arange(g13)), ("w2", np.arange(g13, g13 + g2))):
    sub = tr[idx]
    out = f"{name:4s} n={len(sub):3d} |"
    for c, label in ((0, "entry"), (6, "waited"), (1, "ready"), (5, "first"), (2, "exit")):
        v = us(sub[:, c][sub[:, c] > 0])
        if len(v):
            out += f" {label} med {np.median(v):6.2f} [{v.min():6.2f} .. {v.max():6.2f}] |"
    print(out, flush=True)
