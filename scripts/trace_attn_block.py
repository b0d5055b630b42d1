"""Timeline of one fused attention-block launch (8B decode shapes, TP1): per role, the median and
spread of workgroup entry / wait-done / exit times (us from the earliest entry), so the hand-offs
(qkv -> attention -> wo) can be priced. usage: python scripts/trace_attn_block.py [pos] [tp]
(tp > 1: rank 0 of a TP-tp group with the exchange in loopback, ComputeOnlyComm)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
pos = int(sys.argv[1]) if len(sys.argv) > 1 else 100
tp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
h = dict(dim=4096, hidden_dim=14336, n_layers=4, n_heads=32, n_kv_heads=8, vocab_size=128256, seq_len=pos + 64,
         rope_theta=500000, weight_type=2)
eng = C.HipEngine("", "q80", synthetic=h, max_seq_len=pos + 64, sync_type="q80",
                  **({} if tp == 1 else dict(rank=0, world=tp, comm=C.ComputeOnlyComm(0, tp, 0))))
assert eng.attn_block
for p in range(0, pos, 32):  # fill the KV cache
    n = min(32, pos - p)
    eng.forward_argmax([1] * n, list(range(p, p + n)), [0] * n)
for rep in range(3):
    t = eng.trace_attn_block(7, pos + rep, 0, 2)
gq, ga, gw = t[:3]
tr = np.array(t[3:], dtype=np.int64).reshape(-1, 8)
t0 = tr[:, 0][tr[:, 0] > 0].min()
us = lambda v: (v - t0) / 100.0  # s_memrealtime: 100 MHz
def row(name, idx, cols):
    sub = tr[idx]
    out = f"{name:10s} n={len(sub):3d} |"
    for c, label in cols:
        v = us(sub[:, c][sub[:, c] > 0])
        if len(v):
            out += f" {label} med {np.median(v):6.2f} [{v.min():6.2f} .. {v.max():6.2f}] |"
    print(out)
q = np.arange(gq); a = np.arange(gq, gq + ga); w = np.arange(gq + ga, gq + ga + gw)
row("qkv", q, [(0, "entry"), (1, "ready"), (5, "first"), (2, "exit")])
row("attention", a, [(0, "entry"), (1, "waited"), (2, "computed"), (3, "exit")])
row("wo", w, [(0, "entry"), (6, "waited"), (1, "ready"), (2, "exit")])
