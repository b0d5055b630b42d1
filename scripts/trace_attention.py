"""Timeline of one long-context MFMA decode-attention launch (kernels.h AttnArgs::trace): per
phase, median [min .. max] over the workgroups of the stamp, us from the earliest entry.
usage: python scripts/trace_attention.py [pos] [seq_len] [batch] [tp]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402

pos = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
seq = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
tp = int(sys.argv[4]) if len(sys.argv) > 4 else 1
C = dl.native()
us, t = C.trace_attention(32 // tp, 4, 128, seq, pos, B)
tr = np.array(t, dtype=np.int64).reshape(-1, 8)
live = tr[:, 0] > 0
tr = tr[live]
t0 = tr[:, 0].min()
print(f"pos {pos} seq {seq} B {B} TP{tp}: {us:.2f} us per launch in a graph; {len(tr)} workgroups traced")
names = ["entry", "DMA issued", "first tile", "loop done", "waves merged", "finish done"]
for k, name in enumerate(names):
    v = (tr[:, k] - t0) / 100.0
    print(f"  {name:13s} {np.median(v):7.2f} [{v.min():7.2f} .. {v.max():7.2f}]")
comb = tr[tr[:, 6] == 1]
if len(comb):
    v = (comb[:, 5] - comb[:, 4]) / 100.0
    w = (tr[tr[:, 6] == 0][:, 5] - tr[tr[:, 6] == 0][:, 4]) / 100.0
    print(f"  combine (last arrivers, n={len(comb)}): {np.median(v):.2f} us; hand-off (others): {np.median(w):.2f} us")
