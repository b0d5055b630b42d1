"""Timeline of one narrow MFMA GEMM launch from per-workgroup stamps (gemm_dev.h gemmTrace):
dispatch skew, first stage landed, K-loop end, split hand-off, exit - per shape and token count.
usage: python scripts/trace_gemm.py [tokens ...]   (DL_GEMM_REG=64 traces the register-ring kernel)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
shapes = [("qkv  tp1", 6144, 4096, 0), ("wo   tp1", 4096, 4096, 0), ("w13  tp1", 28672, 4096, 4),
          ("w2   tp1", 4096, 14336, 0), ("qkv  tp8", 768, 4096, 0), ("w13  tp8", 3584, 4096, 4)]
for m in [int(x) for x in sys.argv[1:]] or [8]:
    for name, rows, n, epi in shapes:
        us, t, splits = C.trace_gemm_q40(rows, n, m, epi)
        a = np.array(t, dtype=np.float64).reshape(-1, 8)
        t0 = a[:, 0].min()
        rel = lambda c: (a[:, c] - t0) / 100.0  # 100 MHz ticks -> us
        comb = a[:, 6] > 0
        span = lambda x: f"{np.percentile(x, 50):6.2f}/{np.percentile(x, 90):6.2f}/{x.max():6.2f}"
        print(f"{name} M={m:3d} {us:7.2f} us/launch  WGs {len(a):5d} S={splits} | p50/p90/max us: "
              f"entry {span(rel(0))} first {span(rel(1))} loop {span(rel(2))} handoff {span(rel(3))} "
              f"exit {span(rel(4))} | combine {span(rel(4)[comb] - rel(3)[comb])} | "
              f"wg life {span(rel(4) - rel(0))} first-entry {span(rel(1) - rel(0))} loop {span(rel(2) - rel(1))}",
              flush=True)
