"""GEMV lanes x passes sweep on the Llama-3.3-70B decode shapes (TP1): us per launch in a graph of
200, 4 weight copies cycled (each copy >= 46 MB: no MALL reuse), TB/s of Q40 bytes. The engine's
default is 'auto'. usage: python scripts/sweep_gemv_big.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402

C = dl.native()
PRO_GLOBAL, PRO_RESNORM = 0, 1
EPI_STORE, EPI_ACT, EPI_QKV, EPI_ACT_Q80 = 0, 1, 2, 3
shapes = [("qkv  70b", 10240, 8192, PRO_RESNORM, EPI_STORE), ("wo   70b", 8192, 8192, PRO_GLOBAL, EPI_STORE),
          ("w13  70b", 57344, 8192, PRO_RESNORM, EPI_ACT_Q80), ("w2   70b", 8192, 28672, PRO_GLOBAL, EPI_STORE),
          ("wcls 70b", 128256, 8192, PRO_RESNORM, EPI_STORE)]
variants = ["auto", "16x1", "16x2", "16x4", "16x8", "32x1", "32x2", "32x4", "32x8", "64x1", "64x2", "64x8"]
for name, rows, n, pro, epi in shapes:
    mb = rows * n * 0.5625 / 1e6
    line = f"{name} {rows:6d}x{n:5d} {mb:7.1f} MB |"
    for v in variants:
        lanes, passes = (0, 0) if v == "auto" else [int(x) for x in v.split("x")]
        if epi == EPI_ACT_Q80 and lanes and (256 // lanes * 2 * passes) % 64:
            continue
        if (256 // max(lanes, 16) * 2 * max(passes, 1)) > rows:
            continue
        us = C.bench_gemv_q40(rows, n, pro, epi, 1, lanes, passes, 4, 100)
        line += f" {v}: {us:6.2f} {mb / us:4.2f} |"
    print(line, flush=True)
