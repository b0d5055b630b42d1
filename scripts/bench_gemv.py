"""Per-shape GEMV micro-benchmark (Llama-3.1-8B decode shapes, TP1 and TP8 shards)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
PRO_GLOBAL, PRO_RESNORM = 0, 1
EPI_STORE, EPI_ACT, EPI_QKV, EPI_ACT_Q80 = 0, 1, 2, 3
shapes = [
    # name, rows, n, pro, epi
    ("qkv  tp1", 6144, 4096, PRO_RESNORM, EPI_STORE),
    ("qkvQ tp1", 6144, 4096, PRO_RESNORM, EPI_QKV),
    ("qkvG tp1", 6144, 4096, PRO_GLOBAL, EPI_STORE),
    ("wo   tp1", 4096, 4096, PRO_GLOBAL, EPI_STORE),
    ("w13  tp1", 28672, 4096, PRO_RESNORM, EPI_ACT_Q80),
    ("w2   tp1", 4096, 14336, PRO_GLOBAL, EPI_STORE),
    ("w13f tp1", 28672, 4096, PRO_RESNORM, EPI_ACT),
    ("w2q  tp1", 4096, 14336, PRO_RESNORM, EPI_STORE),
    ("wcls tp1", 128256, 4096, PRO_RESNORM, EPI_STORE),
    ("qkv  tp8", 768, 4096, PRO_RESNORM, EPI_STORE),
    ("wo   tp8", 4096, 512, PRO_GLOBAL, EPI_STORE),
    ("w13  tp8", 3584, 4096, PRO_RESNORM, EPI_ACT),
    ("w2   tp8", 4096, 1792, PRO_RESNORM, EPI_STORE),
]
variants = [l for l in sys.argv[1:]] or ["auto"]
for name, rows, n, pro, epi in shapes:
    mb = rows * n * 0.5625 / 1e6
    line = f"{name} {rows:6d}x{n:5d} {mb:7.1f} MB |"
    for v in variants:
        lanes, passes = 0, 0  # 0 = engine default (lanes per row / residency rule)
        if v != "auto":
            lanes, passes = [int(x) for x in v.split("x")]
        us = C.bench_gemv_q40(rows, n, pro, epi, int(os.environ.get("BATCH", "1")), lanes, passes,
                              int(os.environ.get("COPIES", "8")), 200)
        line += f" {v}: {us:6.2f} us {mb / us:5.2f} TB/s |"
    print(line, flush=True)
