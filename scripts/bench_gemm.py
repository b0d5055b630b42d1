"""Per-shape batched MFMA GEMM micro-benchmark (Llama-3.1-8B prefill / multi-user shapes, TP1 and
TP8 shards): us per launch and effective weight-stream TB/s (8 weight copies cycled so the 256 MB
infinity cache cannot hold them). usage: python scripts/bench_gemm.py [tokens ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
EPI_STORE, EPI_ACT_F16 = 0, 4
shapes = [
    ("qkv  tp1", 6144, 4096, EPI_STORE),
    ("wo   tp1", 4096, 4096, EPI_STORE),
    ("w13  tp1", 28672, 4096, EPI_ACT_F16),
    ("w2   tp1", 4096, 14336, EPI_STORE),
    ("wcls tp1", 128256, 4096, EPI_STORE),
    ("qkv  tp8", 768, 4096, EPI_STORE),
    ("wo   tp8", 4096, 512, EPI_STORE),
    ("w13  tp8", 3584, 4096, EPI_ACT_F16),
    ("w2   tp8", 4096, 1792, EPI_STORE),
]
tokens = [int(x) for x in sys.argv[1:]] or [8, 16, 32, 64]
for name, rows, n, epi in shapes:
    mb = rows * n * 0.5625 / 1e6
    line = f"{name} {rows:6d}x{n:5d} {mb:7.1f} MB |"
    for m in tokens:
        us = C.bench_gemm_q40(rows, n, m, epi, 8 if mb < 100 else 2, 50)
        line += f" M={m}: {us:7.2f} us {mb / us:5.2f} TB/s |"
    print(line, flush=True)
