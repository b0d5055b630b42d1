"""Narrow GEMM launches at 8 tokens for a PMC pass: w13 (16-lane tiling: the 16-block-chunk kernel)
and wo (32-lane tiling: the 8-block kernel), Llama-3.1-8B shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402

C = dl.native()
print("w13 M=8", C.bench_gemm_q40(28672, 4096, 8, 4, 2, 20))
print("wo  M=8", C.bench_gemm_q40(4096, 4096, 8, 0, 2, 20))
print("w2  M=8", C.bench_gemm_q40(4096, 14336, 8, 0, 2, 20))
