"""One GEMM and one GEMV launch series for PMC passes (rocprofv3 --pmc): w13 (28672 x 4096) at
M tokens through the batched MFMA GEMM, and the batch-1 GEMV on the same shape for comparison."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl

C = dl.native()
M = int(os.environ.get("M", "8"))
rows, n = int(os.environ.get("ROWS", "28672")), int(os.environ.get("N", "4096"))
print("gemm us", C.bench_gemm_q40(rows, n, M, 0, 4, 20), flush=True)
print("gemv us", C.bench_gemv_q40(rows, n, 1, 0, 1, 0, 0, 4, 20), flush=True)
