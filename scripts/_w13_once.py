import sys; sys.path.insert(0, '/root/repo')
import distributed_llama_multiusers_amd as dl
C = dl.native()
print(C.bench_gemv_q40(28672, 4096, 1, 3, 1, 0, 2, 8, 50))
