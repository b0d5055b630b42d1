"""8B FFN GEMV pair, two hand-off formats: w13 SwiGLU -> Q80 blocks (whole 32-hidden blocks per
workgroup: 448 workgroups of 64 rows) + w2 reading Q80, vs w13 SwiGLU -> f32 on a balanced grid
(lanes x passes giving 256 workgroups) + w2 quantizing the f32 rows in its prologue. us per launch
(graph of 200, 8 weight copies)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402

C = dl.native()
PRO_GLOBAL, PRO_RESNORM = 0, 1
EPI_STORE, EPI_ACT, EPI_ACT_Q80 = 0, 1, 3
r = {}
r["w13 q80 auto"] = C.bench_gemv_q40(28672, 4096, PRO_RESNORM, EPI_ACT_Q80, 1, 0, 0, 8, 200)
r["w13 q80 16x4"] = C.bench_gemv_q40(28672, 4096, PRO_RESNORM, EPI_ACT_Q80, 1, 16, 4, 8, 200)
for lp in ((32, 7), (64, 14), (16, 4), (16, 7)):
    r[f"w13 f32 {lp[0]}x{lp[1]}"] = C.bench_gemv_q40(28672, 4096, PRO_RESNORM, EPI_ACT, 1, lp[0], lp[1], 8, 200)
r["w2 q80-in auto"] = C.bench_gemv_q40(4096, 14336, PRO_GLOBAL, EPI_STORE, 1, 0, 0, 8, 200)
r["w2 f32-in auto"] = C.bench_gemv_q40(4096, 14336, PRO_RESNORM, EPI_STORE, 1, 0, 0, 8, 200)
for k, v in r.items():
    print(f"{k:18s} {v:7.2f} us", flush=True)
