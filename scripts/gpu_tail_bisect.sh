# TP8 wo / w2 GEMV with the TP tail in loopback (f32 / Q80) vs without, and the TP-rank decode.
set -o pipefail
mkdir -p gpurun_out/tail
R=gpurun_out/tail/after.log
COPIES=48 timeout -k 10 100 python -u scripts/trace_gemv.py wo8 w2_8 wo8tp w2_8tp 2>&1 | grep -v "exit by\|amdgpu" >> $R || exit 1
DL_BENCH_TP_Q80=0 COPIES=48 timeout -k 10 100 python -u scripts/trace_gemv.py wo8tp w2_8tp 2>&1 | grep -v "exit by\|amdgpu" >> $R || exit 1
for n in 2 4 8; do timeout -k 10 120 python -u scripts/tp_rank_compute.py --tp $n 2>&1 | grep -v "^ℹ\|amdgpu" >> $R || exit 1; done
timeout -k 10 120 python -u scripts/tp_rank_compute.py --tp 8 --sync-type f32 2>&1 | grep -v "^ℹ\|amdgpu" >> $R || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_xgmi.py tests/test_gpu_engine.py tests/test_gpu_rccl.py > gpurun_out/tail/tests.log 2>&1
