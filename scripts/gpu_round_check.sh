# One GPU call: TP tails + TP-rank decode, the GPU test files touched by TP / engine changes, and
# the headline bench (CLI point included).
set -o pipefail
mkdir -p gpurun_out/rc
R=gpurun_out/rc/tp.log
COPIES=48 timeout -k 10 100 python -u scripts/trace_gemv.py wo8 wo8tp w2_8tp 2>&1 | grep -v "exit by\|amdgpu" >> $R || exit 1
for n in 2 4 8; do timeout -k 10 120 python -u scripts/tp_rank_compute.py --tp $n 2>&1 | grep -v "^ℹ\|amdgpu" >> $R || exit 1; done
timeout -k 10 300 python -u bench.py > gpurun_out/rc/bench.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_xgmi.py tests/test_gpu_engine.py > gpurun_out/rc/tests.log 2>&1
