# Narrow GEMM: 8- vs 4-block chunks at 32 / 64 tokens (with 2 / 3 stages), kernel bench, numerics
# tests, and the batched decode step.
set -o pipefail
mkdir -p gpurun_out/ch
R=gpurun_out/ch/gemm.log
echo "default" >> $R; timeout -k 10 200 python -u scripts/bench_gemm.py 32 64 2>&1 | grep -v amdgpu >> $R || exit 1
for stg in 2 3; do
  echo "CH=4 STG=$stg" >> $R
  DL_GEMM_CH4=4 DL_GEMM_CH2=4 DL_GEMM_STG4=$stg DL_GEMM_STG2=$stg timeout -k 10 200 python -u scripts/bench_gemm.py 32 64 2>&1 | grep -v amdgpu >> $R || exit 1
done
DL_GEMM_CH4=4 DL_GEMM_CH2=4 DL_GEMM_STG4=2 DL_GEMM_STG2=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k gemm > gpurun_out/ch/tests.log 2>&1 || exit 1
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0 --tp-rank-compute= --steps 32 --warmup 8"
for b in 32 64; do
  timeout -k 10 300 python -u bench.py --batch $b $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default batch $b', d['ms_per_step'])" >> $R || exit 1
  DL_GEMM_CH4=4 DL_GEMM_CH2=4 DL_GEMM_STG4=2 DL_GEMM_STG2=2 timeout -k 10 300 python -u bench.py --batch $b $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ch4 stg2 batch $b', d['ms_per_step'])" >> $R || exit 1
done
