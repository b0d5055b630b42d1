#!/bin/bash
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmc3
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q -k "gemm or batched or prefill" --timeout 120 --timeout-method thread > gpurun_out/swz_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/swz_tests.log; exit 1; }
tail -1 gpurun_out/swz_tests.log
timeout -k 10 200 python -u scripts/bench_gemm.py 8 32 64 > gpurun_out/bench_gemm_swz.log 2>&1 || { echo "bench failed"; exit 1; }
grep tp1 gpurun_out/bench_gemm_swz.log
for b in 8 64; do timeout -k 10 200 python -u bench.py --batch $b --steps 16 --warmup 4 --long-ctx 0 --no-cli --no-f32kv --no-prefill4k > gpurun_out/swz_b$b.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*\|"eval_ms_per_token": [0-9.]*' gpurun_out/swz_b$b.log | tr '\n' ' '; echo; done
cd /tmp && export TMPDIR=/tmp && export M=32
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -d $R/gpurun_out/pmc3/b -o run --output-format csv -- python3 $R/scripts/prof_gemm_one.py > $R/gpurun_out/pmc3/b.log 2>&1 && echo "pmc ok"
