#!/bin/bash
# 16-block-chunk narrow GEMM: batched-path tests, bench_gemm at 8/16/32 tokens, bench.py batch 8/16.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-g16}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_engine.py $R/tests/test_gpu_ops.py -k "8b_shape or prefill_mfma or gemm or wide" -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
case $rc in 0|1|5) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 300 python -u $R/scripts/bench_gemm.py 8 16 32 > $O/gemm.log 2>&1 || exit $?
for b in 8 16 32 64; do
  timeout -k 10 240 python3 $R/bench.py --batch $b --steps 16 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k --no-cap128k > $O/b$b.log 2>&1 || exit $?
done
exit 0
