#!/bin/bash
# Non-temporal LDS-DMA check: GEMM / attention tests, bench_gemm, bench_attn, batch bench, decode bench x2, profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-nt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_xgmi.py $R/tests/test_gpu_engine.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
timeout -k 10 300 python -u $R/scripts/bench_gemm.py 8 16 32 64 > $O/gemm.log 2>&1 || exit $?
timeout -k 10 300 python -u $R/scripts/bench_attn.py > $O/attn.log 2>&1 || exit $?
B="--steps 32 --warmup 4 --no-cli --no-f32kv --no-prefill4k --no-cap128k --long-ctx 0"
for b in 8 32 64; do timeout -k 10 240 python3 $R/bench.py $B --batch $b > $O/b$b.log 2>&1 || exit $?; done
timeout -k 10 300 python3 $R/bench.py $B > $O/d1.log 2>&1 || exit $?
timeout -k 10 300 python3 $R/bench.py $B > $O/d2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -- python3 $R/bench.py $B > $O/prof.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof > $O/prof.md 2>&1
exit 0
