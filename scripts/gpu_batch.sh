#!/bin/bash
# Batched decode: GEMV chunk tests, then bench.py at batch 8 / 16 / 64 on the default path and with
# the MFMA GEMM forced (DL_GEMM_MIN=3). usage: scripts/gpu_batch.sh <out-name>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-batch}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
B="--steps 16 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k --no-cap128k"
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_engine.py -k "gemv_chunks or prefill_mfma" -x -q --timeout 180 --timeout-method thread > $O/t_batch.log 2>&1
rc=$?; tail -3 $O/t_batch.log
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
for b in 8 16 64; do
  timeout -k 10 240 python3 $R/bench.py $B --batch $b > $O/bench_b$b.log 2>&1 || exit $?
  DL_GEMM_MIN=3 timeout -k 10 240 python3 $R/bench.py $B --batch $b > $O/bench_b${b}_mfma.log 2>&1 || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -- python3 $R/bench.py $B --batch 8 > $O/prof_b8.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof_b8 > $O/prof_b8.md 2>&1
exit 0
