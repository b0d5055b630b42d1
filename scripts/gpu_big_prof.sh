#!/bin/bash
# 70B decode on one GPU: GEMV lanes x passes sweep on its shapes, then a per-kernel profile of the
# decode. usage: scripts/gpu_big_prof.sh <out-name>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-bigp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 400 python3 -u $R/scripts/sweep_gemv_big.py > $O/sweep.txt 2>&1 || exit $?
B="--no-cli --no-f32kv --no-prefill4k --no-cap128k --long-ctx 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof70 -- python3 $R/bench.py $B --shape llama3_3_70b --steps 16 --warmup 2 --prompt 32 > $O/prof70.log 2>&1 || exit $?
python3 $R/scripts/prof_summary.py $O/prof70 > $O/prof70.md 2>&1
exit 0
