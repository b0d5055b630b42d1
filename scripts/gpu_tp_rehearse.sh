#!/bin/bash
# Same-GPU rehearsals of the multi-rank bench (every phase, 1B shape): --gpus 4 and --gpus 8 with all
# ranks on one MI355X. usage: scripts/gpu_tp_rehearse.sh <out-name>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tpr}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
for n in 4 8; do
  DL_BENCH_SAME_GPU=1 timeout -k 10 400 python3 -u $R/bench.py --gpus $n --shape llama3_2_1b --steps 16 --warmup 4 > $O/bench_tp$n.log 2>&1 || exit $?
  grep "self-test\|timed out" $O/bench_tp$n.log; tail -1 $O/bench_tp$n.log
done
exit 0
