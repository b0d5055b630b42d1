# Per-kernel profiles of batch-1 decode: TP1 and a TP8 rank (exchange in loopback).
set -o pipefail
mkdir -p gpurun_out/pd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pd/tp1 -o p -- python3 scripts/tp_rank_compute.py --tp 1 --steps 64 > gpurun_out/pd/tp1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pd/tp8 -o p -- python3 scripts/tp_rank_compute.py --tp 8 --steps 64 > gpurun_out/pd/tp8.log 2>&1
