set -o pipefail
mkdir -p gpurun_out/tpr3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=gpurun_out/tpr3/runs.log
run() { timeout -k 10 120 env "$@" >> $R 2>&1 || exit 1; }
run python -u scripts/tp_rank_compute.py --tp 1
run DL_ARGMAX_TAIL=0 python -u scripts/tp_rank_compute.py --tp 1
run DL_ATTN_BLOCK=0 python -u scripts/tp_rank_compute.py --tp 8
run DL_ATTN_BLOCK=0 DL_SYNC_MEASURE=0 python -u scripts/tp_rank_compute.py --tp 8
run DL_ATTN_BLOCK=0 DL_ARGMAX_TAIL=0 python -u scripts/tp_rank_compute.py --tp 8
run DL_ATTN_BLOCK=0 DL_SYNC_MEASURE=0 DL_ARGMAX_TAIL=0 python -u scripts/tp_rank_compute.py --tp 8
export DL_ATTN_BLOCK=0 DL_SYNC_MEASURE=0
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tpr3/prof8 -o p -- python3 scripts/tp_rank_compute.py --tp 8 --steps 32 > gpurun_out/tpr3/prof8.log 2>&1
