# Per-kernel split of batched decode steps (batch 64 and 8), rocprofv3 kernel trace.
set -o pipefail
mkdir -p gpurun_out/b64
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0 --tp-rank-compute= --prompt 32 --warmup 4 --steps 16"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b64/p64 -o p -- python3 bench.py --batch 64 $F > gpurun_out/b64/b64.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b64/p8 -o p -- python3 bench.py --batch 8 $F > gpurun_out/b64/b8.log 2>&1
