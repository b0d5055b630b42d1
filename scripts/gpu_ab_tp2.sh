# Same-box A/B of the same-GPU TP2 rehearsal (8B, f32 and q80 sync): the current tree vs a side
# build of an older commit in old_build/ (a git worktree built in-tree; not tracked).
set -o pipefail
mkdir -p gpurun_out/abtp
export DL_BENCH_SAME_GPU=1 HSA_ENABLE_IPC_MODE_LEGACY=0
F="--steps 32 --warmup 8 --no-prefill4k --no-cap128k --no-f32kv --long-ctx 0 --no-cli"
pj() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$1', c['pred_ms_per_token'], c.get('tp_f32_pred_ms_per_token'), c['eval_ms_per_token'])"; }
port=29560
for i in 1; do
  port=$((port+1)); (cd old_build && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 $F 2>&1 | tail -n 1 | pj old) >> gpurun_out/abtp/runs.log || exit 1
  port=$((port+1)); timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 $F --tp-rank-compute= 2>&1 | tail -n 1 | pj new >> gpurun_out/abtp/runs.log || exit 1
done
