# Same-GPU TP2 bench (8B, pred only) under the engine's A/B switches.
set -o pipefail
mkdir -p gpurun_out/tpb
export DL_BENCH_SAME_GPU=1 HSA_ENABLE_IPC_MODE_LEGACY=0
F="--steps 32 --warmup 8 --no-prefill4k --no-cap128k --no-f32kv --long-ctx 0 --tp-rank-compute= --no-cli"
port=29570
for envs in ${ENVS:-X=1 DL_SYNC_COPY=0}; do
  port=$((port+1))
  env $envs timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 2 $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$envs', c['pred_ms_per_token'], c.get('tp_f32_pred_ms_per_token'), c['eval_ms_per_token'], c['tp_fused_exchange'])" >> gpurun_out/tpb/runs2.log || exit 1
done
