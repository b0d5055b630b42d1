# Decode attention vs the minimum keys per split (DL_ATTN_CHUNK), batch 1 / 4, and the long-context
# decode point of bench.py.
set -o pipefail
mkdir -p gpurun_out/attn
for c in 256 128 64; do
  echo "chunk $c" >> gpurun_out/attn/chunk.log
  DL_ATTN_CHUNK=$c BATCHES=1,4 TPS=1,8 timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -v amdgpu >> gpurun_out/attn/chunk.log || exit 1
done
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --tp-rank-compute= --steps 32 --warmup 8"
for c in 256 128; do
  DL_ATTN_CHUNK=$c timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk $c pred', d['config']['pred_ms_per_token'], 'long', d['config']['long_ctx_pred_ms_per_token'])" >> gpurun_out/attn/chunk.log || exit 1
done
