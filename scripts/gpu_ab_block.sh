# Same-box A/B of the TP1 headline decode with and without the fused attention block.
set -o pipefail
mkdir -p gpurun_out/abblk
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --tp-rank-compute="
for i in 1 2; do
  for b in default 0; do
    if [ $b = 0 ]; then export DL_ATTN_BLOCK=0; else unset DL_ATTN_BLOCK; fi
    timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('block=$b', c['pred_ms_per_token'], 'long', c['long_ctx_pred_ms_per_token'])" >> gpurun_out/abblk/runs.log || exit 1
  done
done
