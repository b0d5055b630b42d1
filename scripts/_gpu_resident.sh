#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for r in 512 256 320 1024 512; do
  DL_GEMV_RESIDENT=$r timeout -k 10 200 python -u bench.py --steps 64 --warmup 8 --no-cli --no-f32kv > gpurun_out/res_$r.log 2>&1 || { tail -5 gpurun_out/res_$r.log; exit 1; }
  echo "resident $r: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/res_$r.log').read().strip().splitlines()[-1]); print(d['config']['pred_ms_per_token'], d['config']['eval_ms_per_token'], d['config']['long_ctx_pred_ms_per_token'])")"
done
