#!/bin/bash
# Split-K knob sweep of the narrow batched GEMM on the bench's eval (32-row chunks) and batch-8 decode
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gemm_knobs}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 -u $R/bench.py --steps 16 --warmup 4 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k"
for cfg in "base" "DL_GEMM_WG=128" "DL_GEMM_WG=512" "DL_GEMM_WG=1024" "DL_GEMM_MAXS=16" "DL_GEMM_MAXS=2" "DL_GEMM_STG2=3"; do
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  env $e timeout -k 10 240 $B > $O/$cfg.log 2>&1 || exit $?
  env $e timeout -k 10 240 $B --batch 8 > $O/$cfg.b8.log 2>&1 || exit $?
  echo "$cfg $(grep -o '"eval_ms_per_token": [0-9.]*' $O/$cfg.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$cfg.b8.log)"
done
exit 0
