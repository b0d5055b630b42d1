# Same-box A/B of the headline decode across builds with different early ring slots (DL_GEMV_KE:
# the tree's default 2, side builds ke1/ and ke4/: git worktrees built in-tree, not tracked).
set -o pipefail
mkdir -p gpurun_out/abke
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --tp-rank-compute=8"
pj() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$1', c['pred_ms_per_token'], 'long', c['long_ctx_pred_ms_per_token'], 'tp8', c.get('tp8_rank_compute_ms_per_token'))"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ke2 >> gpurun_out/abke/runs2.log || exit 1
  (cd ke6 && timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ke6) >> gpurun_out/abke/runs2.log || exit 1
  (cd ke8 && timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ke8) >> gpurun_out/abke/runs2.log || exit 1
  (cd ke4 && timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ke4) >> gpurun_out/abke/runs2.log || exit 1
done
