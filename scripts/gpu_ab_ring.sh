# Same-box A/B of the headline decode across GEMV ring depths (DL_GEMV_RING: the tree's 8, side
# builds ring3/ and ring12/: git worktrees built in-tree, not tracked).
set -o pipefail
mkdir -p gpurun_out/abring
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --tp-rank-compute=8"
pj() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$1', c['pred_ms_per_token'], 'long', c['long_ctx_pred_ms_per_token'], 'tp8', c.get('tp8_rank_compute_ms_per_token'))"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ring8 >> gpurun_out/abring/runs3.log || exit 1
  (cd ring3 && timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ring3) >> gpurun_out/abring/runs3.log || exit 1
  (cd ring4 && timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ring4) >> gpurun_out/abring/runs3.log || exit 1
  (cd ring2 && timeout -k 10 300 python -u bench.py $F 2>&1 | tail -n 1 | pj ring2) >> gpurun_out/abring/runs3.log || exit 1
done
