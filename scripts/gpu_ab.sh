# Same-box A/B of bench.py between this tree and side builds (scripts/ab_build.sh -> ab/<name>),
# alternating runs.  usage: bash scripts/gpu_ab.sh "<bench flags>" <rounds> name1 [name2 ...]
# ("." = this tree). One line per run in gpurun_out/ab/runs.log: pred (f32 KV), bf16-KV pred,
# long-context pred, tp8 rank compute, eval.
set -o pipefail
mkdir -p gpurun_out/ab
F=$1; N=$2; shift 2
pj() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=d['config']; print('$1', 'pred', c['pred_ms_per_token'], 'bf16', c.get('bf16_kv_pred_ms_per_token'), 'long', c.get('long_ctx_pred_ms_per_token'), 'tp8', c.get('tp8_rank_compute_ms_per_token'), 'eval', c['eval_ms_per_token'], 'value', d['value'])"; }
for i in $(seq 1 $N); do
  for name in "$@"; do
    d=$GRAFT_REPO_ROOT; [ "$name" != "." ] && d=$GRAFT_REPO_ROOT/ab/$name
    (cd $d && timeout -k 10 300 python3 -u bench.py $F 2> $GRAFT_REPO_ROOT/gpurun_out/ab/$name.err | pj $name) >> gpurun_out/ab/runs.log || exit 1
  done
done
cat gpurun_out/ab/runs.log
