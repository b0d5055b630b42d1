# Same-box A/B of the headline decode: the current tree vs a side build of an older commit
# (old_build/, a git worktree built in-tree; not tracked).
set -o pipefail
mkdir -p gpurun_out/ab
R=gpurun_out/ab/old_new.log
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0"
pj() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['config']['pred_ms_per_token'], d['config']['eval_ms_per_token'])"; }
for i in 1 2; do
  (cd old_build && timeout -k 10 200 python -u bench.py $F 2>&1 | tail -n 1 | pj old) >> $R || exit 1
  timeout -k 10 200 python -u bench.py $F --tp-rank-compute= 2>&1 | tail -n 1 | pj new >> $R || exit 1
done
