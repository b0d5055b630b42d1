#!/bin/bash
# Same-box A/B: head-major KV (repo) vs interleaved KV (build/ab_old worktree), decode points.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-abkv}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
B="--steps 32 --warmup 4 --no-cli --no-f32kv --no-prefill4k"
for i in 1 2; do
  timeout -k 10 400 python3 $R/bench.py $B > $O/new$i.log 2>&1 || exit $?
  timeout -k 10 400 python3 $R/build/ab_old/bench.py $B > $O/old$i.log 2>&1 || exit $?
done
exit 0
