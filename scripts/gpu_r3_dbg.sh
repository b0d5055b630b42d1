#!/bin/bash
# Round-3 iteration: attention tests, VALU vs MFMA decode-attention microbench, long-context bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3dbg3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py $R/tests/test_gpu_engine.py -q --timeout 120 --timeout-method thread -k "attention or long_context or decode or greedy or paged" > $O/tests.log 2>&1
for m in 0 1; do
  DL_ATTN_MFMA=$m timeout -k 10 200 python -u $R/scripts/bench_attn.py > $O/attn_mfma$m.log 2>&1 || exit $?
done
timeout -k 10 300 python -u $R/bench.py --steps 64 --warmup 8 --no-cli --no-f32kv --no-prefill4k > $O/bench.log 2>&1 || exit $?
exit 0
