#!/bin/bash
# Round-3 iteration: tr16 probe, MFMA decode attention (both V-read forms), paged KV, FFN block
# modes, then decode A/B of the FFN block modes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3dbg}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/build/probe_tr16 > $O/probe.log 2>&1 || exit $?
DL_ATTN_TR=0 timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "attention" > $O/tests_tr0.log 2>&1
timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread -k "attention" > $O/tests_tr1.log 2>&1
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_engine.py -q --timeout 120 --timeout-method thread -k "paged or ffn_block or wide" > $O/tests_eng.log 2>&1
for m in 0 2; do
  DL_FFN_BLOCK=$m timeout -k 10 200 python $R/bench.py --steps 64 --warmup 8 --no-cli --long-ctx 0 --no-f32kv --no-prefill4k > $O/bench_ffn$m.log 2>&1 || exit $?
done
exit 0
