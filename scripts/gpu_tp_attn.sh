#!/bin/bash
# TP fused-exchange self-test + xGMI tests, then the long-context attention timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tpattn}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export DL_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_xgmi.py -x -v --timeout 240 --timeout-method thread > $O/t_xgmi.log 2>&1
rc=$?; tail -3 $O/t_xgmi.log
case $rc in 0|1) ;; *) echo "xgmi tests rc=$rc: stopping"; exit $rc ;; esac
for args in "8000 8192 1 1" "8000 8192 4 1" "1500 2048 1 1" "8000 8192 1 8"; do
  timeout -k 10 120 python -u $R/scripts/trace_attention.py $args >> $O/trace_attn.log 2>&1 || exit $?
done
exit 0
