#!/bin/bash
# One GPU session: tests then bench then profile; stops at the first crash/timeout (exit codes
# 124/134/137/139 or negative signals) so nothing else runs on a faulted GPU.
# usage: scripts/gpu_session.sh "<step cmd>" "<step cmd>" ...
export DL_SKIP_BUILD=1
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a gpurun_out/session.log
  bash -c "$cmd" >> gpurun_out/step$i.log 2>&1
  rc=$?
  echo "=== step $i exit $rc" | tee -a gpurun_out/session.log
  tail -5 gpurun_out/step$i.log
  case $rc in
    0|1|2|5) ;;   # ok / test failures / usage / no tests: keep going
    *) echo "stopping: step $i crashed or timed out (rc=$rc)"; exit $rc ;;
  esac
done
