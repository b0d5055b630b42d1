cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in "llama3_1_8b 0" "llama3_3_70b 8" "llama3_1_405b 4"; do
  set -- $m
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$1 -- python3 $R/scripts/profile_decode.py --model $1 --layers $2 > $R/gpurun_out/prof_$1.log 2>&1 || exit $?
  python3 $R/scripts/prof_summary.py $R/gpurun_out/prof_$1 --by-grid > $R/gpurun_out/sum_$1.md || exit $?
done
