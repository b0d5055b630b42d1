# PMC of the TP8 wo / w2 GEMV with and without the TP tail (loopback exchange): instruction
# fetch misses vs waits. One pass per counter set, one kernel per process.
set -o pipefail
mkdir -p gpurun_out/pmc_tail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "4096 512 0 0 wo8" "4096 512 0 5 wo8tp" "4096 1792 1 0 w2_8" "4096 1792 1 5 w2_8tp"; do
  set -- $spec
  for pass in "SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 60 rocprofv3 --pmc $pass -d gpurun_out/pmc_tail/$5_$tag -o p --output-format csv -- \
      python3 -c "import sys; sys.path.insert(0,'.'); import distributed_llama_multiusers_amd as dl; print(dl.native().bench_gemv_q40($1,$2,$3,$4,1,0,0,48,100))" \
      > gpurun_out/pmc_tail/$5_$tag.log 2>&1 || echo "pass $5 $tag failed" >> gpurun_out/pmc_tail/errors.log
  done
done
exit 0
