# Decode attention: the VALU kernel vs the MFMA kernel (DL_ATTN_MFMA=0/1) by batch and position.
set -o pipefail
mkdir -p gpurun_out/attn
for m in 0 1; do
  echo "DL_ATTN_MFMA=$m" >> gpurun_out/attn/mfma.log
  DL_ATTN_MFMA=$m BATCHES=1,4,8,16,64 TPS=1 SHORT=1 timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -v amdgpu >> gpurun_out/attn/mfma.log || exit 1
done
