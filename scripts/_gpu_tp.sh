# TP fused-exchange validation on one GPU (same-GPU multi-process rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DL_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_xgmi.py > gpurun_out/r2_tp_tests.log 2>&1 && \
for f in 1 0; do
  DL_TP_FUSED=$f DL_BENCH_SAME_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 64 --warmup 8 > gpurun_out/r2_tp2_fused$f.log 2>&1 || exit 1
done
