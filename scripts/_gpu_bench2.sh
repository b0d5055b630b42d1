set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DL_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_ops.py > gpurun_out/r2_engine_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 > gpurun_out/r2_bench_n1.log 2>&1 && \
for st in q80 f32; do
  DL_BENCH_SAME_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 64 --warmup 8 --sync-type $st > gpurun_out/r2_tp2_$st.log 2>&1 || exit 1
done
