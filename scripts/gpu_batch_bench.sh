# Batched decode steps (bench.py --batch B), plus the engine / API GPU tests.
set -o pipefail
mkdir -p gpurun_out/batch
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0 --tp-rank-compute= --steps 32 --warmup 8"
for b in ${BATCHES:-8 16 64}; do
  timeout -k 10 300 python -u bench.py --batch $b $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch $b', d['ms_per_step'], 'ms/step', d['config']['pred_tokens_per_s'], 'tok/s')" >> gpurun_out/batch/bench.log || exit 1
done
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py > gpurun_out/batch/tests.log 2>&1
