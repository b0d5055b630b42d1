# Round check: the whole GPU test suite (one process), smoke(), the headline bench.
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread > gpurun_out/full/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u __graft_entry__.py > gpurun_out/full/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/full/bench.log 2>&1
