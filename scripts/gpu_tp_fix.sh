# Same-GPU TP rehearsals after the attention-block rule change, and the TP tests.
set -o pipefail
mkdir -p gpurun_out/tpfix
bash scripts/gpu_tp_rehearse.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_xgmi.py > gpurun_out/tpfix/xgmi.log 2>&1
