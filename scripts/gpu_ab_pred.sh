# Same box: headline decode through bench.py vs the TP-rank script at TP1, argmax tail on / off.
set -o pipefail
mkdir -p gpurun_out/ab
R=gpurun_out/ab/pred.log
F="--no-cli --no-cap128k --no-prefill4k --no-f32kv --long-ctx 0 --tp-rank-compute="
timeout -k 10 200 python -u bench.py $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench default', d['config']['pred_ms_per_token'], d['config']['eval_ms_per_token'])" >> $R || exit 1
DL_ARGMAX_TAIL=0 timeout -k 10 200 python -u bench.py $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench tail off', d['config']['pred_ms_per_token'])" >> $R || exit 1
timeout -k 10 120 python -u scripts/tp_rank_compute.py --tp 1 --steps 128 2>&1 | grep -v "^ℹ\|amdgpu" >> $R || exit 1
DL_ARGMAX_TAIL=0 timeout -k 10 120 python -u scripts/tp_rank_compute.py --tp 1 --steps 128 2>&1 | grep -v "^ℹ\|amdgpu" >> $R || exit 1
timeout -k 10 200 python -u bench.py $F 2>&1 | tail -n 1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench again', d['config']['pred_ms_per_token'])" >> $R || exit 1
