#!/bin/bash
# One wrapper for the GPU-box runs (gpurun -- 'bash scripts/gpu.sh <task> ...'); every step has its
# own time limit and the first failing step ends the run. Outputs under gpurun_out/<task>/.
#
#   tests [pytest args]          GPU test suite (default: all of -m gpu) in one process, then smoke()
#   bench [bench.py args]        the headline bench (default flags: the driver's)
#   ab "<bench flags>" N a b ..  same-box A/B of bench.py: this tree (".") vs side builds ab/<name>
#                                (scripts/ab_build.sh), N alternating rounds -> gpurun_out/ab/runs.log
#   env "<bench flags>" N "A=1 B=2" "A=0" ..   bench.py under each set of environment switches
#   prof-decode [tp list] [kv] [pos]  rocprofv3 kernel trace of batch-1 decode (TP1 / a TP-N rank in
#                                loopback, scripts/tp_rank_compute.py) + per-kernel tables
#   batch [B list]               batched decode steps (bench.py --batch B)
#   big                          70B-shaped decode on one GPU + dllama-api throughput (64 / 16 requests)
#   tp-rehearse                  same-GPU multi-rank bench rehearsals (TP2 8B, TP4 1B; not scaling points)
#                                + the CLI root/worker TP2 product path (scripts/cli_tp_probe.py)
#   pmc <name> "<counters>" <cmd..>   one rocprofv3 PMC pass (counters only) over a command
set -o pipefail
task=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/$task
mkdir -p "$O"
# one bench JSON line -> the points an A/B compares
pj() {
  python3 -c "import json,sys
d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]); c=d['config']
print('$1', 'value', d['value'], 'pred', c['pred_ms_per_token'], 'eval', c['eval_ms_per_token'], 'bf16kv_pred',
      c.get('bf16_kv_pred_ms_per_token'), 'long', c.get('long_ctx_pred_ms_per_token'), 'tp2', c.get('tp2_rank_compute_ms_per_token'),
      'tp4', c.get('tp4_rank_compute_ms_per_token'), 'tp8', c.get('tp8_rank_compute_ms_per_token'),
      'p4k', c.get('prompt_4k_eval_ms_per_token'), 'p4k_big', c.get('prompt_4k_eval_big_chunk_ms_per_token'))"
}
QUICK="--no-cli --no-cap128k --no-prefill4k --steps 64 --warmup 8"
case $task in
  tests)
    [ $# -eq 0 ] && set -- tests -m gpu
    timeout -k 10 1500 python3 -u -m pytest "$@" -v --timeout 170 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
    tail -3 $O/tests.log
    timeout -k 10 180 python3 -u __graft_entry__.py > $O/smoke.log 2>&1 || exit 1
    tail -n 2 $O/smoke.log ;;
  bench)
    timeout -k 10 600 python3 -u bench.py "$@" > $O/bench.json 2> $O/bench.err || exit 1
    cat $O/bench.json ;;
  ab)
    F=$1; N=$2; shift 2
    for i in $(seq 1 $N); do
      for name in "$@"; do
        d=$R; [ "$name" != "." ] && d=$R/ab/$name
        (cd $d && timeout -k 10 400 python3 -u bench.py $F 2> $R/$O/$name.err | pj $name) >> $O/runs.log || exit 1
      done
    done
    cat $O/runs.log ;;
  env)
    F=$1; N=$2; shift 2
    for i in $(seq 1 $N); do
      for envs in "$@"; do
        env $envs timeout -k 10 400 python3 -u bench.py $F 2>> $O/err.log | pj "[$envs]" >> $O/runs.log || exit 1
      done
    done
    cat $O/runs.log ;;
  prof-decode)
    kv=${2:-f32}; pos=${3:-64}
    for tp in ${1:-1 8}; do
      n=tp${tp}_${kv}_p$pos
      timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$n -o p -- python3 scripts/tp_rank_compute.py --tp $tp --steps 64 --kv $kv --pos $pos > $O/$n.log 2>&1 || exit 1
      python3 scripts/prof_summary.py $O/$n --skip-first 3000 > $O/$n.md 2>&1
      grep "pred" $O/$n.log
    done ;;
  batch)
    for b in ${1:-8 16 64}; do
      timeout -k 10 300 python3 -u bench.py --batch $b $QUICK --long-ctx 0 --tp-rank-compute= --no-altkv 2>> $O/err.log | \
        python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print('batch $b', d['ms_per_step'], 'ms/step', d['config']['pred_tokens_per_s'], 'tok/s')" >> $O/bench.log || exit 1
    done
    cat $O/bench.log ;;
  big)
    timeout -k 10 500 python3 -u bench.py --shape llama3_3_70b $QUICK --long-ctx 0 --tp-rank-compute= --no-altkv > $O/b70.json 2> $O/b70.err || exit 1
    timeout -k 10 400 python3 -u scripts/bench_api.py --n 64 > $O/api64.log 2>&1 || exit 1
    timeout -k 10 300 python3 -u scripts/bench_api.py --n 16 > $O/api16.log 2>&1 || exit 1
    tail -n 1 $O/b70.json; tail -n 2 $O/api64.log $O/api16.log ;;
  tp-rehearse)
    export DL_BENCH_SAME_GPU=1
    F="--steps 32 --warmup 8 --no-prefill4k --no-cap128k --no-altkv --long-ctx 0"
    timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
      bench.py --gpus 2 $F > $O/tp2.log 2>&1 || exit 1
    timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 \
      bench.py --gpus 4 --shape llama3_2_1b $F > $O/tp4_1b.log 2>&1 || exit 1
    timeout -k 10 600 python3 -u scripts/cli_tp_probe.py --tp 2 > $O/cli_tp2.json 2> $O/cli_tp2.err || exit 1
    tail -n 1 $O/tp2.log $O/tp4_1b.log $O/cli_tp2.json ;;
  pmc)
    name=$1; counters=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $O/$name -- "$@" > $O/$name.log 2>&1 || exit 1
    python3 scripts/pmc_summary.py $O/$name > $O/$name.md 2>&1 ;;
  *)
    sed -n 2,17p "$0"; exit 2 ;;
esac
