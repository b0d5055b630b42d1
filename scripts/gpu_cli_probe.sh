#!/bin/bash
# CLI product-path probe: per-forward wall times of `dllama inference --synthetic` (bench's cli point)
# under first-use variants (deferred code-object loading on / off, graphs off)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-cli_probe}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
python3 -c "import sys; sys.path.insert(0, '$R'); from distributed_llama_multiusers_amd.models.synthetic import make_tokenizer; make_tokenizer('/tmp/t.t', 128256)" || exit $?
P=$(python3 -c "print(('The quick brown fox jumps over the lazy dog ' * 8)[:64])")
run() {  # name, extra args...
  local n=$1; shift
  timeout -k 10 180 $R/build/dllama inference --synthetic llama3_1_8b --tokenizer /tmp/t.t --prompt "$P" --steps 84 \
    --temperature 0 --gpu-index 0 --max-seq-len 92 --buffer-float-type q80 --log-level 0 --metrics $O/metrics_$n.jsonl "$@" > $O/cli_$n.log 2>&1
}
run base || exit $?
HIP_ENABLE_DEFERRED_LOADING=0 run eager_load || exit $?
run nograph --graph 0 || exit $?
exit 0
