#!/bin/bash
# Long-generation determinism check (the reference's examples/macbeth.sh compares one fixed
# output string captured on one machine). Here the same seeded generation is run at TP=1 and
# TP=$N on local GPUs and the generated text must match token for token.
#
#   MODEL=m.m TOKENIZER=t.t N=2 STEPS=512 bash examples/determinism.sh
set -eu
cd "$(dirname "$0")/.."
N=${N:-2}
STEPS=${STEPS:-512}
PROMPT=${PROMPT:-"Duncan. What bloody man is that? He can report, As seemeth by his plight, of the revolt The newest state."}
run() {
    build/dllama inference --model "$MODEL" --tokenizer "$TOKENIZER" --buffer-float-type q80 --gpu-index 0 \
        --seed 12345 --temperature 0.9 --topp 0.9 --steps "$STEPS" --prompt "$PROMPT" --log-level 0 "$@"
}
A=$(run)
W=$((N - 1)) bash examples/n-workers.sh start > /dev/null
trap 'W=$((N - 1)) bash examples/n-workers.sh stop > /dev/null' EXIT
WORKERS=()
for ((w = 1; w < N; w++)); do WORKERS+=("127.0.0.1:$((9998 - w))"); done
B=$(run --workers "${WORKERS[@]}")
if [ "$A" == "$B" ]; then echo "✅ Output is same (TP1 vs TP$N, $STEPS steps)"; else echo "❌ Output is different"; exit 1; fi
