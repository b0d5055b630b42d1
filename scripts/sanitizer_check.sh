#!/bin/bash
# Host sanitizer runs: builds the native code with AddressSanitizer+UBSan and with
# ThreadSanitizer in scratch copies of the tree, then drives the multi-threaded / multi-process
# host paths on the CPU backend under each:
#   * tensor parallelism over the TCP control + data plane (root + 1 worker, 16 decode steps)
#   * dllama-api with 4 concurrent requests batched by the scheduler (thread per connection)
# Any sanitizer report fails the run. Device code is not sanitized (no GPU ASan on this pool).
#   bash scripts/sanitizer_check.sh [outdir]
set -u
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/dl_sanitize}
mkdir -p "$OUT"
python3 -c "
import sys; sys.path.insert(0, '$REPO')
from distributed_llama_multiusers_amd.models.synthetic import make_test_assets
from distributed_llama_multiusers_amd.utils.mfile import FloatType
make_test_assets('$OUT/assets', 'tiny', FloatType.Q40, seq_len=128, seed=7, dim=512, n_heads=8, n_kv_heads=4, hidden_dim=1024)
"
M=$OUT/assets/tiny_q40.m
T=$OUT/assets/tiny.t
status=0
for kind in asan tsan; do
    dir=$OUT/$kind
    rm -rf "$dir" && mkdir -p "$dir"
    (cd "$REPO" && git archive HEAD) | tar -x -C "$dir"
    flag=$([ $kind = asan ] && echo DEBUG=1 || echo TSAN=1)
    (cd "$dir" && make -j8 $flag all > build.log 2>&1) || { echo "$kind: build failed"; status=1; continue; }
    export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1 TSAN_OPTIONS=halt_on_error=0
    log=$dir/run.log
    : > "$log"
    port=$((20000 + RANDOM % 20000))
    "$dir/build/dllama" worker --port $port --nthreads 2 >> "$log" 2>&1 &
    wpid=$!
    sleep 1
    "$dir/build/dllama" inference --model $M --tokenizer $T --buffer-float-type q80 --nthreads 2 \
        --prompt "hello world the" --steps 16 --temperature 0 --workers 127.0.0.1:$port >> "$log" 2>&1
    kill $wpid 2>/dev/null
    wait $wpid 2>/dev/null
    aport=$((20000 + RANDOM % 20000))
    "$dir/build/dllama-api" --model $M --tokenizer $T --buffer-float-type q80 --nthreads 2 --port $aport \
        --slots 4 --temperature 0 >> "$log" 2>&1 &
    apid=$!
    for i in $(seq 50); do curl -s -o /dev/null http://127.0.0.1:$aport/health && break; sleep 0.2; done
    cpids=()
    for i in 1 2 3 4; do
        body="{\"messages\":[{\"role\":\"user\",\"content\":\"request $i\"}],\"max_tokens\":8}"
        curl -s -X POST http://127.0.0.1:$aport/v1/chat/completions -H 'Content-Type: application/json' \
            -d "$body" > /dev/null &
        cpids+=($!)
    done
    wait "${cpids[@]}"
    curl -s -o /dev/null http://127.0.0.1:$aport/v1/metrics
    kill $apid 2>/dev/null
    wait $apid 2>/dev/null
    n=$(grep -c -E "ERROR: AddressSanitizer|runtime error:|WARNING: ThreadSanitizer" "$log")
    echo "$kind: $n sanitizer reports ($(grep -c 'Prediction' "$log") inference summary, log $log)"
    [ "$n" = 0 ] || status=1
done
exit $status
