#!/bin/bash
# Start/stop N local `dllama worker` processes (one per GPU, --gpu-index 1..N) for testing TP.
#
#   W=7 bash examples/n-workers.sh start     # workers on ports 9997, 9996, ... and GPUs 1..7
#   W=7 bash examples/n-workers.sh stop
#   CPU=1 T=4 W=3 bash examples/n-workers.sh start   # CPU workers with 4 threads each
#
# Then run the root on GPU 0, e.g.
#   build/dllama inference --model m.m --tokenizer t.t --buffer-float-type q80 --gpu-index 0 \
#       --steps 64 --prompt "Hello" --workers 127.0.0.1:9997 127.0.0.1:9996 ...
# PIDs are kept in examples/dllama_worker_<w>/pid; `stop` kills exactly those processes.
set -u
cd "$(dirname "$0")"
W=${W:-3}
T=${T:-1}
CPU=${CPU:-0}
export HSA_ENABLE_IPC_MODE_LEGACY=0

case "${1:-}" in
start)
    for ((w = 1; w <= W; w++)); do
        port=$((9998 - w))
        dir=dllama_worker_$w
        mkdir -p "$dir"
        if [ -f "$dir/pid" ] && kill -0 "$(cat "$dir/pid")" 2>/dev/null; then
            echo "worker $w already running (pid $(cat "$dir/pid"))"
            continue
        fi
        if [ "$CPU" = "1" ]; then dev="--nthreads $T"; else dev="--gpu-index $w"; fi
        nohup ../build/dllama worker --port "$port" $dev > "$dir/log.txt" 2>&1 &
        echo $! > "$dir/pid"
        echo "Started worker $w on port $port (pid $!)"
    done
    sleep 2
    ;;
stop)
    for ((w = 1; w <= W; w++)); do
        dir=dllama_worker_$w
        [ -f "$dir/pid" ] || continue
        kill "$(cat "$dir/pid")" 2>/dev/null && echo "Stopped worker $w"
        rm -f "$dir/pid"
    done
    ;;
*)
    echo "Usage: W=<n> $0 {start|stop}"
    exit 1
    ;;
esac
