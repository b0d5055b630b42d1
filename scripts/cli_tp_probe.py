"""The product path's tensor-parallel per-token overhead: `dllama inference
--synthetic llama3_1_8b` with a root and `--workers` (one worker process per extra rank, all on
GPU 0 here: a same-GPU rehearsal, not a scaling point) against the same engine without workers,
both with greedy decode chained on the device (Cmd::CHAIN: the root sends one TCP control packet
per token, workers launch on receipt). Prints one JSON line: eval / pred ms per token at TP1 and
TP-N through the CLI; compare with `bench.py --gpus N` (DL_BENCH_SAME_GPU=1), which drives the
same engines without the TCP control plane.

    python scripts/cli_tp_probe.py --tp 2
"""
import argparse
import json
import os
import re
import socket
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(base, workers, env):
    procs, addrs = [], []
    try:
        for _ in range(workers):
            p = port()
            procs.append(subprocess.Popen([os.path.join(REPO, "build", "dllama"), "worker", "--port", str(p),
                                           "--gpu-index", "0"], stdout=subprocess.DEVNULL, stderr=subprocess.STDOUT,
                                          env=env))
            addrs.append(f"127.0.0.1:{p}")
        time.sleep(1.0)
        cmd = base + (["--workers", *addrs] if addrs else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    finally:
        for p in procs:
            p.kill()
            p.wait()
    m = re.findall(r"tokens/s:\s*([\d.]+)\s*\(([\d.]+) ms/tok\)", r.stdout)
    if r.returncode != 0 or len(m) < 2:
        raise SystemExit(f"dllama failed ({r.returncode}): {(r.stdout + r.stderr)[-1500:]}")
    return float(m[0][1]), float(m[1][1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--prompt", type=int, default=64)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--kv", default="f32")
    a = ap.parse_args()
    from distributed_llama_multiusers_amd.models.synthetic import make_tokenizer
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", DL_TP_COMM=os.environ.get("DL_TP_COMM", "xgmi"))
    with tempfile.TemporaryDirectory() as d:
        tok = os.path.join(d, "t.t")
        make_tokenizer(tok, 128256)
        prompt = ("The quick brown fox jumps over the lazy dog " * 8)[:a.prompt]
        base = [os.path.join(REPO, "build", "dllama"), "inference", "--synthetic", "llama3_1_8b", "--tokenizer", tok,
                "--prompt", prompt, "--steps", str(a.prompt + a.steps), "--temperature", "0", "--gpu-index", "0",
                "--max-seq-len", "4096", "--buffer-float-type", "q80", "--kv-dtype", a.kv, "--log-level", "0"]
        e1, p1 = run(base, 0, env)
        en, pn = run(base, a.tp - 1, env)
    print(json.dumps({"cli_tp1_eval_ms": e1, "cli_tp1_pred_ms": p1, f"cli_tp{a.tp}_eval_ms": en,
                      f"cli_tp{a.tp}_pred_ms": pn, "same_gpu_rehearsal": True, "kv": a.kv}), flush=True)


if __name__ == "__main__":
    main()
