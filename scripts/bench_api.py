"""Serving throughput of `dllama-api` on one GPU: N concurrent chat requests, greedy vs sampled.

Starts build/dllama-api on random-init Llama-3.1-8B weights (--synthetic, a synthetic 128256-token
tokenizer), fires N concurrent /v1/chat/completions requests of max_tokens each (threads, one HTTP
connection per request), and reports the aggregate completion tokens/s for temperature 0 (greedy)
and temperature 0.8 / top_p 0.9 with per-request seeds (device sampling: only token ids come back
to the host). One untimed round first captures the graphs.

  python scripts/bench_api.py [--n 64] [--max-tokens 64] [--port 0]
"""
import argparse
import http.client
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _post(port, body, out, i):
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=300)
        c.request("POST", "/v1/chat/completions", json.dumps(body), {"Content-Type": "application/json"})
        r = c.getresponse()
        data = json.loads(r.read())
        out[i] = data["usage"]["completion_tokens"]
    except Exception as e:  # noqa: BLE001 - counted as a failed request
        out[i] = e


def _round(port, n, max_tokens, temperature, seed0):
    out = [None] * n
    th = []
    for i in range(n):
        body = {"messages": [{"role": "user", "content": f"hello world {i} the"}], "max_tokens": max_tokens,
                "temperature": temperature, "top_p": 0.9, "seed": seed0 + i}
        th.append(threading.Thread(target=_post, args=(port, body, out, i)))
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    bad = [o for o in out if not isinstance(o, int)]
    if bad:
        raise RuntimeError(f"{len(bad)} requests failed: {bad[:3]}")
    return sum(out), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--max-batch", type=int, default=0,
                    help="rows per forward (default 4 x --n: prompts prefill in big chunks, MALL-resident weights)")
    ap.add_argument("--kv-pages", type=int, default=0,
                    help="paged KV cache: pool pages per layer (0: contiguous slots x seq_len)")
    ap.add_argument("--kv-page-size", type=int, default=64)
    ap.add_argument("--kv-dtype", default="f32", choices=["f32", "bf16"], help="KV cache (f32: the reference's, the default)")
    args = ap.parse_args()
    from distributed_llama_multiusers_amd.models.synthetic import make_tokenizer
    tmp = tempfile.mkdtemp()
    tok = os.path.join(tmp, "tok.t")
    make_tokenizer(tok, 128256)
    port = args.port or _port()
    cmd = [os.path.join(REPO, "build", "dllama-api"), "--synthetic", "llama3_1_8b", "--tokenizer", tok,
           "--gpu-index", "0", "--port", str(port), "--slots", str(args.n), "--max-batch", str(args.max_batch or 4 * args.n),
           "--max-seq-len", str(64 + args.max_tokens + 32), "--buffer-float-type", "q80", "--kv-dtype", args.kv_dtype]
    if args.kv_pages:
        cmd += ["--kv-pages", str(args.kv_pages), "--kv-page-size", str(args.kv_page_size)]
    log = open(os.path.join(tmp, "api.log"), "w")
    srv = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT)
    try:
        for _ in range(600):
            try:
                c = http.client.HTTPConnection("127.0.0.1", port, timeout=2)
                c.request("GET", "/v1/models")
                if c.getresponse().status == 200:
                    break
            except OSError:
                pass
            if srv.poll() is not None:
                raise RuntimeError("dllama-api exited: " + open(log.name).read()[-2000:])
            time.sleep(0.2)
        _round(port, args.n, 8, 0.0, 0)      # untimed: graph capture for the batch sizes
        _round(port, args.n, 8, 0.8, 100)
        res = {}

        def health():
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
            c.request("GET", "/health")
            return json.loads(c.getresponse().read())

        for name, temp, seed in (("greedy", 0.0, 0), ("sampled", 0.8, 1000)):
            h0 = health()
            toks, dt = _round(port, args.n, args.max_tokens, temp, seed)
            h1 = health()
            d = {k: h1[k] - h0[k] for k in ("forwards", "rows", "prefill_rows", "decode_rows", "busy_ms") if k in h1}
            res[name] = {"completion_tokens": toks, "s": round(dt, 3), "tok_s": round(toks / dt, 1),
                         "forwards": d.get("forwards"), "rows": d.get("rows"), "prefill_rows": d.get("prefill_rows"),
                         "forward_ms": round(d.get("busy_ms", 0.0), 1),
                         "host_ms": round(dt * 1000 - d.get("busy_ms", 0.0), 1)}
            print(name, res[name], flush=True)
        res["sampled_vs_greedy"] = round(res["sampled"]["tok_s"] / res["greedy"]["tok_s"], 3)
        res["concurrent_requests"] = args.n
        res["kv_cache"] = args.kv_dtype
        res["max_batch"] = args.max_batch or 4 * args.n
        res["max_tokens"] = args.max_tokens
        print(json.dumps(res), flush=True)
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
        log.close()
        print(open(log.name).read()[-1500:])


if __name__ == "__main__":
    main()
