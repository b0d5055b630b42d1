"""dllama-api end-to-end on the CPU backend: OpenAI + reference response shapes, SSE streaming,
/v1/models, and concurrent requests batched by the scheduler giving the same tokens as solo runs
(the reference's shared-KV multi-user loop could not)."""
import concurrent.futures
import json
import os
import socket
import subprocess
import time
import urllib.request

import pytest

from conftest import REPO

API = os.path.join(REPO, "build", "dllama-api")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def server(assets):
    port = _free_port()
    proc = subprocess.Popen([API, "--model", assets["q40"], "--tokenizer", assets["tok"], "--buffer-float-type", "q80",
                             "--port", str(port), "--nthreads", "2", "--slots", "4", "--temperature", "0",
                             "--max-seq-len", "128", "--web-ui", os.path.join(REPO, "web-ui")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{port}"
    for _ in range(200):
        try:
            urllib.request.urlopen(url + "/health", timeout=1).read()
            break
        except Exception:
            time.sleep(0.05)
    else:
        proc.kill()
        raise RuntimeError("server did not start: " + proc.stdout.read().decode(errors="replace"))
    yield url
    proc.kill()
    proc.wait()


def _post(url, body, timeout=60):
    req = urllib.request.Request(url + "/v1/chat/completions", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    return urllib.request.urlopen(req, timeout=timeout)


def _chat(url, content, max_tokens=12, **kw):
    body = {"messages": [{"role": "user", "content": content}], "max_tokens": max_tokens, "temperature": 0}
    body.update(kw)
    return json.loads(_post(url, body).read())


def test_models(server):
    d = json.loads(urllib.request.urlopen(server + "/v1/models").read())
    assert d["object"] == "list" and d["data"][0]["id"].endswith(".m")


def test_completion_shapes(server):
    d = _chat(server, "hello world")
    assert "generated_text" in d  # web-ui / reference shape
    assert d["object"] == "chat.completion"
    assert d["choices"][0]["message"]["content"] == d["generated_text"]
    assert d["usage"]["completion_tokens"] <= 12
    assert d["usage"]["total_tokens"] == d["usage"]["prompt_tokens"] + d["usage"]["completion_tokens"]
    assert d["choices"][0]["finish_reason"] in ("stop", "length")


def test_streaming_matches_blocking(server):
    full = _chat(server, "the world")["generated_text"]
    r = _post(server, {"messages": [{"role": "user", "content": "the world"}], "max_tokens": 12, "temperature": 0,
                       "stream": True})
    assert r.headers["Content-Type"].startswith("text/event-stream")
    text, done, reasons = "", False, []
    for raw in r.read().decode().split("\r\n\r\n"):
        if not raw.startswith("data: "):
            continue
        payload = raw[6:]
        if payload == "[DONE]":
            done = True
            continue
        ch = json.loads(payload)
        assert ch["object"] == "chat.completion.chunk"
        text += ch["choices"][0]["delta"].get("content", "")
        reasons.append(ch["choices"][0]["finish_reason"])
    assert done and text == full and reasons[-1] in ("stop", "length")


def test_concurrent_requests_match_solo(server):
    prompts = ["hello", "the world", "and the", "hello world the end"]
    solo = [_chat(server, p)["generated_text"] for p in prompts]
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        conc = list(ex.map(lambda p: _chat(server, p)["generated_text"], prompts * 2))
    assert conc == solo * 2
    h = json.loads(urllib.request.urlopen(server + "/health").read())
    assert h["completed"] >= 12 and h["decode_rows"] > 0 and h["prefill_rows"] > 0


def test_bad_request(server):
    with pytest.raises(urllib.error.HTTPError) as e:
        _post(server, {"nope": 1})
    assert e.value.code == 400


def test_web_ui_served(server):
    html = urllib.request.urlopen(server + "/", timeout=5).read().decode()
    assert "app.js" in html
    js = urllib.request.urlopen(server + "/app.js", timeout=5).read().decode()
    assert "generated_text" in js and "/chat/completions" in js


def test_launcher_writes_tp_script(tmp_path):
    import sys
    sys.path.insert(0, REPO)
    import launch
    assert launch.main(["llama3_1_8b_instruct_q40", "--gpus", "4", "--no-download", "--dir", str(tmp_path)]) == 0
    script = (tmp_path / "run_llama3_1_8b_instruct_q40_tp4.sh").read_text()
    assert script.count("build/dllama worker") == 3 and "--gpu-index 3" in script
    assert "--workers 127.0.0.1:9997 127.0.0.1:9996 127.0.0.1:9995" in script
    assert len(launch.MODELS["llama3_1_405b_instruct_q40"].urls) == 56


def test_prometheus_metrics(server):
    _chat(server, "metrics please", max_tokens=4)
    text = urllib.request.urlopen(server + "/v1/metrics").read().decode()
    vals = {}
    for line in text.splitlines():
        if line and not line.startswith("#"):
            name, v = line.split()
            vals[name] = float(v)
    assert vals["dllama_requests_completed_total"] >= 1
    assert vals["dllama_rows_total"] == vals["dllama_prefill_rows_total"] + vals["dllama_decode_rows_total"]
    assert vals["dllama_generated_tokens_total"] >= 1 and vals["dllama_kv_slots"] == 4
    assert "# TYPE dllama_forwards_total counter" in text


def test_stream_client_disconnect_frees_slot(server):
    """A streaming client that hangs up mid-generation: the handler's write fails, the request is
    cancelled and its KV slot returns to the pool instead of generating to the end of the context."""
    h0 = json.loads(urllib.request.urlopen(server + "/health").read())
    host, port = server.split("//")[1].split(":")
    body = json.dumps({"messages": [{"role": "user", "content": "tell me a long story"}], "max_tokens": 0,
                       "temperature": 0, "stream": True}).encode()
    sock = socket.create_connection((host, int(port)), timeout=30)
    sock.sendall(b"POST /v1/chat/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                 b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
    assert b"200" in sock.recv(64)  # response started: generation is under way
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, b"\x01\x00\x00\x00\x00\x00\x00\x00")  # RST
    sock.close()
    for _ in range(400):
        h = json.loads(urllib.request.urlopen(server + "/health").read())
        if h["cancelled"] > h0["cancelled"] and h["active"] == 0:
            break
        time.sleep(0.05)
    assert h["cancelled"] == h0["cancelled"] + 1, h
    assert h["active"] == 0 and h["completed"] == h0["completed"], h
    assert _chat(server, "still serving", max_tokens=3)["choices"][0]["finish_reason"] in ("length", "stop")


def test_sampled_requests_reproducible_per_seed(server):
    """temperature > 0: the scheduler draws each row with the request's own seeded coin on the
    backend (device sampler on GPUs); the same seed gives the same text, another seed may not."""
    a = _chat(server, "sample me", max_tokens=10, temperature=0.9, top_p=0.9, seed=42)
    b = _chat(server, "sample me", max_tokens=10, temperature=0.9, top_p=0.9, seed=42)
    assert a["choices"][0]["message"]["content"] == b["choices"][0]["message"]["content"]
    assert a["usage"]["completion_tokens"] >= 1
