#!/usr/bin/env python3
"""Tiny client for dllama-api (reference: examples/chat-api-client.js), stdlib only.

    build/dllama-api --model m.m --tokenizer t.t --buffer-float-type q80 --gpu-index 0 --port 5000
    HOST=127.0.0.1 PORT=5000 python examples/chat_api_client.py [--stream]
"""
import json
import os
import sys
import urllib.request

HOST = os.environ.get("HOST", "127.0.0.1")
PORT = int(os.environ.get("PORT", "5000"))
URL = f"http://{HOST}:{PORT}/v1/chat/completions"


def chat(messages, max_tokens, stream=False):
    body = {"messages": messages, "temperature": 0.7, "stop": ["<|eot_id|>"], "max_tokens": max_tokens,
            "stream": stream}
    req = urllib.request.Request(URL, data=json.dumps(body).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req) as r:
        if not stream:
            return json.loads(r.read())
        text = ""
        for line in r:
            line = line.decode().strip()
            if not line.startswith("data:") or line == "data: [DONE]":
                continue
            delta = json.loads(line[5:])["choices"][0]["delta"].get("content", "")
            text += delta
            sys.stdout.write(delta)
            sys.stdout.flush()
        print()
        return {"choices": [{"message": {"content": text}}], "usage": None}


def ask(system, user, max_tokens, stream):
    print(f"> system: {system}\n> user: {user}")
    r = chat([{"role": "system", "content": system}, {"role": "user", "content": user}], max_tokens, stream)
    if not stream:
        print(r["usage"])
        print(r["choices"][0]["message"]["content"])


if __name__ == "__main__":
    s = "--stream" in sys.argv
    ask("You are an excellent math teacher.", "What is 1 + 2?", 128, s)
    ask("You are a romantic.", "Where is Europe?", 128, s)
