"""`.t` tokenizer file format (reference: converter/tokenizer-writer.py:3-55, src/tokenizer.cpp:42-170)."""
from __future__ import annotations

import struct
from typing import List, Optional

TOKENIZER_MAGIC = 0x567124
TOKENIZER_KEYS = {"version": 0, "vocab_size": 1, "max_token_length": 2, "bos_id": 3, "chat_template": 7,
                  "n_eos_tokens": 9}


def write_tokenizer(path: str, tokens: List[bytes], scores: List[float], chat_template: Optional[bytes],
                    bos_id: int, eos_tokens: List[int]) -> None:
    params = {"bos_id": bos_id, "version": 1, "vocab_size": len(tokens),
              "max_token_length": max(len(t) for t in tokens)}
    if chat_template:
        params["chat_template"] = len(chat_template)
    params["n_eos_tokens"] = len(eos_tokens)
    data = b"".join(struct.pack("<ii", TOKENIZER_KEYS[k], v) for k, v in params.items())
    with open(path, "wb") as f:
        f.write(struct.pack("<ii", TOKENIZER_MAGIC, 8 + len(data)))
        f.write(data)
        if chat_template:
            f.write(chat_template)
        for e in eos_tokens:
            f.write(struct.pack("<i", e))
        for t, s in zip(tokens, scores):
            assert len(t) > 0
            f.write(struct.pack("<fI", s, len(t)))
            f.write(t)


def read_tokenizer(path: str) -> dict:
    with open(path, "rb") as f:
        data = f.read()
    off = 0

    def get(fmt):
        nonlocal off
        v = struct.unpack_from(fmt, data, off)
        off += struct.calcsize(fmt)
        return v

    magic, = get("<i")
    if magic != TOKENIZER_MAGIC:
        raise ValueError("Invalid tokenizer file")
    header_size, = get("<i")
    kv = get(f"<{(header_size - 8) // 4}i")
    params = {}
    inv = {v: k for k, v in TOKENIZER_KEYS.items()}
    for i in range(0, len(kv), 2):
        params[inv.get(kv[i], kv[i])] = kv[i + 1]
    tmpl = None
    if params.get("chat_template", 0) > 0:
        tmpl = data[off:off + params["chat_template"]]
        off += params["chat_template"]
    eos = [get("<i")[0] for _ in range(params.get("n_eos_tokens", 0))]
    tokens, scores = [], []
    for _ in range(params["vocab_size"]):
        s, n = get("<fI")
        tokens.append(data[off:off + n])
        off += n
        scores.append(s)
    return {"params": params, "chat_template": tmpl, "eos": eos, "tokens": tokens, "scores": scores}
