"""Hugging Face tokenizer (tokenizer.json fast tokenizers or sentencepiece tokenizer.model) -> `.t`.

Same token/score conventions as the reference converter (converter/convert-tokenizer-hf.py):
byte-level BPE tokens are mapped back to raw bytes through the GPT-2 byte<->unicode table and
scored -id (earlier merges win); sentencepiece pieces keep their scores, '▁' becomes ' ' and
<0xXX> byte pieces become raw bytes. The chat template and eos ids are embedded.

usage: python -m distributed_llama_multiusers_amd.convert.tokenizer_hf <hf_dir> <name> [out_dir]
"""
from __future__ import annotations

import json
import os
import sys

from ..utils.tfile import write_tokenizer


def unicode_to_bytes() -> dict:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip([chr(c) for c in cs], bs))


def _json(path):
    with open(path, encoding="utf-8") as f:
        return json.load(f)


def resolve_fast(folder: str):
    from tokenizers import Tokenizer
    tok = Tokenizer.from_file(os.path.join(folder, "tokenizer.json"))
    utb = unicode_to_bytes()
    n = tok.get_vocab_size(with_added_tokens=True)
    tokens, scores = [], []
    for i in range(n):
        piece = tok.id_to_token(i)
        if piece is None:
            piece = f"<unused{i}>"
        out = []
        for ch in piece:
            if ch in utb:
                out.append(utb[ch])
            else:
                out += list(ch.encode("utf-8"))
        tokens.append(bytes(out))
        scores.append(-float(i))
    return tokens, scores


def resolve_sentencepiece(folder: str):
    from sentencepiece import SentencePieceProcessor
    sp = SentencePieceProcessor(model_file=os.path.join(folder, "tokenizer.model"))
    tokens, scores = [], []
    for i in range(sp.vocab_size()):
        t = sp.id_to_piece(i).replace("▁", " ")
        b = bytes.fromhex(t[3:-1]) if (len(t) == 6 and t.startswith("<0x") and t.endswith(">")) else t.encode("utf-8")
        tokens.append(b)
        scores.append(sp.get_score(i))
    return tokens, scores, sp.bos_id(), [sp.eos_id()]


def convert(folder: str, out_path: str) -> str:
    cfg = _json(os.path.join(folder, "tokenizer_config.json"))
    cls = cfg.get("tokenizer_class", "PreTrainedTokenizerFast")
    bos, eos = None, None
    if cls == "LlamaTokenizer" and os.path.exists(os.path.join(folder, "tokenizer.model")):
        tokens, scores, bos, eos = resolve_sentencepiece(folder)
    elif os.path.exists(os.path.join(folder, "tokenizer.json")):
        tokens, scores = resolve_fast(folder)
    else:
        raise ValueError(f"Tokenizer {cls} is not supported")
    if bos is None or not eos:
        model_cfg = _json(os.path.join(folder, "config.json")) if os.path.exists(os.path.join(folder, "config.json")) else {}
        by_text = {t: i for i, t in enumerate(tokens)}
        def tid(v):
            if isinstance(v, dict):
                v = v.get("content")
            return by_text.get(v.encode()) if isinstance(v, str) else v
        bos = bos if bos is not None else (tid(cfg.get("bos_token")) if cfg.get("bos_token") else model_cfg.get("bos_token_id"))
        e = tid(cfg.get("eos_token")) if cfg.get("eos_token") else model_cfg.get("eos_token_id")
        eos = eos or (e if isinstance(e, list) else [e])
        extra = model_cfg.get("eos_token_id")
        if isinstance(extra, list):
            eos = list(dict.fromkeys(eos + extra))
    if bos is None or not eos or None in eos:
        raise ValueError("Cannot resolve bosId or eosIds")
    tmpl = cfg.get("chat_template")
    write_tokenizer(out_path, tokens, scores, tmpl.encode("utf-8") if isinstance(tmpl, str) else None, bos, eos)
    return out_path


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print(__doc__)
        return 1
    out = os.path.join(argv[2] if len(argv) > 2 else ".", f"dllama_tokenizer_{argv[1]}.t")
    convert(argv[0], out)
    print(f"✅ Created {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
