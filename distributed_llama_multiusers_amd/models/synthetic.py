"""Synthetic (random-init) Llama models and tokenizers in the reference `.m` / `.t` formats.

There is no network: benchmarks and tests use random weights of the real architectures
(shapes: SURVEY.md Appendix A). For big models the HIP engine can also initialise weights
directly on device (see HipEngine(synthetic=...)), which skips the multi-GB file.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from ..utils.mfile import FloatType, ModelSpec, tensor_plan, write_model
from ..utils.tfile import write_tokenizer

# Public Llama shapes
LLAMA_SHAPES = {
    "llama3_2_1b": dict(dim=2048, hidden_dim=8192, n_layers=16, n_heads=32, n_kv_heads=8, vocab_size=128256),
    "llama3_2_3b": dict(dim=3072, hidden_dim=8192, n_layers=28, n_heads=24, n_kv_heads=8, vocab_size=128256),
    "llama3_1_8b": dict(dim=4096, hidden_dim=14336, n_layers=32, n_heads=32, n_kv_heads=8, vocab_size=128256),
    "llama3_3_70b": dict(dim=8192, hidden_dim=28672, n_layers=80, n_heads=64, n_kv_heads=8, vocab_size=128256),
    "llama3_1_405b": dict(dim=16384, hidden_dim=53248, n_layers=126, n_heads=128, n_kv_heads=8, vocab_size=128256),
    "llama2_7b": dict(dim=4096, hidden_dim=11008, n_layers=32, n_heads=32, n_kv_heads=32, vocab_size=32000),
}

LLAMA31_ROPE = dict(rope_theta=500000, rope_scaling_factor=8, rope_scaling_low_freq_factor=1,
                    rope_scaling_high_freq_factory=4, rope_scaling_orig_max_seq_len=8192, rope_type=2)

LLAMA3_CHAT_TEMPLATE = (b"{% set loop_messages = messages %}{% for message in loop_messages %}"
                        b"{% set content = '<|start_header_id|>' + message['role'] + '<|end_header_id|>\\n\\n'"
                        b"+ message['content'] | trim + '<|eot_id|>' %}{{ content }}{% endfor %}"
                        b"{% if add_generation_prompt %}{{ '<|start_header_id|>assistant<|end_header_id|>\\n\\n' }}"
                        b"{% endif %}")

SPECIAL_TOKENS = [b"<|begin_of_text|>", b"<|end_of_text|>", b"<|start_header_id|>", b"<|end_header_id|>",
                  b"<|eot_id|>"]

_MERGES = ["th", "he", "in", "er", "an", "re", "on", "at", "en", "nd", "ti", "es", "or", "te", "of", "ed", "is",
           "it", "al", "ar", "st", "to", "nt", "ng", "se", "ha", "as", "ou", "io", "le", "ve", "co", "me", "de",
           "hi", "ri", "ro", "ic", "ne", "ea", "ra", "ce", "li", "ch", "ll", "be", "ma", "si", "om", "ur", " t",
           " a", " s", " w", " o", " i", " c", " b", " the", "the", " of", " and", "and", "ing", " to", " in",
           "ion", "tion", " is", " that", "ent", " for", " it", " was", " on", " as", " with", "er ", "ed ",
           " he", " be", "hello", " hello", " world", "world", "Hello", " Hello", "Th", "The", " The", "ll",
           "llo", "ello", "wor", "orld", "rld"]


def make_tokenizer(path: str, vocab_size: int, chat_template: Optional[bytes] = LLAMA3_CHAT_TEMPLATE) -> dict:
    """Writes a synthetic BPE tokenizer whose regular vocabulary is the 256 bytes + common merges.

    Regular tokens occupy ids [0, bos_id); special tokens follow (the reference's convention,
    tokenizer.cpp:137-138)."""
    n_special = len(SPECIAL_TOKENS)
    n_regular = vocab_size - n_special
    assert n_regular >= 256, "vocab too small"
    tokens = [bytes([i]) for i in range(256)]
    scores = [0.0] * 256
    seen = set(tokens)
    for i, m in enumerate(_MERGES):
        b = m.encode()
        if b not in seen and len(tokens) < n_regular:
            seen.add(b)
            tokens.append(b)
            scores.append(float(len(b)) + 0.001 * i)
    i = 0
    while len(tokens) < n_regular:
        b = f"<x{i}>".encode()
        i += 1
        if b in seen:
            continue
        seen.add(b)
        tokens.append(b)
        scores.append(-1.0)
    bos_id = len(tokens)
    tokens += SPECIAL_TOKENS
    scores += [0.0] * n_special
    eos = [bos_id + 1, bos_id + 4]  # <|end_of_text|>, <|eot_id|>
    write_tokenizer(path, tokens, scores, chat_template, bos_id, eos)
    return {"bos_id": bos_id, "eos": eos, "tokens": tokens}


def make_spec(name: str = "tiny", weights: int = FloatType.Q40, seq_len: int = 256, **overrides) -> ModelSpec:
    if name == "tiny":
        base = dict(dim=256, hidden_dim=512, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=512)
    else:
        base = dict(LLAMA_SHAPES[name])
    base.update(overrides)
    return ModelSpec(max_seq_len=seq_len, weights_float_type=weights, **base)


def random_tensors(spec: ModelSpec, seed: int = 0) -> Dict[tuple, np.ndarray]:
    rng = np.random.default_rng(seed)
    out = {}
    for name, layer, rows, cols, _ in tensor_plan(spec):
        if name == "embedding":
            x = rng.standard_normal((rows, cols), dtype=np.float32)
        elif name.startswith("rms"):
            x = (1.0 + 0.1 * rng.standard_normal((rows, cols))).astype(np.float32)
        else:
            x = (rng.standard_normal((rows, cols), dtype=np.float32) / np.sqrt(cols)).astype(np.float32)
        out[(name, layer)] = x
    return out


def make_model(path: str, spec: ModelSpec, seed: int = 0) -> Dict[tuple, np.ndarray]:
    t = random_tensors(spec, seed)
    write_model(path, spec, t)
    return t


def make_test_assets(directory: str, name: str = "tiny", weights: int = FloatType.Q40, seq_len: int = 256,
                     seed: int = 0, **overrides) -> tuple:
    os.makedirs(directory, exist_ok=True)
    spec = make_spec(name, weights, seq_len, **overrides)
    wt = "q40" if weights == FloatType.Q40 else "f32"
    mpath = os.path.join(directory, f"{name}_{wt}.m")
    tpath = os.path.join(directory, f"{name}.t")
    if not os.path.exists(mpath):
        make_model(mpath, spec, seed)
    if not os.path.exists(tpath):
        make_tokenizer(tpath, spec.vocab_size)
    return mpath, tpath, spec
