"""Hugging Face (safetensors) Llama/Mistral checkpoint -> `.m` model file.

Behaviour follows the reference converter (converter/convert-hf.py): header mapping from
config.json (:152-195), Q/K rows permuted from HF's rotate-half layout to adjacent pairs (:11-14),
tensor order (:51-89) with `lm_head` falling back to the tied `embed_tokens`. Tensors are streamed
one at a time (safetensors memory maps), so converting a 405B checkpoint needs little RAM.

usage: python -m distributed_llama_multiusers_amd.convert.hf <hf_dir> <q40|f32|f16|q80> <name> [out_dir]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

from ..utils.mfile import ARCH_LLAMA, FLOAT_TYPE_NAMES, FloatType, encode_tensor, write_header


def permute_rotary(w: np.ndarray, n_heads: int) -> np.ndarray:
    """HF stores each head's rotary dims as [first half | second half]; the runtime rotates
    adjacent pairs, so interleave the halves: row (h, i, j) <- (h, j, i)."""
    rows = w.shape[0]
    return w.reshape(n_heads, 2, rows // n_heads // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def load_config(folder: str, weights_type: int) -> dict:
    with open(os.path.join(folder, "config.json")) as f:
        c = json.load(f)
    arch = {"llama": ARCH_LLAMA, "mistral": ARCH_LLAMA}.get(c["model_type"])
    if arch is None:
        raise ValueError(f"Unsupported arch type: {c['model_type']}")
    act = {"gelu": 0, "silu": 1}.get(c.get("hidden_act", "silu"))
    if act is None:
        raise ValueError(f"Unsupported hidden act: {c['hidden_act']}")
    h = {
        "version": 0,
        "arch_type": arch,
        "hidden_act": act,
        "dim": c["hidden_size"],
        "hidden_dim": c["intermediate_size"],
        "n_layers": c["num_hidden_layers"],
        "n_heads": c["num_attention_heads"],
        "n_kv_heads": c.get("num_key_value_heads", c["num_attention_heads"]),
        "weights_float_type": weights_type,
        "max_seq_len": c["max_position_embeddings"],
        "vocab_size": c["vocab_size"],
    }
    n_exp = c.get("num_local_experts")
    if n_exp:
        raise ValueError("Mixture-of-experts checkpoints are not supported by this runtime")
    h["n_experts"] = 0
    h["n_active_experts"] = 0
    if c.get("rope_theta") is not None:
        h["rope_theta"] = int(c["rope_theta"])
    rs = c.get("rope_scaling")
    if rs is not None:
        if rs.get("rope_type", rs.get("type")) != "llama3":
            raise ValueError(f"Unsupported rope scaling: {rs}")
        h["rope_scaling_factor"] = int(rs["factor"])
        h["rope_scaling_low_freq_factor"] = int(rs["low_freq_factor"])
        h["rope_scaling_high_freq_factory"] = int(rs["high_freq_factor"])
        h["rope_scaling_orig_max_seq_len"] = int(rs["original_max_position_embeddings"])
        h["rope_type"] = 2
    return h


class _Tensors:
    """Name -> array lookup over all *.safetensors files of a folder (lazy, one tensor at a time)."""

    def __init__(self, folder: str):
        from safetensors import safe_open
        files = sorted(f for f in os.listdir(folder) if f.endswith(".safetensors") and not f.startswith("."))
        if not files:
            raise FileNotFoundError("Not found any model file")
        self.handles = [safe_open(os.path.join(folder, f), framework="np") for f in files]
        self.index = {}
        for i, h in enumerate(self.handles):
            for k in h.keys():
                self.index[k] = i

    def get(self, *names: str) -> np.ndarray:
        for n in names:
            if n in self.index:
                return np.asarray(self.handles[self.index[n]].get_tensor(n), dtype=np.float32)
        raise KeyError(f"Layer {names[0]} not found")


def plan(h: dict):
    wt = h["weights_float_type"]
    yield FloatType.F32, None, ("model.embed_tokens.weight",)
    for l in range(h["n_layers"]):
        p = f"model.layers.{l}."
        yield wt, h["n_heads"], (p + "self_attn.q_proj.weight",)
        yield wt, h["n_kv_heads"], (p + "self_attn.k_proj.weight",)
        yield wt, None, (p + "self_attn.v_proj.weight",)
        yield wt, None, (p + "self_attn.o_proj.weight",)
        yield wt, None, (p + "mlp.gate_proj.weight",)   # w1
        yield wt, None, (p + "mlp.down_proj.weight",)   # w2
        yield wt, None, (p + "mlp.up_proj.weight",)     # w3
        yield FloatType.F32, None, (p + "input_layernorm.weight",)
        yield FloatType.F32, None, (p + "post_attention_layernorm.weight",)
    yield FloatType.F32, None, ("model.norm.weight",)
    yield wt, None, ("lm_head.weight", "model.embed_tokens.weight")


def convert(folder: str, weights_type: int, out_path: str, verbose: bool = True) -> str:
    h = load_config(folder, weights_type)
    src = _Tensors(folder)
    with open(out_path, "wb") as f:
        write_header(f, h)
        for ftype, permute_heads, names in plan(h):
            t = src.get(*names)
            if permute_heads is not None:
                t = permute_rotary(t, permute_heads)
            if verbose:
                print(f"🔶 Writing tensor {names[0]} {tuple(t.shape)}...")
            f.write(encode_tensor(t, ftype))
    return out_path


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 3:
        print(__doc__)
        return 1
    folder, wt, name = argv[0], argv[1], argv[2]
    out_dir = argv[3] if len(argv) > 3 else "."
    out = os.path.join(out_dir, f"dllama_model_{name}_{wt}.m")
    print(f"Output file: {out}")
    convert(folder, FLOAT_TYPE_NAMES[wt], out)
    print(f"✅ Created {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
