"""Meta-format Llama checkpoint (params.json + consolidated.NN.pth model-parallel shards) -> `.m`.

Same tensor order and shard-merge axes as the reference (converter/convert-llama.py:33-97): the
embedding, wo and w2 are split along columns across `consolidated.*.pth` files, everything else
along rows; Meta checkpoints already use the adjacent-pair rotary layout (no permutation).
Shards are opened with `torch.load(weights_only=True, mmap=True)`, so nothing in the file is
executed and each tensor is paged in only when it is written.

usage: python -m distributed_llama_multiusers_amd.convert.meta <model_dir> <q40|f32|f16|q80> [out_dir]
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np

from ..utils.mfile import ARCH_LLAMA, FLOAT_TYPE_NAMES, FloatType, encode_tensor, write_header

_COL_SPLIT = ("tok_embeddings.weight", ".attention.wo.weight", ".feed_forward.w2.weight")
_F32 = ("tok_embeddings.weight", ".attention_norm.weight", ".ffn_norm.weight")


def tensor_names(n_layers: int):
    yield "tok_embeddings.weight"
    for l in range(n_layers):
        for n in ("attention.wq", "attention.wk", "attention.wv", "attention.wo",
                  "feed_forward.w1", "feed_forward.w2", "feed_forward.w3", "attention_norm", "ffn_norm"):
            yield f"layers.{l}.{n}.weight"
    yield "norm.weight"
    yield "output.weight"


def convert(model_dir: str, weights_type: int, out_path: str, verbose: bool = True) -> str:
    import torch
    with open(os.path.join(model_dir, "params.json")) as f:
        p = json.load(f)
    if p.get("vocab_size", 0) < 1:
        raise ValueError("vocab_size is invalid, please update params.json file")
    if p.get("max_seq_len") is None:
        raise ValueError("max_seq_len is required, please update params.json file")
    shards = sorted(Path(model_dir).glob("consolidated.*.pth"))
    if not shards:
        raise FileNotFoundError("no consolidated.*.pth files")
    models = [torch.load(str(s), map_location="cpu", weights_only=True, mmap=True) for s in shards]
    h = {"version": 0, "arch_type": ARCH_LLAMA, "dim": p["dim"],
         "hidden_dim": models[0]["layers.0.feed_forward.w1.weight"].shape[0] * len(models),
         "n_layers": p["n_layers"], "n_heads": p["n_heads"], "n_kv_heads": p.get("n_kv_heads") or p["n_heads"],
         "n_experts": 0, "n_active_experts": 0, "vocab_size": p["vocab_size"], "max_seq_len": p["max_seq_len"],
         "weights_float_type": weights_type}
    if "rope_theta" in p:
        h["rope_theta"] = int(p["rope_theta"])
    with open(out_path, "wb") as f:
        write_header(f, h)
        for name in tensor_names(p["n_layers"]):
            parts = [m[name] for m in models]
            if len(parts) == 1 or parts[0].dim() == 1:
                t = parts[0]
            else:
                t = torch.cat(parts, dim=1 if name.endswith(_COL_SPLIT) else 0)
            ftype = FloatType.F32 if (name.endswith(_F32) or name == "norm.weight") else weights_type
            if verbose:
                print(f"🔶 Exporting {name} {tuple(t.shape)}...")
            f.write(encode_tensor(t.float().numpy(), ftype))
    return out_path


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print(__doc__)
        return 1
    name = os.path.basename(os.path.normpath(argv[0])).lower()
    out = os.path.join(argv[2] if len(argv) > 2 else ".", f"dllama_model_{name}_{argv[1]}.m")
    print(f"Target file: {out}")
    convert(argv[0], FLOAT_TYPE_NAMES[argv[1]], out)
    print("Done!")
    return 0


if __name__ == "__main__":
    sys.exit(main())
