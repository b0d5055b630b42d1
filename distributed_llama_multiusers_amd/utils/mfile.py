"""`.m` model file format: header writer/reader and tensor codecs (F32 / F16 / Q40 / Q80).

Byte-compatible with the reference format (converter/writer.py:29-145, src/llm.cpp:26-98,
tensor order src/llm.cpp:447-483). Quantizers are vectorised numpy versions with the same
semantics as the reference writer: Q40 uses d = (signed max-magnitude value) / -8 and
q = clip(x/d + 8.5, 0, 15) truncated; Q80 uses d = amax / 127 and round-half-even.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import BinaryIO, Dict, List, Optional

import numpy as np

MODEL_MAGIC = 0xA00ABCD
ARCH_LLAMA = 0xABCD00


class FloatType:
    F32 = 0
    F16 = 1
    Q40 = 2
    Q80 = 3


FLOAT_TYPE_NAMES = {"f32": FloatType.F32, "f16": FloatType.F16, "q40": FloatType.Q40, "q80": FloatType.Q80}

HEADER_KEYS = {
    "version": 0,
    "arch_type": 1,
    "dim": 2,
    "hidden_dim": 3,
    "n_layers": 4,
    "n_heads": 5,
    "n_kv_heads": 6,
    "n_experts": 7,
    "n_active_experts": 8,
    "vocab_size": 9,
    "max_seq_len": 10,
    "hidden_act": 11,
    "rope_theta": 12,
    "weights_float_type": 13,
    "rope_scaling_factor": 14,
    "rope_scaling_low_freq_factor": 15,
    "rope_scaling_high_freq_factory": 16,
    "rope_scaling_orig_max_seq_len": 17,
    "rope_type": 18,
}
HEADER_KEYS_INV = {v: k for k, v in HEADER_KEYS.items()}

Q40_DTYPE = np.dtype([("d", "<f2"), ("qs", "u1", (16,))])
Q80_DTYPE = np.dtype([("d", "<f2"), ("qs", "i1", (32,))])


def quantize_q40(x: np.ndarray) -> np.ndarray:
    """float array (size % 32 == 0) -> structured Q40 blocks."""
    g = np.asarray(x, dtype=np.float32).reshape(-1, 32)
    gmax = g.max(axis=1)
    gmin = g.min(axis=1)
    deltas = np.where(-gmin > gmax, gmin, gmax) / np.float32(-8.0)
    deltas = deltas.astype(np.float32)
    with np.errstate(divide="ignore"):
        ids = np.where(deltas != 0, np.float32(1.0) / deltas, np.float32(0.0)).astype(np.float32)
    q = np.clip(g * ids[:, None] + np.float32(8.5), 0, 15).astype(np.int32)
    out = np.empty(g.shape[0], dtype=Q40_DTYPE)
    out["d"] = deltas.astype(np.float16)
    out["qs"] = ((q[:, :16] & 0xF) | ((q[:, 16:] & 0xF) << 4)).astype(np.uint8)
    return out


def dequantize_q40(blocks: np.ndarray) -> np.ndarray:
    d = blocks["d"].astype(np.float32)[:, None]
    qs = blocks["qs"].astype(np.int32)
    lo = (qs & 0xF) - 8
    hi = (qs >> 4) - 8
    return (np.concatenate([lo, hi], axis=1).astype(np.float32) * d).reshape(-1)


def quantize_q80(x: np.ndarray) -> np.ndarray:
    g = np.asarray(x, dtype=np.float32).reshape(-1, 32)
    amax = np.abs(g).max(axis=1)
    d = (amax / np.float32(127.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        ids = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    q = np.clip(np.rint(g * ids[:, None]), -127, 127).astype(np.int8)
    out = np.empty(g.shape[0], dtype=Q80_DTYPE)
    out["d"] = d.astype(np.float16)
    out["qs"] = q
    return out


def dequantize_q80(blocks: np.ndarray) -> np.ndarray:
    return (blocks["qs"].astype(np.float32) * blocks["d"].astype(np.float32)[:, None]).reshape(-1)


def tensor_bytes(ftype: int, n: int) -> int:
    if ftype == FloatType.F32:
        return 4 * n
    if ftype == FloatType.F16:
        return 2 * n
    if ftype == FloatType.Q40:
        return n // 32 * 18
    if ftype == FloatType.Q80:
        return n // 32 * 34
    raise ValueError(ftype)


def encode_tensor(x: np.ndarray, ftype: int) -> bytes:
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float32)).reshape(-1)
    if ftype == FloatType.F32:
        return x.astype("<f4").tobytes()
    if ftype == FloatType.F16:
        return x.astype("<f2").tobytes()
    if ftype == FloatType.Q40:
        return quantize_q40(x).tobytes()
    if ftype == FloatType.Q80:
        return quantize_q80(x).tobytes()
    raise ValueError(ftype)


def decode_tensor(buf: bytes, ftype: int, n: int) -> np.ndarray:
    if ftype == FloatType.F32:
        return np.frombuffer(buf, dtype="<f4", count=n).astype(np.float32)
    if ftype == FloatType.F16:
        return np.frombuffer(buf, dtype="<f2", count=n).astype(np.float32)
    if ftype == FloatType.Q40:
        return dequantize_q40(np.frombuffer(buf, dtype=Q40_DTYPE, count=n // 32))
    if ftype == FloatType.Q80:
        return dequantize_q80(np.frombuffer(buf, dtype=Q80_DTYPE, count=n // 32))
    raise ValueError(ftype)


def write_header(f: BinaryIO, params: Dict[str, int]) -> None:
    data = b""
    for k, v in params.items():
        if k not in HEADER_KEYS:
            raise KeyError(f"unknown header key {k}")
        data += struct.pack("<ii", HEADER_KEYS[k], int(v))
    f.write(struct.pack("<ii", MODEL_MAGIC, 8 + len(data)))
    f.write(data)


@dataclass
class ModelSpec:
    dim: int
    hidden_dim: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    vocab_size: int
    max_seq_len: int
    weights_float_type: int = FloatType.Q40
    hidden_act: int = 1  # 0 gelu, 1 silu
    rope_theta: int = 10000
    rope_scaling_factor: Optional[int] = None
    rope_scaling_low_freq_factor: Optional[int] = None
    rope_scaling_high_freq_factory: Optional[int] = None
    rope_scaling_orig_max_seq_len: Optional[int] = None
    rope_type: Optional[int] = None
    extra: Dict[str, int] = field(default_factory=dict)

    @property
    def head_size(self) -> int:
        return self.dim // self.n_heads

    @property
    def kv_dim(self) -> int:
        return self.head_size * self.n_kv_heads

    def header_params(self) -> Dict[str, int]:
        p = {
            "version": 0,
            "arch_type": ARCH_LLAMA,
            "dim": self.dim,
            "hidden_dim": self.hidden_dim,
            "n_layers": self.n_layers,
            "n_heads": self.n_heads,
            "n_kv_heads": self.n_kv_heads,
            "n_experts": 0,
            "n_active_experts": 0,
            "vocab_size": self.vocab_size,
            "max_seq_len": self.max_seq_len,
            "hidden_act": self.hidden_act,
            "rope_theta": self.rope_theta,
            "weights_float_type": self.weights_float_type,
        }
        for k in ("rope_scaling_factor", "rope_scaling_low_freq_factor", "rope_scaling_high_freq_factory",
                  "rope_scaling_orig_max_seq_len", "rope_type"):
            v = getattr(self, k)
            if v is not None:
                p[k] = v
        p.update(self.extra)
        return p


def tensor_plan(spec: ModelSpec) -> List[tuple]:
    """(name, layer, rows, cols, float_type) in file order (llm.cpp:460-475)."""
    w = spec.weights_float_type
    t = [("embedding", -1, spec.vocab_size, spec.dim, FloatType.F32)]
    for l in range(spec.n_layers):
        t += [
            ("q", l, spec.dim, spec.dim, w),
            ("k", l, spec.kv_dim, spec.dim, w),
            ("v", l, spec.kv_dim, spec.dim, w),
            ("wo", l, spec.dim, spec.dim, w),
            ("w1", l, spec.hidden_dim, spec.dim, w),
            ("w2", l, spec.dim, spec.hidden_dim, w),
            ("w3", l, spec.hidden_dim, spec.dim, w),
            ("rms_att", l, 1, spec.dim, FloatType.F32),
            ("rms_ffn", l, 1, spec.dim, FloatType.F32),
        ]
    t += [("rms_final", -1, 1, spec.dim, FloatType.F32), ("wcls", -1, spec.vocab_size, spec.dim, w)]
    return t


def write_model(path: str, spec: ModelSpec, tensors: Dict[tuple, np.ndarray]) -> None:
    """tensors keyed by (name, layer) with shape (rows, cols) or flat."""
    with open(path, "wb") as f:
        write_header(f, spec.header_params())
        for name, layer, rows, cols, ftype in tensor_plan(spec):
            x = tensors[(name, layer)]
            assert x.size == rows * cols, (name, layer, x.shape)
            f.write(encode_tensor(x, ftype))


def read_header(path: str) -> Dict[str, int]:
    with open(path, "rb") as f:
        magic, header_size = struct.unpack("<ii", f.read(8))
        if magic != MODEL_MAGIC:
            raise ValueError("Unsupported magic number")
        n = (header_size - 8) // 4
        vals = struct.unpack(f"<{n}i", f.read(header_size - 8))
    out = {"header_size": header_size}
    for i in range(0, n, 2):
        out[HEADER_KEYS_INV[vals[i]]] = vals[i + 1]
    return out


def spec_from_header(h: Dict[str, int]) -> ModelSpec:
    return ModelSpec(
        dim=h["dim"], hidden_dim=h["hidden_dim"], n_layers=h["n_layers"], n_heads=h["n_heads"],
        n_kv_heads=h["n_kv_heads"], vocab_size=h["vocab_size"], max_seq_len=h["max_seq_len"],
        weights_float_type=h["weights_float_type"], hidden_act=h.get("hidden_act", 1),
        rope_theta=h.get("rope_theta", 10000), rope_scaling_factor=h.get("rope_scaling_factor"),
        rope_scaling_low_freq_factor=h.get("rope_scaling_low_freq_factor"),
        rope_scaling_high_freq_factory=h.get("rope_scaling_high_freq_factory"),
        rope_scaling_orig_max_seq_len=h.get("rope_scaling_orig_max_seq_len"), rope_type=h.get("rope_type"))


def read_model(path: str) -> tuple:
    """Returns (header dict, spec, {(name, layer): float32 array (rows, cols)}) — dequantized."""
    h = read_header(path)
    spec = spec_from_header(h)
    out = {}
    with open(path, "rb") as f:
        f.seek(h["header_size"])
        for name, layer, rows, cols, ftype in tensor_plan(spec):
            nbytes = tensor_bytes(ftype, rows * cols)
            out[(name, layer)] = decode_tensor(f.read(nbytes), ftype, rows * cols).reshape(rows, cols)
        rest = f.read()
        if rest:
            raise ValueError(f"Missing bytes in weight file: {-len(rest)}")
    return h, spec, out


def write_random_model(path: str, spec: ModelSpec, seed: int = 0, chunk_bytes: int = 64 << 20) -> int:
    """Write a full-size model of random weights without materialising it: Q40 tensors get random
    nibbles and scales of 1/sqrt(21.5 n) (unit-variance activations, like the engine's synthetic
    init), f32 tensors uniform [-1, 1) (norm weights 1). Streams `chunk_bytes` at a time, so an
    8B-parameter file (4.6 GB) needs ~100 MB of RAM. Returns the file size."""
    rng = np.random.default_rng(seed)
    q40 = np.dtype([("d", "<f2"), ("qs", "u1", (16,))])
    with open(path, "wb") as f:
        write_header(f, spec.header_params())
        for name, layer, rows, cols, ftype in tensor_plan(spec):
            n = rows * cols
            if ftype == FloatType.Q40:
                nblk, per = n // 32, max(1, chunk_bytes // 18)
                scale = np.float16(1.0 / np.sqrt(21.5 * cols))
                for b0 in range(0, nblk, per):
                    m = min(per, nblk - b0)
                    blk = np.empty(m, dtype=q40)
                    blk["d"] = scale
                    blk["qs"] = rng.integers(0, 256, size=(m, 16), dtype=np.uint8)
                    f.write(blk.tobytes())
            elif ftype == FloatType.F32:
                if name.startswith("rms"):
                    f.write(np.ones(n, dtype=np.float32).tobytes())
                    continue
                per = max(1, chunk_bytes // 4)
                for e0 in range(0, n, per):
                    m = min(per, n - e0)
                    # uniform [-1, 1) from raw bits: mantissa into [1, 2), then 2 x - 3
                    u = (rng.integers(0, 1 << 32, size=m, dtype=np.uint32) >> np.uint32(9)) | np.uint32(0x3F800000)
                    v = u.view(np.float32)
                    v *= 2
                    v -= 3
                    f.write(v.tobytes())
            else:
                raise ValueError(f"write_random_model: unsupported float type {ftype}")
        return f.tell()
