"""Kernel-level access to the gfx950 HIP kernels, plus plain PyTorch fp32 references of the same ops.

Each `*` function runs exactly one kernel of `csrc/hip/kernels.hip` the way the engine launches it
(same weight tiling, fused prologue / epilogue) through `_C.ops` (csrc/hip/ops.cpp); each `ref_*`
is the textbook fp32 definition. They exist for numerics tests (tests/test_gpu_ops.py) and for
experiments; the inference hot path never goes through Python.

Reference semantics: OP_MATMUL Q80 x Q40 (nn-cpu-ops.cpp:222-440), RMS norm
(nn-cpu-ops.cpp:105-166), RoPE over adjacent pairs (nn-cpu-ops.cpp:1090-1120), multi-head attention
with GQA (nn-cpu-ops.cpp:749-784), SiLU (nn-cpu-ops.cpp:453-491), embedding (nn-cpu-ops.cpp:880-892).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import native


def _np(x, dtype=np.float32):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(x, dtype=dtype)


# ---------------------------------------------------------------------------------------- codecs
def quantize_q40(w: torch.Tensor) -> np.ndarray:
    """[rows, n] float -> Q40 blocks in file layout (uint8, rows * n/32 * 18 bytes)."""
    return native().quantize_q40(_np(w).reshape(-1))


def dequantize_q40(blocks: np.ndarray, rows: int, n: int) -> torch.Tensor:
    return torch.from_numpy(native().dequantize_q40(blocks).reshape(rows, n))


def dequantize_q80(x: torch.Tensor) -> torch.Tensor:
    """Round trip through the reference Q80 quantizer (what a Q80 hand-off between kernels does)."""
    C = native()
    flat = _np(x).reshape(-1)
    return torch.from_numpy(C.dequantize_q80(C.quantize_q80(flat)).reshape(x.shape))


# ------------------------------------------------------------------------------- HIP kernels
def gemv_q40(blocks, rows: int, n: int, x, residual=None, norm_w=None, eps: float = 1e-5, swiglu: bool = False):
    """Decode GEMV (1, 2 or 4 rows): (x + residual) -> RMS norm (norm_w) -> Q80 -> W.x.
    swiglu: rows are interleaved (w1, w3) pairs and the result is silu(w1.x) * (w3.x).
    Returns (out [B, rows or rows/2], x + residual or None)."""
    out, xn = native().ops.gemv_q40(_np(blocks, np.uint8), rows, n, _np(x), _np(residual), _np(norm_w), eps,
                                    1 if swiglu else 0)
    return torch.from_numpy(out), (torch.from_numpy(xn) if xn is not None else None)


def gemv_q40_q80_in(blocks, rows: int, n: int, x) -> torch.Tensor:
    """Decode GEMV on activations handed over as Q80 blocks (the wo / w2 path)."""
    return torch.from_numpy(native().ops.gemv_q40_q80_in(_np(blocks, np.uint8), rows, n, _np(x)))


def gemm_q40(blocks, rows: int, n: int, x, residual=None, norm_w=None, eps: float = 1e-5,
             splits: int = 0) -> torch.Tensor:
    """Batched (MFMA) matmul for 1..2048 tokens: (x + residual) -> RMS norm -> f16 -> W.x (f32
    accumulate); narrow 64-row tiles up to 64 tokens, 128 x 128 wide tiles above. `splits` > 0
    forces the K split (a divisor of n / 32)."""
    return torch.from_numpy(native().ops.gemm_q40(_np(blocks, np.uint8), rows, n, _np(x), _np(residual),
                                                  _np(norm_w), eps, splits))


def gemm_f32(w, x, norm_w=None, eps: float = 1e-5) -> torch.Tensor:
    """Batched (MFMA, v_mfma_f32_16x16x4_f32) matmul for F32 weights [rows][n], 1..256 tokens:
    x -> RMS norm -> f16 -> W.x (weights exact in f32, f32 accumulate)."""
    rows, n = w.shape
    return torch.from_numpy(native().ops.gemm_f32(_np(w), rows, n, _np(x), _np(norm_w), eps))


def qkv_rope(blocks, q0: int, kv0: int, head_size: int, n: int, x, norm_w, eps: float, rope, seq_len: int,
             pos, kv_bf16: bool = True):
    """QKV GEMV with the RoPE + KV-cache-append epilogue. Returns (q rotated, k row, v row)."""
    q, k, v = native().ops.qkv_rope(_np(blocks, np.uint8), q0, kv0, head_size, n, _np(x), _np(norm_w), eps,
                                    _np(rope), seq_len, [int(p) for p in pos], kv_bf16)
    return torch.from_numpy(q), torch.from_numpy(k), torch.from_numpy(v)


def attention(q, k_cache, v_cache, n_heads0: int, kv_mul: int, head_size: int, pos, slot,
              kv_bf16: bool = True, prefill: bool = False, impl: str = "auto") -> torch.Tensor:
    """Decode attention. k_cache / v_cache: [slots, seq_len, kv0]; q: [B, n_heads0 * head_size].
    prefill=True (impl "prefill"): the MFMA prefill kernel (bf16 MFMAs for a bf16 cache, f32 MFMAs
    for an f32 one; row blocks of 64 / kv_mul rows share a slot). impl "valu" / "mfma": force the VALU or the MFMA decode kernel ("auto": the
    engine's choice, MFMA for bf16 caches of >= 1024 positions)."""
    n_slots, seq_len, _ = k_cache.shape
    code = {"auto": 0, "prefill": 1, "valu": 2, "mfma": 3}["prefill" if prefill else impl]
    return torch.from_numpy(native().ops.attention(_np(q), _np(k_cache), _np(v_cache), n_slots, seq_len, n_heads0,
                                                   kv_mul, head_size, [int(p) for p in pos], [int(s) for s in slot],
                                                   kv_bf16, code))


def sample(logits, temperatures, topps, coins) -> list:
    """Device sampler: per row softmax(logits / T) then multinomial (top-p >= 1) or nucleus draw."""
    x = _np(logits)
    B = x.shape[0] if x.ndim == 2 else 1
    spec = np.stack([np.asarray(temperatures, np.float32), np.asarray(topps, np.float32),
                     np.asarray(coins, np.float32), np.zeros(B, np.float32)], axis=1)
    return native().ops.sample(x, B, spec)


def argmax(logits) -> list:
    x = _np(logits)
    return native().ops.argmax(x, x.shape[0] if x.ndim == 2 else 1)


def embedding(table, tokens) -> torch.Tensor:
    t = _np(table)
    return torch.from_numpy(native().ops.embedding(t, t.shape[0], t.shape[1], [int(x) for x in tokens]))


# --------------------------------------------------------------------------- fp32 references
def ref_rmsnorm(x: torch.Tensor, w: torch.Tensor | None, eps: float = 1e-5) -> torch.Tensor:
    x = x.float()
    if w is None:
        return x
    return w.float() * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps))


def ref_swiglu(y: torch.Tensor) -> torch.Tensor:
    """Interleaved (w1, w3) rows -> silu(w1 x) * (w3 x)."""
    return torch.nn.functional.silu(y[..., 0::2]) * y[..., 1::2]


def ref_rope(x: torch.Tensor, rope: torch.Tensor, pos: int, head_size: int) -> torch.Tensor:
    """Rotate adjacent pairs (i, i+1) of every head by the table row at `pos` ([seq_len, hs/2, 2])."""
    v = x.float().reshape(-1, head_size // 2, 2)
    cs = rope[pos].float()
    c, s = cs[:, 0], cs[:, 1]
    out = torch.stack([v[..., 0] * c - v[..., 1] * s, v[..., 0] * s + v[..., 1] * c], dim=-1)
    return out.reshape(x.shape)


def ref_rope_table(seq_len: int, head_size: int, theta: float = 10000.0) -> torch.Tensor:
    i = torch.arange(0, head_size, 2, dtype=torch.float64) / head_size
    freq = 1.0 / (theta ** i)
    ang = torch.arange(seq_len, dtype=torch.float64)[:, None] * freq[None, :]
    return torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).float()


def ref_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, n_heads0: int, kv_mul: int,
                  head_size: int, pos, slot) -> torch.Tensor:
    out = torch.zeros(q.shape[0], n_heads0 * head_size)
    for b in range(q.shape[0]):
        for h in range(n_heads0):
            kvh = h // kv_mul
            qh = q[b, h * head_size:(h + 1) * head_size].float()
            K = k_cache[slot[b], :pos[b] + 1, kvh * head_size:(kvh + 1) * head_size].float()
            V = v_cache[slot[b], :pos[b] + 1, kvh * head_size:(kvh + 1) * head_size].float()
            p = torch.softmax(K @ qh / head_size ** 0.5, dim=0)
            out[b, h * head_size:(h + 1) * head_size] = p @ V
    return out


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("annotations", "np", "torch", "native")]
