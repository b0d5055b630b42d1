"""Plain PyTorch fp32 Llama forward used as the numerical oracle for the C++ CPU backend and the
HIP kernels (SURVEY §4 "HIP-vs-PyTorch oracle tests").

Semantics follow the reference graph (src/llm.cpp:184-434): pre-norm blocks, RoPE over adjacent
pairs (Q/K rows are pre-permuted in the .m file, convert-hf.py:11-14), GQA attention, SwiGLU
(or GELU·up when hidden_act = 0), final norm, vocab projection. With `q80=True` every matmul input
is rounded through Q80 exactly like the Q40/Q80 runtime path.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from ..utils.mfile import ModelSpec, read_model


def rope_table(spec: ModelSpec, seq_len: int) -> torch.Tensor:
    hs = spec.head_size
    half = hs // 2
    freqs = []
    scale = spec.rope_scaling_factor not in (None, 1)
    for i in range(half):
        f = 1.0 / (spec.rope_theta ** (2 * i / hs))
        if scale:
            orig = spec.rope_scaling_orig_max_seq_len
            lo, hi = spec.rope_scaling_low_freq_factor, spec.rope_scaling_high_freq_factory
            wave = 2 * math.pi / f
            if wave < orig / hi:
                pass
            elif wave > orig / lo:
                f = f / spec.rope_scaling_factor
            else:
                s = (orig / wave - lo) / (hi - lo)
                f = (1 - s) * f / spec.rope_scaling_factor + s * f
        freqs.append(f)
    fr = torch.tensor(freqs, dtype=torch.float64)
    pos = torch.arange(seq_len, dtype=torch.float64)[:, None]
    ang = pos * fr[None, :]
    return torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).float()  # [seq, half, 2]


def q80_round(x: torch.Tensor) -> torch.Tensor:
    """Quantize-dequantize through Q80 blocks along the last dim (d stored as f16)."""
    shp = x.shape
    g = x.reshape(-1, 32)
    amax = g.abs().amax(dim=1)
    d = amax / 127.0
    idv = torch.where(d != 0, 1.0 / d, torch.zeros_like(d))
    q = torch.clamp(torch.round(g * idv[:, None]), -127, 127)
    return (q * d.half().float()[:, None]).reshape(shp)


class TorchLlama:
    def __init__(self, path: str, device: str = "cpu", q80: Optional[bool] = None):
        self.header, self.spec, w = read_model(path)
        self.q80 = (self.spec.weights_float_type == 2) if q80 is None else q80
        self.device = device
        self.w: Dict[tuple, torch.Tensor] = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in w.items()}
        self.rope = rope_table(self.spec, self.spec.max_seq_len).to(device)

    def _mm(self, W: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        if self.q80:
            x = q80_round(x)
        return x @ W.T

    def _norm(self, x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
        inv = 1.0 / torch.sqrt((x * x).mean(dim=-1, keepdim=True) + eps)
        return w.reshape(-1) * (inv * x)

    def _rope(self, x: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
        # x [T, n]; pairs (2i, 2i+1) use frequency index (2i % head_size) / 2
        T, n = x.shape
        hs = self.spec.head_size
        xp = x.reshape(T, n // 2, 2)
        fi = (torch.arange(n // 2, device=x.device) * 2 % hs) // 2
        cs = self.rope[pos][:, fi]  # [T, n/2, 2]
        c, s = cs[..., 0], cs[..., 1]
        o0 = xp[..., 0] * c - xp[..., 1] * s
        o1 = xp[..., 0] * s + xp[..., 1] * c
        return torch.stack([o0, o1], dim=-1).reshape(T, n)

    @torch.no_grad()
    def forward(self, tokens, start_pos: int = 0, kv: Optional[dict] = None) -> torch.Tensor:
        """Full causal forward of `tokens` at positions start_pos.. ; returns logits [T, vocab].
        `kv` (dict) carries the cache between calls for incremental decoding."""
        sp = self.spec
        w = self.w
        tok = torch.as_tensor(tokens, dtype=torch.long, device=self.device)
        T = tok.shape[0]
        pos = torch.arange(start_pos, start_pos + T, device=self.device)
        x = w[("embedding", -1)][tok]
        hs, kvmul = sp.head_size, sp.n_heads // sp.n_kv_heads
        if kv is None:
            kv = {}
        for l in range(sp.n_layers):
            xn = self._norm(x, w[("rms_att", l)])
            q = self._rope(self._mm(w[("q", l)], xn), pos)
            k = self._rope(self._mm(w[("k", l)], xn), pos)
            v = self._mm(w[("v", l)], xn)
            kc, vc = kv.get(l, (torch.zeros(0, sp.kv_dim, device=self.device), torch.zeros(0, sp.kv_dim, device=self.device)))
            kc = torch.cat([kc, k]) if kc.shape[0] == start_pos else torch.cat([kc[:start_pos], k])
            vc = torch.cat([vc, v]) if vc.shape[0] == start_pos else torch.cat([vc[:start_pos], v])
            kv[l] = (kc, vc)
            S = kc.shape[0]
            qh = q.reshape(T, sp.n_heads, hs).transpose(0, 1)                      # [H, T, hs]
            kh = kc.reshape(S, sp.n_kv_heads, hs).transpose(0, 1).repeat_interleave(kvmul, 0)
            vh = vc.reshape(S, sp.n_kv_heads, hs).transpose(0, 1).repeat_interleave(kvmul, 0)
            sc = qh @ kh.transpose(1, 2) / math.sqrt(hs)                          # [H, T, S]
            mask = torch.arange(S, device=self.device)[None, :] > pos[:, None]
            sc = sc.masked_fill(mask[None], float("-inf"))
            att = torch.softmax(sc, dim=-1) @ vh                                   # [H, T, hs]
            att = att.transpose(0, 1).reshape(T, sp.dim)
            x = x + self._mm(w[("wo", l)], att)
            xn = self._norm(x, w[("rms_ffn", l)])
            g = self._mm(w[("w1", l)], xn)
            u = self._mm(w[("w3", l)], xn)
            if sp.hidden_act == 0:
                a = 0.5 * g * (1 + torch.tanh(0.7978845608028654 * g * (1 + 0.044715 * g * g)))
            else:
                a = g * torch.sigmoid(g)
            x = x + self._mm(w[("w2", l)], a * u)
        xn = self._norm(x, w[("rms_final", -1)])
        return self._mm(w[("wcls", -1)], xn)
