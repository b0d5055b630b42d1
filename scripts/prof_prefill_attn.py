"""Prefill-attention kernel shapes for a rocprofv3 kernel trace (one launch each through the ops
harness; the trace gives the kernel's device time): 8B head layout, rows at a context offset.
usage: rocprofv3 --kernel-trace --stats -d out -- python3 scripts/prof_prefill_attn.py [f32|bf16]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llama_multiusers_amd import ops  # noqa: E402

kv_bf16 = len(sys.argv) > 1 and sys.argv[1] == "bf16"
g = torch.Generator().manual_seed(1)
for rows, p0, seq in ((32, 2048, 2112), (32, 64, 128), (256, 3072, 3328)):
    kv0 = 8 * 128
    k = torch.randn(1, seq, kv0, generator=g)
    v = torch.randn(1, seq, kv0, generator=g)
    q = torch.randn(rows, 32 * 128, generator=g)
    for _ in range(3):
        out = ops.attention(q, k, v, 32, 4, 128, list(range(p0, p0 + rows)), [0] * rows, kv_bf16, prefill=True)
    print(f"rows {rows} p0 {p0}: {float(out.abs().mean()):.4f}", flush=True)
