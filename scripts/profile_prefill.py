"""Batched-forward profiling helper: per-class eager breakdown + repeated graph-replayed forwards of
`--tokens` rows (run under `rocprofv3 --kernel-trace --stats` for per-kernel device time)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3_1_8b")
ap.add_argument("--tokens", type=int, default=32)
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--kv", choices=["f32", "bf16"], default="f32")
ap.add_argument("--pos0", type=int, default=0, help="first position of the rows (earlier KV rows: zeros, same work)")
args = ap.parse_args()

import distributed_llama_multiusers_amd as dl
from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES

C = dl.native()
seq = max(1024, args.pos0 + args.tokens + 8)
h = dict(LLAMA_SHAPES[args.model], seq_len=seq, rope_theta=500000, weight_type=2)
eng = C.HipEngine("", "q80", synthetic=h, max_seq_len=seq, n_slots=1, max_batch=max(32, args.tokens),
                  kv_bf16=args.kv == "bf16")
n = args.tokens
toks = [(i * 31 + 7) % 1000 for i in range(n)]
pos = list(range(args.pos0, args.pos0 + n))
eng.forward_argmax(toks, pos, [0] * n)
eng.profile_forward(toks, pos, [0] * n)
t = time.perf_counter()
for r in range(args.reps):
    eng.forward_argmax(toks, pos, [0] * n)
eng.synchronize()
wall = (time.perf_counter() - t) * 1000 / args.reps
print(f"prefill {args.model} {n} tokens: {wall:.3f} ms per forward, {wall / n:.4f} ms/token")
