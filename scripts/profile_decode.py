"""Decode-step profiling helper: per-kernel-class eager breakdown + graph-replayed decode steps
(run under `rocprofv3 --kernel-trace --stats` for per-kernel device time)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3_1_8b")
ap.add_argument("--steps", type=int, default=32)
ap.add_argument("--layers", type=int, default=0)
ap.add_argument("--batch", type=int, default=1)
args = ap.parse_args()

import distributed_llama_multiusers_amd as dl
from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES

C = dl.native()
shape = dict(LLAMA_SHAPES[args.model])
if args.layers:
    shape["n_layers"] = args.layers
h = dict(shape, seq_len=1024, rope_theta=500000, weight_type=2)
eng = C.HipEngine("", "q80", synthetic=h, max_seq_len=1024, n_slots=args.batch, max_batch=max(32, args.batch))
B = args.batch
toks, pos, slots = [1] * B, [0] * B, list(range(B))
eng.forward(toks, pos, slots)
eng.profile_forward(toks, [1] * B, slots)
eng.decode_greedy(8, toks, [2] * B, slots)
t = time.perf_counter()
ms, _ = eng.decode_greedy(args.steps, toks, [10] * B, slots)
wall = (time.perf_counter() - t) * 1000
print(f"decode {args.model} batch {B}: {ms / args.steps:.4f} ms/step device, {wall / args.steps:.4f} ms/step wall")
