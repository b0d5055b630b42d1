"""Batch-1 decode ms/token of the 8B shapes at a short context (~70 positions) against the KV cache's
capacity and layout: contiguous [slot][kvHead][pos][hs] caches of 4096 and 131072 positions, and a
paged 131072-position cache (pages of 256 positions handed out on demand, so a short context
touches a few pages next to each other). usage: python scripts/probe_kv_capacity.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402
from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES  # noqa: E402

C = dl.native()
base = dict(LLAMA_SHAPES["llama3_1_8b"])
prompt = [(i * 7919 + 13) % 128000 for i in range(64)]
for name, cap, pages in [("contig 4096", 4096, 0), ("contig 131072", 131072, 0), ("paged 131072", 131072, 512),
                         ("contig 4096", 4096, 0), ("paged 131072", 131072, 512), ("contig 131072", 131072, 0)]:
    eng = C.HipEngine("", "q80", max_seq_len=cap, max_batch=32, n_slots=1, kv_bf16=True, synthetic=dict(base, seq_len=cap),
                      seed=1234, kv_pages=pages)
    for s in range(0, 64, 32):
        eng.forward_argmax(prompt[s:s + 32], list(range(s, s + 32)), [0] * 32)
    eng.decode_greedy(4, [prompt[-1]], [64], [0])
    t = time.perf_counter()
    dev_ms, _ = eng.decode_greedy(32, [prompt[-1]], [68], [0])
    wall = (time.perf_counter() - t) * 1000 / 32
    print(f"{name:14s}: {wall:.4f} ms/token wall, {dev_ms / 32:.4f} device", flush=True)
    del eng
