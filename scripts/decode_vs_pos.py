"""Batch-1 decode ms/token of the Llama-3.1-8B shapes at a sweep of start positions (32 steps each,
one engine sized to 4096 positions): shows the context-bucket steps of the decode schedule.
usage: python scripts/decode_vs_pos.py [f32|bf16]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402
from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES  # noqa: E402

kv_bf16 = len(sys.argv) > 1 and sys.argv[1] == "bf16"
C = dl.native()
h = dict(LLAMA_SHAPES["llama3_1_8b"], seq_len=4096, rope_theta=500000, weight_type=2)
e = C.HipEngine("", "q80", synthetic=h, max_seq_len=4096, n_slots=1, max_batch=32, kv_bf16=kv_bf16)
print("block", e.attn_block, flush=True)
for p in (64, 96, 120, 130, 160, 200, 250, 260, 400, 520, 1000, 2000, 3000):
    e.decode_greedy(4, [1], [p], [0])
    e.synchronize()
    t = time.perf_counter()
    e.decode_greedy(32, [1], [p + 4], [0])
    e.synchronize()
    print(f"pos {p + 4:5d}: {(time.perf_counter() - t) * 1000 / 32:.4f} ms/token", flush=True)
