"""Timeline of one layer of the persistent decode engine (decode_engine.hip, PdeArgs::trace):
per-workgroup s_memrealtime stamps (10 ns) of the aux waves' phase events and the ring waves'
per-phase consumption window, summarized as median [min .. max] across workgroups, microseconds
from the layer's first stamp. usage: python scripts/trace_decode_engine.py [pos] [layer]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402

EVENTS = {0: "layer start", 1: "w2(l-1) arrived", 2: "qkv act staged", 3: "qkv rows done (ring)",
          4: "qkv published", 5: "attn: group arrived", 6: "attn: published", 7: "att arrived (all heads)",
          8: "wo act staged", 9: "wo rows done", 10: "wo published", 11: "wo arrived (all)",
          12: "w13 act staged", 13: "w13 rows done", 14: "h published", 15: "h arrived (all)",
          16: "w2 act staged", 17: "w2 rows done", 18: "w2 published",
          20: "ring qkv start", 21: "ring qkv end", 22: "ring wo start", 23: "ring wo end",
          24: "ring w13 start", 25: "ring w13 end", 26: "ring w2 start", 27: "ring w2 end"}


def main():
    pos = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    layer = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    C = dl.native()
    h = dict(dim=4096, hidden_dim=14336, n_layers=32, n_heads=32, n_kv_heads=8, vocab_size=128256, seq_len=4096,
             rope_theta=500000, weight_type=2)
    eng = C.HipEngine("", "q80", synthetic=h, max_seq_len=4096, gpu_index=0, max_batch=32)
    print("decode engine:", eng.decode_engine, flush=True)
    eng.decode_greedy(8, [7], [pos - 8], [0])
    for rep in range(3):
        t = np.array(eng.trace_decode_engine(7, pos, 0, layer), dtype=np.uint64).reshape(-1, 32)
    t0 = t[:, 0][t[:, 0] > 0].min()
    t = np.where((t >= t0) & (t < t0 + 10 ** 8), t, 0).astype(np.int64)  # drop unset / garbage stamps
    print(f"layer {layer}, pos {pos}, {t.shape[0]} workgroups; us from the first layer-start stamp")
    for k, name in EVENTS.items():
        v = t[:, k]
        v = v[v > 0]
        t0i = int(t0)
        if len(v) == 0:
            continue
        us = (v - t0i) / 100.0
        print(f"  {k:2d} {name:26s} {np.median(us):8.2f} [{us.min():7.2f} .. {us.max():7.2f}]  n={len(v)}")


if __name__ == "__main__":
    main()
