#!/usr/bin/env python3
"""Decode-attention micro-benchmark: microseconds per launch of the attention kernel (bf16 KV cache,
Q80 output) inside a hipGraph of back-to-back launches, for the Llama-3.1-8B head layout at each
tensor-parallel degree (heads and KV heads per rank shrink with TP).

    python scripts/bench_attn.py                # default sweep
    DL_ATTN_MFMA=0 python scripts/bench_attn.py # the VALU kernel at every length
    BATCHES=1,8,64 TPS=1 SHORT=1 DL_ATTN_GRID_MAX=1024 python scripts/bench_attn.py
    KV=f32 python scripts/bench_attn.py         # f32 cache (the reference's precision)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import distributed_llama_multiusers_amd as dl
    C = dl.native()
    copies = 32  # one KV cache per layer: a decode step revisits a layer's KV only every token
    iters = 200
    print(f"attention µs/launch (graph of {iters}, {copies} KV copies), KV={os.environ.get('KV', 'bf16')} "
          f"DL_ATTN_MFMA={os.environ.get('DL_ATTN_MFMA', '')} DL_ATTN_GRID_MAX={os.environ.get('DL_ATTN_GRID_MAX', '')}")
    batches = [int(b) for b in os.environ.get("BATCHES", "1,4").split(",")]
    tps = [int(t) for t in os.environ.get("TPS", "1,2,4,8").split(",")]
    points = ((256, 50), (256, 150), (2048, 1500), (8192, 8000)) if os.environ.get("SHORT") else \
        ((256, 150), (2048, 1500), (8192, 8000))
    for tp in tps:
        nh, kvm = 32 // tp, 4
        for seq, pos in points:
            for B in batches:
                us = C.bench_attention(nh, kvm, 128, seq, pos, B, copies, iters, kv_bf16=os.environ.get("KV") != "f32")
                print(f"tp{tp} heads {nh:2d} kvMul {kvm} seqLen {seq:5d} pos {pos:5d} B {B}: {us:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
