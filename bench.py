#!/usr/bin/env python3
"""Headline benchmark: Llama-3.1-8B Q40 weights / Q80 activations, single-stream decode
(tokens/s = 1000 / ms-per-token), tensor-parallel over N MI355X GPUs (one process per GPU,
RCCL over xGMI for the per-layer all-reduces).

Metric and config are the ones BASELINE.json names (reference: `dllama inference` Evaluation /
Prediction summary lines, src/dllama.cpp:98-113). Weights are random-init on device with the real
Llama-3.1-8B shapes (no network for checkpoints). One timed "step" = one full decode token:
embedding -> 32 layers -> logits -> argmax, with the sampled token fed back on device.

    python bench.py --gpus 1 --steps 128 --warmup 16
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 128 --warmup 16
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_MS = {1: 1312.50, 2: 793.69, 4: 494.00, 8: 588.19}  # BASELINE.md (Llama 2 7B, RPi 4B cluster)
BASELINE_MS_70B = {8: 4842.81}  # BASELINE.md (Llama 2 70B, 8x RPi 4B)
METRIC = "avg eval+pred ms/token (= tokens/sec) for Llama-3.1-8B Q40 at 1/2/4/8 MI355X"

LLAMA31_8B = dict(dim=4096, hidden_dim=14336, n_layers=32, n_heads=32, n_kv_heads=8, vocab_size=128256,
                  rope_theta=500000, rope_scaling_factor=8.0, rope_scaling_low_freq_factor=1.0,
                  rope_scaling_high_freq_factor=4.0, rope_scaling_orig_max_seq_len=8192, rope_type=2,
                  weight_type=2, hidden_act=1)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--prompt", type=int, default=64, help="prompt tokens prefilled before decoding (eval)")
    ap.add_argument("--batch", type=int, default=1, help="concurrent sequences decoded together")
    ap.add_argument("--model", default="", help="optional .m file instead of synthetic 8B weights")
    ap.add_argument("--shape", default="llama3_1_8b",
                    help="synthetic shape (models/synthetic.py LLAMA_SHAPES); the headline metric is llama3_1_8b")
    ap.add_argument("--no-graphs", action="store_true")
    args = ap.parse_args()

    import torch
    import distributed_llama_multiusers_amd as dl
    C = dl.native()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DL_BENCH_SAME_GPU") == "1":  # rehearsal of the multi-rank path on one GPU
        local = 0
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    uid = None
    comm = None
    max_batch = max(32, args.batch)
    comm_kind = os.environ.get("DL_TP_COMM", "xgmi")
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as tdist
        dist = tdist
        # control plane only (barriers, timing max, IPC handle / RCCL id exchange); the data plane
        # is the engine's own device communicator
        dist.init_process_group("gloo")
        from distributed_llama_multiusers_amd.parallel import init_device_comm
        hdr = C.load_header(args.model) if args.model else dict(
            LLAMA31_8B, **__import__("distributed_llama_multiusers_amd.models.synthetic",
                                     fromlist=["LLAMA_SHAPES"]).LLAMA_SHAPES[args.shape])
        vocab0 = -(-hdr["vocab_size"] // world)
        comm, uid, comm_kind = init_device_comm(C, dist, rank, world, max_batch * max(hdr["dim"], vocab0), local,
                                                comm_kind)

    seq_len = args.prompt + args.warmup + args.steps + 8
    shape = LLAMA31_8B
    if args.shape != "llama3_1_8b":
        from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES
        shape = dict(LLAMA31_8B, **LLAMA_SHAPES[args.shape])
    synthetic = None if args.model else dict(shape, seq_len=seq_len)
    t0 = time.time()
    eng = C.HipEngine(args.model, "q80", max_seq_len=seq_len, max_batch=max_batch, n_slots=args.batch,
                      gpu_index=local, use_graphs=not args.no_graphs, synthetic=synthetic, seed=1234, rank=rank,
                      world=world, uid=uid, comm=comm)
    load_s = time.time() - t0
    B = args.batch

    def barrier():
        if dist is not None:
            dist.barrier()

    # eval: prefill the prompt (chunks of 32 rows per forward, like the reference nBatches=32);
    # one untimed chunk first so the batch-32 graph is captured outside the timed region
    prompt = [(i * 7919 + 13) % 128000 for i in range(args.prompt)]
    if len(prompt) >= 32:
        for b in range(B):
            eng.forward_argmax(prompt[:32], list(range(32)), [b] * 32)
    torch.cuda.synchronize()
    barrier()
    te = time.perf_counter()
    for s in range(0, len(prompt), 32):
        chunk = prompt[s:s + 32]
        for b in range(B):
            eng.forward_argmax(chunk, list(range(s, s + len(chunk))), [b] * len(chunk))
    torch.cuda.synchronize()
    eval_ms = (time.perf_counter() - te) * 1000.0
    barrier()

    pos0 = len(prompt)
    tokens = [prompt[-1]] * B
    if args.warmup > 0:
        eng.decode_greedy(args.warmup, tokens, [pos0] * B, list(range(B)))
    pos1 = pos0 + args.warmup

    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    dev_ms, out = eng.decode_greedy(args.steps, tokens, [pos1] * B, list(range(B)))
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    barrier()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])

    ms_per_step = elapsed * 1000.0 / args.steps
    tok_s = B * 1000.0 / ms_per_step
    # the published baselines are per model family: 7B/8B at 1/2/4/8 devices, 70B at 8 devices
    base = (BASELINE_MS.get(world) if args.shape == "llama3_1_8b" and not args.model
            else BASELINE_MS_70B.get(world) if args.shape == "llama3_3_70b" and not args.model else None)
    result = {
        "metric": METRIC,
        "value": round(tok_s, 3),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(tok_s / (1000.0 / base), 2) if base else None,
        "dtype": "q40-weights/q80-activations (f32 accumulate)",
        "data": (f"synthetic: random-init {args.shape} weights on device, synthetic prompt" if not args.model
                 else "model file weights, synthetic prompt"),
        "config": {
            "model": ({"llama3_1_8b": "Llama-3.1-8B"}.get(args.shape, args.shape) if not args.model
                      else os.path.basename(args.model)),
            "global_batch": B,
            "seq_len": seq_len,
            "prompt_tokens": args.prompt,
            "parallelism": f"tp{world}",
            "kv_cache": "bf16",
            "eval_ms_per_token": round(eval_ms / max(1, len(prompt)) / B, 4),
            "device_ms_per_step": round(dev_ms / args.steps, 4),
            "load_s": round(load_s, 2),
            "hip_graphs": not args.no_graphs,
            "tp_comm": comm_kind if world > 1 else None,
        },
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
