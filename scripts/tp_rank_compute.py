"""One TP-N rank's own decode work on one GPU: rank `--rank` of `--tp` with the exchange removed
(ComputeOnlyComm: fused exchange in loopback, separate collectives no-ops). Prints ms per token of
greedy decode (and of 32-row prompt chunks); run under rocprofv3 for the per-kernel split.
bench.py reports the same points as tp{N}_rank_compute_ms_per_token."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--shape", default="llama3_1_8b")
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--sync-type", default="q80")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv", default="bf16", choices=["bf16", "f32"], help="KV-cache dtype")
    ap.add_argument("--pos", type=int, default=64, help="decode position (context length) of the timed steps")
    args = ap.parse_args()
    import torch
    import distributed_llama_multiusers_amd as dl
    from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES
    from bench import LLAMA31_8B
    C = dl.native()
    torch.cuda.set_device(0)
    shape = dict(LLAMA31_8B, **LLAMA_SHAPES[args.shape])
    e = C.HipEngine("", "q80", max_seq_len=max(4096, args.pos + 128), max_batch=32, n_slots=1, kv_bf16=args.kv == "bf16", gpu_index=0,
                    use_graphs=not args.no_graphs, synthetic=dict(shape, seq_len=max(4096, args.pos + 128)), seed=1234, rank=args.rank,
                    **(dict(world=args.tp, comm=C.ComputeOnlyComm(args.rank, args.tp, 0)) if args.tp > 1 else {}),
                    sync_type=args.sync_type)
    prompt = [(i * 7919 + 13) % 128000 for i in range(64)]
    for _ in range(2):
        e.forward_argmax(prompt[:32], list(range(32)), [0] * 32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(0, 64, 32):
        e.forward_argmax(prompt[s:s + 32], list(range(s, s + 32)), [0] * 32)
    torch.cuda.synchronize()
    ev = (time.perf_counter() - t0) * 1000.0 / 64
    p0 = max(64, args.pos)
    e.decode_greedy(8, [prompt[-1]], [p0], [0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.decode_greedy(args.steps, [prompt[-1]], [p0 + 8], [0])
    torch.cuda.synchronize()
    pred = (time.perf_counter() - t0) * 1000.0 / args.steps
    print(f"tp{args.tp} rank {args.rank} ({args.shape}, {args.sync_type}, kv {args.kv}, pos {max(64, args.pos)}): pred {pred:.4f} ms/token, "
          f"eval {ev:.4f} ms/token, fused {bool(e.tp_fused)}, attn block {bool(e.attn_block)} "
          f"[{' '.join(k + '=' + v for k, v in os.environ.items() if k.startswith('DL_'))}]", flush=True)


if __name__ == "__main__":
    main()
