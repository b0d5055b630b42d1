#!/usr/bin/env python3
"""Headline benchmark: Llama-3.1-8B Q40 weights / Q80 activations, tensor-parallel over N MI355X
GPUs (one process per GPU; per-layer partial sums exchanged over xGMI inside the producing GEMVs).

Metric and config are the ones BASELINE.json names: "avg eval+pred ms/token" (reference:
`dllama inference` Evaluation / Prediction summary lines, src/dllama.cpp:98-113). Weights are
random-init on device with the real Llama-3.1-8B shapes (no network for checkpoints).
* eval = prompt evaluation, chunks of 32 rows per forward (the reference's nBatches), timed
  between barrier + device syncs;
* pred = single-stream decode; one timed "step" = one full decode token (embedding -> 32 layers ->
  logits -> argmax, the token fed back on device), K steps between barrier + device syncs;
* value = B * 1000 / ((eval_ms_per_token + pred_ms_per_token) / 2), the named metric; the decode-only
  rate is reported as config.pred_tokens_per_s.
The KV cache is f32, the reference's precision (src/llm.cpp:197-198, nn/nn-core.cpp:198-205), for
the headline and every extra point (`--kv f32`, default); the same eval + pred with a bf16 cache is
reported next to it (config.bf16_kv_*), never as `value`.
The engine is sized to --max-seq-len positions (default 4096, the reference run script's
`--max-seq-len 4096`); attention launches follow the context actually reached (context buckets),
not the capacity. Extra points in `config`: decode at position >= 4096 (long_ctx_pred_ms_per_token),
the same short-context decode on an engine sized to the model's full 131072-position context
(cap131072_pred_ms_per_token) and, on one GPU, the product path through
`build/dllama inference --synthetic llama3_1_8b` (cli_*: per-token host round trips included).

    python bench.py --gpus 1 --steps 128 --warmup 16
    python bench.py --gpus 8 --steps 128 --warmup 16        # launches its own 8 ranks
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 128 --warmup 16

Multi-GPU: one process per GPU. Started without a launcher (no WORLD_SIZE) and --gpus N > 1, the
parent spawns the N ranks itself (before touching any GPU), relays rank 0's JSON line and fails if
any rank fails - the reference's root drives its workers the same way (src/app.cpp:233-312).
`n_gpus` is the number of distinct devices the ranks ran on: DL_BENCH_SAME_GPU=1 rehearses N ranks on
one GPU, labelled "same_gpu_rehearsal": true with n_gpus 1 and no vs_baseline.
TP partial sums default to the reference's wire format, Q80 blocks (syncType = bufferFloatType,
src/app.cpp:81, llm.cpp:150); the exact f32 exchange is reported next to it (tp_f32_*).
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


def _cli_point(local: int, prompt_tokens: int, steps: int, max_seq: int, kv: str) -> dict:
    """Product path on one GPU: `dllama inference --synthetic llama3_1_8b` with greedy sampling
    (per forward: H2D inputs, graph replay, D2H token, host sync), parsed from the reference's
    Evaluation / Prediction summary lines (src/dllama.cpp:98-113)."""
    import re
    import subprocess
    import tempfile
    from distributed_llama_multiusers_amd.models.synthetic import make_tokenizer
    exe = os.path.join(REPO, "build", "dllama")
    if not os.path.exists(exe):
        return {"cli_error": "build/dllama missing"}
    with tempfile.TemporaryDirectory() as d:
        tok = os.path.join(d, "llama3_synth.t")
        make_tokenizer(tok, 128256)
        # ~1 token per character of the synthetic tokenizer's byte fallback
        prompt = ("The quick brown fox jumps over the lazy dog " * 8)[:prompt_tokens]
        cmd = [exe, "inference", "--synthetic", "llama3_1_8b", "--tokenizer", tok, "--prompt", prompt, "--steps",
               str(prompt_tokens + steps), "--temperature", "0", "--gpu-index", str(local), "--max-seq-len",
               str(max_seq), "--buffer-float-type", "q80", "--kv-dtype", kv, "--log-level", "0"]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        except subprocess.TimeoutExpired:
            return {"cli_error": "timeout"}
    out = r.stdout
    m = re.findall(r"tokens/s:\s*([\d.]+)\s*\(([\d.]+) ms/tok\)", out)
    if r.returncode != 0 or len(m) < 2:
        return {"cli_error": (out + r.stderr)[-300:]}
    return {"cli_eval_ms_per_token": float(m[0][1]), "cli_pred_ms_per_token": float(m[1][1]),
            "cli_avg_tokens_per_s": round(1000.0 / ((float(m[0][1]) + float(m[1][1])) / 2), 2)}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n: int) -> int:
    """--gpus N without a launcher: start N ranks of this script (one per GPU, LOCAL_RANK = GPU
    ordinal), relay rank 0's JSON line, fail if any rank fails. Runs before anything in this
    process touches a GPU (torch.cuda.device_count() only counts devices on this image)."""
    import subprocess
    import tempfile
    import torch
    same = os.environ.get("DL_BENCH_SAME_GPU") == "1"
    ndev = torch.cuda.device_count()
    if not same and ndev < n:
        print(f"bench.py: --gpus {n} but only {ndev} GPU(s) visible; set DL_BENCH_SAME_GPU=1 to rehearse "
              f"{n} ranks on one GPU (not a scaling point)", file=sys.stderr)
        return 2
    port = _free_port()
    out = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=out if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        alive = set(range(n))
        while alive:
            for r in list(alive):
                c = procs[r].poll()
                if c is None:
                    continue
                alive.discard(r)
                if c != 0 and rc == 0:
                    rc = c
                    print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                    for q in alive:
                        procs[q].terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    out.seek(0)
    lines = [l for l in out.read().splitlines() if l.startswith("{")]
    if rc == 0 and lines:
        print(lines[-1], flush=True)
    return rc if rc else (0 if lines else 1)


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
    ap.add_argument("--sync-type", default=os.environ.get("DL_SYNC_TYPE", "q80"), choices=["f32", "q80"],
                    help="TP partial-sum exchange: q80 (the reference's ZQ wire format, default) or f32 (exact)")
    ap.add_argument("--max-seq-len", type=int, default=4096,
                    help="engine context capacity (KV cache positions) of the headline engine")
    ap.add_argument("--no-cap128k", action="store_true", help="skip the 131072-capacity decode point")
    ap.add_argument("--long-ctx", type=int, default=4096, help="position of the long-context decode point (0: off)")
    ap.add_argument("--no-cli", action="store_true", help="skip the dllama CLI product-path point (1 GPU)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv", default="f32", choices=["f32", "bf16"],
                    help="KV-cache dtype of the headline and the extra points (f32: the reference's)")
    ap.add_argument("--no-altkv", action="store_true",
                    help="skip the eval + pred point with the other KV-cache dtype (bf16 next to an f32 headline)")
    ap.add_argument("--no-f32kv", dest="no_altkv", action="store_true", help=argparse.SUPPRESS)  # round-5 name
    ap.add_argument("--no-prefill4k", action="store_true", help="skip the 4096-token prompt-eval point")
    ap.add_argument("--tp-rank-compute", default="2,4,8",
                    help="1 GPU: TP degrees whose rank-0 shard is timed with the exchange removed "
                         "(compute-only comm; '' = off)")
    ap.add_argument("--prefill-chunk", type=int, default=1024,
                    help="rows per forward of the second 4096-token prompt point (the first uses the reference's 32)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _launch_ranks(args.gpus)

    import torch
    import distributed_llama_multiusers_amd as dl
    C = dl.native()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    same_gpu = world > 1 and os.environ.get("DL_BENCH_SAME_GPU") == "1"
    if same_gpu:  # rehearsal of the multi-rank path on one GPU (not a scaling point)
        local = 0
        # ranks sharing one GPU: with 256+ prompt rows per forward a rank's kernels spinning on a
        # peer (argmax winners, all-reduce flags) can keep that peer's kernels from being
        # dispatched until the wait gives up, so the rehearsal keeps to the 32-row prompt chunks
        args.prefill_chunk = 32
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    uid = None
    comm = None
    max_batch = max(32, args.batch)
    comm_kind = os.environ.get("DL_TP_COMM", "xgmi")
    torch.cuda.set_device(local)
    hdr = C.load_header(args.model) if args.model else dict(
        LLAMA31_8B, **__import__("distributed_llama_multiusers_amd.models.synthetic",
                                 fromlist=["LLAMA_SHAPES"]).LLAMA_SHAPES[args.shape])
    if world > 1:
        import torch.distributed as tdist
        dist = tdist
        # control plane only (barriers, timing max, IPC handle / RCCL id exchange); the data plane
        # is the engine's own device communicator
        dist.init_process_group("gloo")
        from distributed_llama_multiusers_amd.parallel import init_device_comm
        vocab0 = -(-hdr["vocab_size"] // world)
        # largest single message: a batch's logits slices (host logits) or a --prefill-chunk forward's
        # [chunk][dim] partial sums (greedy rows exchange 2 floats per row)
        max_floats = max(max_batch * max(hdr["dim"], vocab0), args.prefill_chunk * hdr["dim"])
        comm, uid, comm_kind = init_device_comm(C, dist, rank, world, max_floats, local, comm_kind)

    long_pos = args.long_ctx if args.long_ctx > 0 else 0
    seq_len = max(args.max_seq_len, args.prompt + args.warmup + args.steps + 8)
    shape = LLAMA31_8B
    if args.shape != "llama3_1_8b":
        from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES
        shape = dict(LLAMA31_8B, **LLAMA_SHAPES[args.shape])

    kv_bf16_main = args.kv == "bf16"

    def make_engine(max_seq=seq_len, kv_bf16=None, sync=None):
        if kv_bf16 is None:
            kv_bf16 = kv_bf16_main
        synthetic = None if args.model else dict(shape, seq_len=max_seq)
        e = C.HipEngine(args.model, "q80", max_seq_len=max_seq, max_batch=max_batch, n_slots=args.batch,
                        kv_bf16=kv_bf16,
                        gpu_index=local, use_graphs=not args.no_graphs, synthetic=synthetic, seed=1234, rank=rank,
                        world=world, uid=uid, comm=comm, sync_type=sync or args.sync_type)
        if dist is not None:  # ranks build their engines seconds apart; start the next phase together
            dist.barrier()
        return e

    t0 = time.time()
    eng = make_engine()
    load_s = time.time() - t0
    B = args.batch

    def barrier():
        if dist is not None:
            dist.barrier()

    prompt = [(i * 7919 + 13) % 128000 for i in range(args.prompt)]
    if world > 1:
        # pre-flight of the exact timed path (captured graphs, fused exchange, distributed argmax):
        # every rank must decode the same tokens without a timed-out peer wait; otherwise every rank
        # agrees to rebuild on RCCL (no rank ever waits on a peer using another data plane)
        import numpy as np
        ok = True
        try:
            eng.forward_argmax(prompt[:8], list(range(8)), [0] * 8)
            _, toks = eng.decode_greedy(4, [prompt[7]], [8], [0])
            if comm is not None and comm.timed_out():
                raise RuntimeError("a peer wait timed out")
        except Exception as e:  # noqa: BLE001 - reported, then the agreed fallback
            print(f"rank {rank}: pre-flight failed: {e}", file=sys.stderr)
            ok, toks = False, [-1] * 4
        got = [None] * world
        dist.all_gather_object(got, list(toks))
        flag = torch.tensor([1 if ok and all(g == got[0] for g in got) else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag[0]):
            if rank == 0:
                print(f"pre-flight over {comm_kind} failed ({got}); rebuilding on rccl", file=sys.stderr)
            del eng
            comm, comm_kind = None, "rccl"
            obj = [C.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            uid = obj[0]
            eng = make_engine()

    pos0 = len(prompt)
    tokens = [prompt[-1]] * B

    def eval_pred(e, steps, warmup):
        """eval: prefill the prompt (chunks of 32 rows per forward, like the reference nBatches=32);
        two untimed chunks first (the engine runs a row count eagerly on first use and captures its
        graph on the second) so the timed chunks replay the batch-32 graph. pred: `warmup` untimed
        decode steps, then `steps` timed ones between barrier + device syncs."""
        if len(prompt) >= 32:
            for _ in range(2):
                for b in range(B):
                    e.forward_argmax(prompt[:32], list(range(32)), [b] * 32)
        torch.cuda.synchronize()
        barrier()
        te = time.perf_counter()
        for s in range(0, len(prompt), 32):
            chunk = prompt[s:s + 32]
            for b in range(B):
                e.forward_argmax(chunk, list(range(s, s + len(chunk))), [b] * len(chunk))
        torch.cuda.synchronize()
        ev_s = time.perf_counter() - te
        barrier()
        if warmup > 0:
            e.decode_greedy(warmup, tokens, [pos0] * B, list(range(B)))
        p1 = pos0 + warmup
        barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        dms, _ = e.decode_greedy(steps, tokens, [p1] * B, list(range(B)))
        torch.cuda.synchronize()
        el = time.perf_counter() - t_start
        barrier()
        return ev_s, el, dms

    eval_s, elapsed, dev_ms = eval_pred(eng, args.steps, args.warmup)
    tp_fused = bool(eng.tp_fused) if world > 1 else None  # after the first forward's self-test

    long_ms = None
    if long_pos:  # decode at a long context, own engine sized for it (KV rows it never wrote are
        del eng   # zeros: same work, same time)
        eng = make_engine(max(seq_len, long_pos + 24))
        eng.decode_greedy(4, tokens, [long_pos] * B, list(range(B)))
        barrier()
        torch.cuda.synchronize()
        tl = time.perf_counter()
        eng.decode_greedy(16, tokens, [long_pos + 4] * B, list(range(B)))
        torch.cuda.synchronize()
        long_ms = (time.perf_counter() - tl) * 1000.0 / 16
        barrier()

    cap_ms = None
    if not args.no_cap128k and not args.model:  # same short-context decode, full 131072-position capacity
        del eng
        eng = make_engine(131072)
        eng.decode_greedy(4, tokens, [pos0] * B, list(range(B)))
        barrier()
        torch.cuda.synchronize()
        tc = time.perf_counter()
        eng.decode_greedy(32, tokens, [pos0 + 4] * B, list(range(B)))
        torch.cuda.synchronize()
        cap_ms = (time.perf_counter() - tc) * 1000.0 / 32
        barrier()

    alt_eval_s = alt_pred_s = None
    alt_kv = "bf16" if args.kv == "f32" else "f32"
    alt_steps = max(16, min(args.steps, 64))
    if not args.no_altkv:  # the same eval + pred with the other KV-cache dtype (never the `value`)
        del eng
        eng = make_engine(kv_bf16=not kv_bf16_main)
        alt_eval_s, alt_pred_s, _ = eval_pred(eng, alt_steps, 4)

    tpf32_ms = None
    if world > 1 and args.sync_type != "f32":  # the exact f32 exchange next to the Q80 wire format
        del eng
        eng = make_engine(max(seq_len, pos0 + 48), sync="f32")
        eng.decode_greedy(4, tokens, [pos0] * B, list(range(B)))
        barrier()
        torch.cuda.synchronize()
        tt = time.perf_counter()
        eng.decode_greedy(32, tokens, [pos0 + 4] * B, list(range(B)))
        torch.cuda.synchronize()
        tpf32_ms = (time.perf_counter() - tt) * 1000.0 / 32
        barrier()

    p4k_ms = p4k_big_ms = None
    if not args.no_prefill4k:  # a 4096-token prompt evaluated in 32-token chunks (attention grows with it)
        del eng
        eng = make_engine(max(seq_len, 4096 + 8))
        p4k = [(i * 7919 + 13) % 128000 for i in range(4096)]

        def prefill(e, chunk):
            for _ in range(2):  # eager first use, then graph capture - both outside the timing
                e.forward_argmax(p4k[:chunk], list(range(chunk)), [0] * chunk)
            barrier()
            torch.cuda.synchronize()
            tp4 = time.perf_counter()
            for s0 in range(0, 4096, chunk):
                e.forward_argmax(p4k[s0:s0 + chunk], list(range(s0, s0 + chunk)), [0] * chunk)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - tp4) * 1000.0 / 4096
            barrier()
            return ms

        p4k_ms = prefill(eng, 32)
        # the same prompt in chunks of `--prefill-chunk` rows (dllama --max-batch / the API's prefill):
        # one wide-GEMM launch per matrix covers every 128-token tile of the chunk
        if args.prefill_chunk > 32:
            del eng
            sl = max(seq_len, 4096 + 8)
            eng = C.HipEngine(args.model, "q80", max_seq_len=sl, max_batch=args.prefill_chunk, n_slots=1,
                              kv_bf16=kv_bf16_main, gpu_index=local, use_graphs=not args.no_graphs,
                              synthetic=None if args.model else dict(shape, seq_len=sl), seed=1234, rank=rank,
                              world=world, uid=uid, comm=comm, sync_type=args.sync_type)
            barrier()
            p4k_big_ms = prefill(eng, args.prefill_chunk)

    if dist is not None:
        t = torch.tensor([elapsed, eval_s, long_ms or 0.0, alt_pred_s or 0.0, p4k_ms or 0.0, tpf32_ms or 0.0,
                          p4k_big_ms or 0.0, cap_ms or 0.0, alt_eval_s or 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, eval_s = float(t[0]), float(t[1])
        long_ms = float(t[2]) if long_ms is not None else None
        alt_pred_s = float(t[3]) if alt_pred_s is not None else None
        alt_eval_s = float(t[8]) if alt_eval_s is not None else None
        p4k_ms = float(t[4]) if p4k_ms is not None else None
        tpf32_ms = float(t[5]) if tpf32_ms is not None else None
        p4k_big_ms = float(t[6]) if p4k_big_ms is not None else None
        cap_ms = float(t[7]) if cap_ms is not None else None

    ms_per_step = elapsed * 1000.0 / args.steps
    pred_ms_tok = ms_per_step / B
    eval_ms_tok = eval_s * 1000.0 / max(1, len(prompt)) / B
    avg_ms_tok = (eval_ms_tok + pred_ms_tok) / 2 if prompt else pred_ms_tok
    tok_s = 1000.0 / avg_ms_tok
    alt = {}
    if alt_pred_s is not None:
        a_eval = alt_eval_s * 1000.0 / max(1, len(prompt)) / B
        a_pred = alt_pred_s * 1000.0 / alt_steps / B
        a_avg = (a_eval + a_pred) / 2 if prompt else a_pred
        alt = {f"{alt_kv}_kv_value": round(1000.0 / a_avg, 3), f"{alt_kv}_kv_eval_ms_per_token": round(a_eval, 4),
               f"{alt_kv}_kv_pred_ms_per_token": round(a_pred, 4)}
    # the published baselines are per model family: 7B/8B at 1/2/4/8 devices, 70B at 8 devices
    base = (BASELINE_MS.get(world) if args.shape == "llama3_1_8b" and not args.model
            else BASELINE_MS_70B.get(world) if args.shape == "llama3_3_70b" and not args.model else None)
    if same_gpu:
        base = None  # a rehearsal on one device is not a point of the scaling curve
    # a TP-N rank's own work on one GPU: rank 0's shard shapes and kernels (fused exchange in
    # loopback, separate collectives no-ops), i.e. the per-token floor of a TP-N rank without sync
    tp_rank = {}
    if world == 1 and args.tp_rank_compute and not args.model:
        del eng
        for n in [int(v) for v in args.tp_rank_compute.split(",") if v]:
            e = C.HipEngine("", "q80", max_seq_len=seq_len, max_batch=max_batch, n_slots=B, kv_bf16=kv_bf16_main,
                            gpu_index=local, use_graphs=not args.no_graphs, synthetic=dict(shape, seq_len=seq_len),
                            seed=1234, rank=0, world=n, comm=C.ComputeOnlyComm(0, n, local),
                            sync_type=args.sync_type)
            for _ in range(2):
                e.forward_argmax(prompt[:32], list(range(32)), [0] * 32)
            torch.cuda.synchronize()
            tq = time.perf_counter()
            for s0 in range(0, len(prompt) - 31, 32):
                e.forward_argmax(prompt[s0:s0 + 32], list(range(s0, s0 + 32)), [0] * 32)
            torch.cuda.synchronize()
            ev = (time.perf_counter() - tq) * 1000.0 / max(32, len(prompt) // 32 * 32)
            e.decode_greedy(8, tokens, [pos0] * B, list(range(B)))
            torch.cuda.synchronize()
            tq = time.perf_counter()
            e.decode_greedy(64, tokens, [pos0 + 8] * B, list(range(B)))
            torch.cuda.synchronize()
            tp_rank[f"tp{n}_rank_compute_ms_per_token"] = round((time.perf_counter() - tq) * 1000.0 / 64 / B, 4)
            tp_rank[f"tp{n}_rank_compute_eval_ms_per_token"] = round(ev / B, 4)
            del e
        eng = None
    cli = {}
    if world == 1 and not args.no_cli and args.shape == "llama3_1_8b" and not args.model:
        eng = None
        cli = _cli_point(local, min(args.prompt, 64), min(args.steps, 64), seq_len, args.kv)
    result = {
        "metric": METRIC,
        "value": round(tok_s, 3),
        "unit": "tokens/s",
        "n_gpus": 1 if same_gpu else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(tok_s / (1000.0 / base), 2) if base else None,
        "dtype": f"q40-weights/q80-activations/{args.kv}-kv-cache (f32 accumulate)",
        "data": (f"synthetic: random-init {args.shape} weights on device, synthetic prompt" if not args.model
                 else "model file weights, synthetic prompt"),
        "config": {
            "model": ({"llama3_1_8b": "Llama-3.1-8B"}.get(args.shape, args.shape) if not args.model
                      else os.path.basename(args.model)),
            "global_batch": B,
            "seq_len": seq_len,
            "prompt_tokens": args.prompt,
            "parallelism": f"tp{world}",
            "kv_cache": args.kv,
            "value_formula": "B*1000/((eval_ms_per_token+pred_ms_per_token)/2)",
            "eval_ms_per_token": round(eval_ms_tok, 4),
            "pred_ms_per_token": round(pred_ms_tok, 4),
            "pred_tokens_per_s": round(1000.0 * B / ms_per_step, 2),
            "device_ms_per_step": round(dev_ms / args.steps, 4),
            "long_ctx_pos": long_pos or None,
            "long_ctx_pred_ms_per_token": round(long_ms / B, 4) if long_ms is not None else None,
            "cap131072_pred_ms_per_token": round(cap_ms / B, 4) if cap_ms is not None else None,
            **alt,
            "prompt_4k_eval_ms_per_token": round(p4k_ms, 4) if p4k_ms is not None else None,
            "prompt_4k_chunk": args.prefill_chunk if p4k_big_ms is not None else None,
            "prompt_4k_eval_big_chunk_ms_per_token": round(p4k_big_ms, 4) if p4k_big_ms is not None else None,
            "load_s": round(load_s, 2),
            "hip_graphs": not args.no_graphs,
            "tp_ranks": world,
            "tp_comm": comm_kind if world > 1 else None,
            "tp_sync": args.sync_type if world > 1 else None,
            "tp_fused_exchange": tp_fused,
            "tp_f32_pred_ms_per_token": round(tpf32_ms / B, 4) if tpf32_ms is not None else None,
            **tp_rank,
            **cli,
        },
    }
    if same_gpu:
        result["same_gpu_rehearsal"] = True
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
