"""Real-file load path: write a full-size Llama-3.1-8B Q40 `.m` of random weights (streamed, not
materialised), then open it with the HIP engine (parallel pread -> tiled repack into pinned
staging -> async H2D) and report GB/s; then a few greedy decode steps as a sanity check.

  python scripts/bench_load.py [--path /tmp/dl_load_8b.m] [--keep] [--drop-cache]

The file sits in the page cache right after it is written, so this measures the warm-cache load
(the common case on a serving node restarting a model); --drop-cache uses posix_fadvise(DONTNEED)
to evict it first (a best effort: the kernel may keep pages another process maps)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default="/tmp/dl_load_8b.m")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--drop-cache", action="store_true")
    ap.add_argument("--seq-len", type=int, default=4096)
    args = ap.parse_args()
    from distributed_llama_multiusers_amd.utils.mfile import ModelSpec, FloatType, write_random_model
    spec = ModelSpec(dim=4096, hidden_dim=14336, n_layers=32, n_heads=32, n_kv_heads=8, vocab_size=128256,
                     max_seq_len=131072, weights_float_type=FloatType.Q40, rope_theta=500000,
                     rope_scaling_factor=8, rope_scaling_low_freq_factor=1, rope_scaling_high_freq_factory=4,
                     rope_scaling_orig_max_seq_len=8192, rope_type=2)
    t0 = time.time()
    if not os.path.exists(args.path):
        size = write_random_model(args.path, spec, seed=3)
        print(f"wrote {size / 1e9:.2f} GB in {time.time() - t0:.1f} s", flush=True)
    size = os.path.getsize(args.path)
    if args.drop_cache:
        fd = os.open(args.path, os.O_RDONLY)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        os.close(fd)
    import distributed_llama_multiusers_amd as dl
    C = dl.native()
    try:
        t0 = time.time()
        e = C.HipEngine(model=args.path, max_seq_len=args.seq_len, max_batch=8, n_slots=1)
        wall = time.time() - t0
        ls = e.load_stats
        toks = e.decode_greedy(16, [1], [0], [0])[1]
        out = {"file_gb": round(size / 1e9, 3), "read_gb": round(ls["file_bytes"] / 1e9, 3),
               "engine_load_s": round(ls["ms"] / 1e3, 3), "wall_s": round(wall, 3),
               "load_gb_per_s": round(ls["file_bytes"] / 1e6 / max(ls["ms"], 1e-3), 2),
               "device_gb": round(ls["device_bytes"] / 1e9, 3), "drop_cache": args.drop_cache}
        print(json.dumps(out), flush=True)
        if toks is not None:
            print("decode ok:", str(toks)[:120], flush=True)
    finally:
        if not args.keep:
            os.remove(args.path)


if __name__ == "__main__":
    main()
