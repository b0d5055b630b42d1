"""Same bytes, two layouts: TP1 8B heads at B=1 (8 KV heads interleaved in each 2 KB key row: a
workgroup reads 256-B slices 2 KB apart) vs 1 KV head at B=8 (each row's keys contiguous: a
workgroup reads one 64 KB range); both 256 workgroups x 128 KB at pos 8000."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_llama_multiusers_amd as dl  # noqa: E402

C = dl.native()
for nh, kvm, B in ((32, 4, 1), (4, 4, 8), (32, 4, 2), (4, 4, 16)):
    us = C.bench_attention(nh, kvm, 128, 8192, 8000, B, 8, 100)
    print(f"heads {nh:2d} kv heads {nh // kvm} B {B:2d}: {us:7.2f} us", flush=True)
