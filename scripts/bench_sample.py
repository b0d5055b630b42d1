"""Device sampler kernel on serving-shaped input: B rows x 128256 logits, temperature 0.8, top-p 0.9
(nucleus) or 1.0 (multinomial). Run under `rocprofv3 --kernel-trace --stats` for the kernel time.
  python scripts/bench_sample.py [B] [iters]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llama_multiusers_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rng = np.random.default_rng(0)
for name, scale, topp in (("flat-nucleus", 1.0, 0.9), ("peaked-nucleus", 8.0, 0.9), ("flat-multinomial", 1.0, 1.0)):
    x = (rng.standard_normal((B, 128256)) * scale).astype(np.float32)
    for _ in range(iters):
        ops.sample(x, [0.8] * B, [topp] * B, list(rng.random(B)))
    print(name, "done", flush=True)
