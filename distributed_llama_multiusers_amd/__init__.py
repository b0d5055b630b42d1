"""MI355X-native distributed Llama inference engine.

Capabilities of LatadosUnited/distributed-llama-MultiUsers (dllama inference|chat|worker,
dllama-api, `.m`/`.t` formats, Q40/Q80 + f32 numerics, 1-D tensor parallelism), rebuilt for
AMD Instinct MI355X: C++ runtime + hand-written gfx950 HIP kernels + RCCL over xGMI.
The native core lives in `libdllama.so`; `_C` is its pybind11 module.
"""
from __future__ import annotations

import os

__version__ = "0.1.0"

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)


def native():
    """Import the native module. torch is imported first so the process shares torch's HIP
    runtime (libamdhip64.so.7 / librccl.so.1 are resolved by soname to torch's copies)."""
    import torch  # noqa: F401  (runtime sharing, see docstring)
    from . import _C
    return _C
