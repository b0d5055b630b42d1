"""Shared fixtures. GPU tests are marked `gpu`; everything else runs on CPU.

The native library is (re)built on demand with `make` (a no-op when up to date)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def _build():
    if os.environ.get("DL_SKIP_BUILD") == "1":
        return
    r = subprocess.run(["make", "-j8", os.environ.get("DL_MAKE_TARGET", "all")], cwd=REPO, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])


_build()


@pytest.fixture(scope="session")
def C():
    import distributed_llama_multiusers_amd as dl
    return dl.native()


@pytest.fixture(scope="session")
def assets(tmp_path_factory):
    """Tiny Q40 + F32 models and a tokenizer shared by the session."""
    from distributed_llama_multiusers_amd.models.synthetic import make_test_assets
    from distributed_llama_multiusers_amd.utils.mfile import FloatType
    d = str(tmp_path_factory.mktemp("assets"))
    q40 = make_test_assets(d, "tiny", FloatType.Q40, seq_len=128, seed=1)
    f32 = make_test_assets(d, "tiny", FloatType.F32, seq_len=128, seed=1)
    return {"dir": d, "q40": q40[0], "f32": f32[0], "tok": q40[1], "spec": q40[2]}


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
