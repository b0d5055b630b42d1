"""Runs the native unit-test binary (tests/cpp/unit_tests.cpp, built by `make`): host-side codecs,
shard plan, RoPE golden, CPU primitives, JSON, chat template and EOS detection in C++."""
import os
import subprocess

from conftest import REPO


def test_native_unit_tests():
    exe = os.path.join(REPO, "build", "unit_tests")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native unit tests passed" in r.stdout
