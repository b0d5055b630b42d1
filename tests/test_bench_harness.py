"""bench.py's multi-GPU contract (the driver's scaling runs depend on it): `--gpus N` without a
launcher spawns its own N ranks, refuses to fake a scaling point when fewer GPUs are visible, and a
same-GPU rehearsal is labelled as one (n_gpus 1, same_gpu_rehearsal, no vs_baseline)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, gpu_available

BENCH = os.path.join(REPO, "bench.py")


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU refusal path")
def test_gpus_n_without_enough_devices_refuses():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("DL_BENCH_SAME_GPU", None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "GPU(s) visible" in r.stderr and "DL_BENCH_SAME_GPU" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]  # no result line at all


@pytest.mark.gpu
def test_same_gpu_rehearsal_self_launch_is_labelled():
    env = dict(os.environ, DL_BENCH_SAME_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--shape", "llama3_2_1b", "--steps", "8", "--warmup", "2",
                        "--prompt", "32", "--long-ctx", "0", "--no-altkv", "--no-cli"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["same_gpu_rehearsal"] is True and res["vs_baseline"] is None
    cfg = res["config"]
    assert cfg["tp_ranks"] == 2 and cfg["tp_sync"] == "q80" and cfg["parallelism"] == "tp2"
    assert cfg["tp_f32_pred_ms_per_token"] > 0 and res["value"] > 0
    # ranks reach their first forward seconds apart: the fused exchange's self-test must wait for them
    assert cfg["tp_fused_exchange"] is True and "self-test failed" not in r.stderr, r.stderr[-3000:]
    assert cfg["prompt_4k_eval_ms_per_token"] > 0
