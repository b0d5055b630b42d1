"""Format and quantization tests (reference goldens: converter/writer-test.py:12-23,
nn-cpu-ops-test.cpp:82-99)."""
import io
import struct

import numpy as np
import pytest
import torch

from distributed_llama_multiusers_amd.utils import mfile
from distributed_llama_multiusers_amd.utils.mfile import FloatType


WRITER_TEST_GOLDEN = ('7e346345a692b89665b2c5790537876e598aaa366d988876a898b8d788a98868ce660c66f6b3a88cba5ce9a871987ba9cc5bcaaa760c1eb556a4455b747b6b9504968828ef2a8d7c1db5c6be3764799e66db6d8e76463126a30e4333cad7a4f645947c6cf97f9de086d468c8d535a6ba7dc799d3d0c657bab6799468cad8bb349eb7d7635c7c798998696bb38e4085a9eb34444ba96a7f8ba7b2b42d746a96cf9660aeb4499d8708ad5c7b9a7558947645f3bbb6b0346a656887ad9a86059baac5c596ab781c703569bb8a4356a4bd58cb78736ba09759bb0e34a6274e827b957d7a67dfa86846955660d234b6d9d78a378094a8a8708a7a774ae92f8a36b8c999a9b77a7d958a69747c807963941235379886d69a7a8767b3a6a4ac71999760')


def test_q40_writer_golden():
    # same input as the reference converter test: torch.randn(32, 16) with seed 1
    torch.manual_seed(1)
    t = torch.randn(32, 16)
    assert mfile.encode_tensor(t.numpy(), FloatType.Q40).hex() == WRITER_TEST_GOLDEN


def test_native_q40_matches_python(C):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(32 * 64).astype(np.float32)
    py = mfile.quantize_q40(x).tobytes()
    cc = C.quantize_q40(x).tobytes()
    # identical except possible ties in the max-magnitude pick; decoded values must agree
    assert np.allclose(C.dequantize_q40(np.frombuffer(cc, np.uint8)), mfile.dequantize_q40(np.frombuffer(py, mfile.Q40_DTYPE)), atol=1e-6)


@pytest.mark.parametrize("scale", [1.0, 1e-3, 100.0])
def test_q80_roundtrip(C, scale):
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(32 * 128) * scale).astype(np.float32)
    q = C.quantize_q80(x)
    y = C.dequantize_q80(q)
    # reference tolerance: 0.01 relative to block amax (nn-cpu-ops-test.cpp:82-99)
    amax = np.abs(x.reshape(-1, 32)).max(axis=1, keepdims=True)
    err = np.abs((y - x).reshape(-1, 32)) / np.maximum(amax, 1e-30)
    assert err.max() < 0.01
    # C++ and numpy quantizers agree on codes
    assert q.tobytes() == mfile.quantize_q80(x).tobytes()


def test_q40_roundtrip(C):
    rng = np.random.default_rng(2)
    x = rng.standard_normal(32 * 128).astype(np.float32)
    y = C.dequantize_q40(C.quantize_q40(x))
    amax = np.abs(x.reshape(-1, 32)).max(axis=1, keepdims=True)
    assert (np.abs((y - x).reshape(-1, 32)) / amax).max() < 0.13


def test_f16(C):
    for v in [0.0, 1.0, -2.5, 65504.0, 1e-5, 0.1]:
        assert C.f16_to_f32(C.f32_to_f16(v)) == float(np.float32(np.float16(v)))


def test_header_roundtrip(C, assets):
    h = C.load_header(assets["q40"])
    spec = assets["spec"]
    assert h["dim"] == spec.dim and h["n_layers"] == spec.n_layers and h["vocab_size"] == spec.vocab_size
    assert h["weight_type"] == FloatType.Q40
    assert h["head_size"] == spec.dim // spec.n_heads
    h2 = C.load_header(assets["q40"], 64)
    assert h2["seq_len"] == 64 and h2["orig_seq_len"] == spec.max_seq_len
    py = mfile.read_header(assets["q40"])
    assert py["dim"] == spec.dim and py["header_size"] == h["header_size"]


def test_tensor_table_matches_file(C, assets):
    t = C.tensor_table(assets["q40"])
    assert t[0]["name"] == "embedding" and t[-1]["name"] == "final_matmul_logits"
    import os
    last = t[-1]
    assert last["offset"] + last["bytes"] == os.path.getsize(assets["q40"])


def test_bad_magic_and_truncation(C, tmp_path):
    p = tmp_path / "bad.m"
    p.write_bytes(struct.pack("<ii", 0xABCD00, 8))
    with pytest.raises(Exception, match="Old model format"):
        C.load_header(str(p))
    p.write_bytes(struct.pack("<ii", 0x1234, 8))
    with pytest.raises(Exception, match="magic"):
        C.load_header(str(p))


def test_truncated_model_rejected(C, assets, tmp_path):
    data = open(assets["q40"], "rb").read()
    p = tmp_path / "trunc.m"
    p.write_bytes(data[:-18])
    with pytest.raises(Exception, match="Missing bytes"):
        C.tensor_table(str(p))


def test_shard_plan(C):
    h = {"dim": 4096, "hidden_dim": 14336, "n_layers": 32, "n_heads": 32, "n_kv_heads": 8, "vocab_size": 128256, "seq_len": 2048}
    for n in (1, 2, 4, 8):
        p = C.shard_plan(h, n, n - 1)
        assert p["q0"] == 4096 // n and p["kv0"] == 1024 // n and p["hidden0"] == 14336 // n
        assert p["vocab0"] == 128256 // n and p["kv_mul"] == 4
    with pytest.raises(Exception):
        C.shard_plan(h, 16, 0)  # more ranks than kv heads (app.cpp:237-238)
