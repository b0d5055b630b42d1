"""CPU reference backend vs the plain PyTorch fp32 oracle (same Q80 activation rounding)."""
import numpy as np
import pytest
import torch

from distributed_llama_multiusers_amd.models.llama import TorchLlama


def _logits_seq(backend, tokens, slot=0):
    out = []
    for p, t in enumerate(tokens):
        out.append(backend.forward([t], [p], [slot])[0])
    return np.stack(out)


@pytest.mark.parametrize("kind", ["q40", "f32"])
def test_cpu_matches_torch_oracle(C, assets, kind):
    buf = "q80" if kind == "q40" else "f32"
    be = C.cpu_backend(assets[kind], buf, 2)
    oracle = TorchLlama(assets[kind])
    tokens = [3, 17, 101, 7, 250, 9, 44, 300]
    got = _logits_seq(be, tokens)
    ref = oracle.forward(tokens).numpy()
    rel = np.abs(got - ref).max() / np.abs(ref).max()
    assert rel < (2e-2 if kind == "q40" else 1e-4), rel
    assert (got.argmax(-1) == ref.argmax(-1)).mean() >= 0.75


def test_cpu_batched_prefill_equals_sequential(C, assets):
    be1 = C.cpu_backend(assets["q40"], "q80", 2)
    be2 = C.cpu_backend(assets["q40"], "q80", 2)
    tokens = [5, 6, 7, 8, 9, 10]
    seq = _logits_seq(be1, tokens)
    bat = be2.forward(tokens, list(range(len(tokens))), [0] * len(tokens))
    np.testing.assert_allclose(bat, seq, rtol=1e-5, atol=1e-5)


def test_cpu_slots_are_independent(C, assets):
    """Two sequences in different KV slots in one batch == each run alone (fixes reference Q2)."""
    be = C.cpu_backend(assets["q40"], "q80", 2, n_slots=2)
    a, b = [11, 12, 13], [200, 201, 202]
    for p in range(3):
        both = be.forward([a[p], b[p]], [p, p], [0, 1])
    ra = C.cpu_backend(assets["q40"], "q80", 2)
    rb = C.cpu_backend(assets["q40"], "q80", 2)
    la = _logits_seq(ra, a)[-1]
    lb = _logits_seq(rb, b)[-1]
    np.testing.assert_allclose(both[0], la, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(both[1], lb, rtol=1e-5, atol=1e-5)


def test_q40_requires_q80_buffers(C, assets):
    with pytest.raises(Exception, match="Q80"):
        C.cpu_backend(assets["q40"], "f32", 1)
