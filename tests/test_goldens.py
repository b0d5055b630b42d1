"""Reference goldens (values printed by the reference's own unit tests) pinned on our primitives.

* invRms 1/0.4402 (src/nn/nn-cpu-ops-test.cpp:102-118), softmax and SiLU of i/8
  (nn-cpu-ops-test.cpp:180-218);
* Llama-3.1-scaled RoPE at positions 6 and 31 (src/nn/nn-vulkan-test.cpp:426-486: dim 2048, 32 heads,
  theta 500000, scaling factor 32 / low 1 / high 4 / original context 8192, x = 1) through the
  engines' RoPE table (csrc/core/plan.cpp buildRopeTable, used by both the CPU backend and the
  HIP kernels);
* the 4096 x 4096 Q80 x Q40 matmul of nn-vulkan-test.cpp:533-587 (x = i * 1e-5, W = i * 1e-6, 4
  rows, every output within 3.5 % of the f32 sum) on the CPU backend's matmul.
The GPU kernels are pinned against the same table and matmul in tests/test_gpu_ops.py.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def co(C):
    return C.cpu_ops


def test_inv_rms_golden(co):
    x = np.array([0.1, 0.3, 0.2, 0.4, 0.6, 0.5, 0.0, 0.8], np.float32)
    assert abs(co.inv_rms(x, 1e-5) - 1.0 / 0.4402) < 1e-3


def test_softmax_golden(co):
    y = co.softmax(np.arange(8, dtype=np.float32) / 8.0)
    want = [0.077399, 0.087780, 0.099500, 0.112761, 0.127778, 0.144793, 0.164072, 0.185917]
    assert np.abs(y - want).max() < 1e-3


def test_silu_golden(co):
    y = co.silu(np.arange(8, dtype=np.float32) / 8.0)
    want = [0.000000, 0.066401, 0.140544, 0.222250, 0.311233, 0.407116, 0.509461, 0.617802]
    assert np.abs(y - want).max() < 1e-3


ROPE_HEADER = dict(dim=2048, hidden_dim=8192, n_layers=1, n_heads=32, n_kv_heads=8, vocab_size=32, seq_len=4096,
                   rope_theta=500000.0, rope_scaling_factor=32.0, rope_scaling_low_freq_factor=1.0,
                   rope_scaling_high_freq_factor=4.0, rope_scaling_orig_max_seq_len=8192, rope_type=2)

# (position, {element: value}) from nn-vulkan-test.cpp:468-483
ROPE_GOLDENS = [
    (6, {0: 1.239586, 1: 0.680755, 2: 0.077202, 3: -1.412105, 1988: -1.356766, 2022: 0.999923, 2023: 1.000077}),
    (31, {0: 1.318780, 1: 0.510705, 1078: 0.999985, 1079: 1.000015}),
]


def rope_goldens_table(C):
    return C.cpu_ops.rope_table(ROPE_HEADER)


@pytest.mark.parametrize("pos,want", ROPE_GOLDENS)
def test_rope_llama31_golden(C, co, pos, want):
    table = rope_goldens_table(C)
    y = co.rope_apply(np.ones(2048, np.float32), pos, 64, table)
    for i, v in want.items():
        assert abs(y[i] - v) < 1e-5, (pos, i, y[i], v)


def test_matmul_q80_q40_golden(C, co):
    n = d = 4096
    B = 4
    x = (np.arange(B * n, dtype=np.float64) * 0.00001).astype(np.float32).reshape(B, n)
    w = (np.arange(n * d, dtype=np.float64) * 0.000001).astype(np.float32).reshape(d, n)
    blocks = C.quantize_q40(w)
    y = co.matmul_q40_q80(blocks, d, n, x)
    ref = x.astype(np.float64) @ w.astype(np.float64).T
    assert np.all(np.abs(y - ref) <= np.abs(ref) * 0.035)


def test_host_sampler_coin_semantics(C, co):
    """sampleHost with an explicit coin follows the reference's Sampler::sample: temperature 0 ->
    argmax, top-p >= 1 -> multinomial in index order, else the nucleus in descending order."""
    rng = np.random.default_rng(3)
    logits = rng.standard_normal(1000).astype(np.float32) * 3
    assert co.sample_host(logits, 0.0, 0.9, 0.5) == int(np.argmax(logits))
    p = np.exp(logits / 0.7 - (logits / 0.7).max())
    p /= p.sum()
    cdf = np.cumsum(p)
    for coin in (0.0, 0.3, 0.77, 0.999):
        assert co.sample_host(logits, 0.7, 1.0, coin) == int(np.searchsorted(cdf, coin, side="right"))
    order = np.argsort(-p, kind="stable")
    cut = np.searchsorted(np.cumsum(p[order]), 0.5, side="right")
    nucleus = order[:cut + 1]
    for coin in (0.0, 0.5, 0.99):
        assert co.sample_host(logits, 0.7, 0.5, coin) in set(nucleus.tolist())


def test_cpu_backend_forward_sample(C, assets):
    b = C.cpu_backend(assets["q40"], "q80", 2, max_batch=8, n_slots=1)
    toks, pos = [1, 2, 3], [0, 1, 2]
    ref = b.forward(toks, pos, [0, 0, 0])
    got = b.forward_sample(toks, pos, [0, 0, 0], [0.0, -1.0, 0.8], [0.9, 0.9, 0.9], [0.1, 0.2, 0.3])
    assert got[0] == int(np.argmax(ref[0])) and got[1] == -1
    assert got[2] == C.cpu_ops.sample_host(ref[2], 0.8, 0.9, 0.3)
