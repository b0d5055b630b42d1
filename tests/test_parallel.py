"""Tensor-parallel helpers on CPU: shard plans vs the native plan, the reference's world-size rules,
and the device-comm bootstrap agreeing on one data plane across ranks (gloo, 2 processes)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llama_multiusers_amd import parallel
from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES

BASE = dict(rope_theta=500000, weight_type=2, seq_len=128)


def header(name):
    return dict(BASE, **LLAMA_SHAPES[name])


@pytest.mark.parametrize("name", ["llama3_1_8b", "llama3_3_70b", "llama3_1_405b"])
def test_shard_plans_partition_every_tensor(C, name):
    h = header(name)
    assert parallel.tp_degrees(h) == [1, 2, 4, 8]
    for world in parallel.tp_degrees(h):
        plans = [parallel.shard_plan(h, world, r) for r in range(world)]
        native = C.shard_plan(h, world, 0)
        for key in ("q0", "kv0", "hidden0", "vocab0", "n_heads0", "kv_mul"):
            assert getattr(plans[0], key) == native[key], key
        # row slices tile [0, total) exactly, in rank order
        kv_dim = h["dim"] // h["n_heads"] * h["n_kv_heads"]
        for start, size, total in (("q_start", "q0", h["dim"]), ("kv_start", "kv0", kv_dim),
                                   ("hidden_start", "hidden0", h["hidden_dim"]),
                                   ("vocab_start", "vocab0", h["vocab_size"])):
            spans = [(getattr(p, start), getattr(p, start) + getattr(p, size)) for p in plans]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        # Q40 shard bytes shrink 1/world (the replicated embedding and norms are not counted)
        full = parallel.shard_plan(h, 1, 0).weight_bytes_q40()
        assert plans[0].weight_bytes_q40() * world == pytest.approx(full, rel=1e-6)


def test_world_size_rules():
    h = header("llama3_1_8b")
    for bad in (0, 3, 6, 16):
        with pytest.raises(ValueError):
            parallel.validate_world(h, bad)
    with pytest.raises(ValueError):
        parallel.shard_plan(h, 4, 4)
    assert parallel.tp_degrees(dict(h, hidden_dim=14336 + 32)) == [1]


def test_405b_q40_shard_fits_one_mi355x():
    h = header("llama3_1_405b")
    p = parallel.shard_plan(h, 8, 3)
    emb = h["vocab_size"] * h["dim"] * 4  # f32 embedding, replicated on every rank
    assert (p.weight_bytes_q40() + emb) / 2**30 < 288 * 0.5  # leaves over half of the 288 GB HBM for KV


class _FakeComm:
    def __init__(self, rank, world, max_floats, device):
        if os.environ.get("FAKE_XGMI_FAIL_RANK") == str(rank):
            raise RuntimeError("no peer access")
        self.world = world

    def handle(self):
        return b"h"

    def connect(self, handles):
        assert len(handles) == self.world

    def all_reduce(self, x):
        return np.full_like(x, self.world * (self.world + 1) / 2)

    def timed_out(self):
        return False

    def set_low_latency(self, on):
        pass

    def reset_error(self):
        pass


class _FakeC:
    XgmiComm = _FakeComm

    @staticmethod
    def rccl_unique_id():
        return b"uid-from-rank-0"


def _worker(rank, world, port, fail_rank, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fail_rank is not None:
        os.environ["FAKE_XGMI_FAIL_RANK"] = str(fail_rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with open(os.devnull, "w") as null:
        comm, uid, kind = parallel.init_device_comm(_FakeC, dist, rank, world, 4096, 0, "xgmi", log=null)
    out[rank] = (kind, uid, comm is not None)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_device_comm_choice_is_agreed_by_all_ranks(fail_rank):
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), fail_rank, out), nprocs=world, join=True)
        res = dict(out)
    if fail_rank is None:
        assert all(res[r] == ("xgmi", None, True) for r in range(world))
    else:  # one rank could not map its peers: every rank falls back to RCCL with rank 0's id
        assert all(res[r] == ("rccl", b"uid-from-rank-0", False) for r in range(world))
