"""RCCL data plane on a device: the fallback the engine (and bench.py) switch to when the xGMI
self-test fails. RCCL accepts a one-rank communicator, so every collective the engine issues -
all-reduce, all-gather, the root-only gather of the logits slices and the integer broadcast - runs
its real RCCL kernels here, eagerly and captured into a hipGraph that is replayed (the engine
captures its whole forward, collectives included). Reference roles: the TCP all-gather + merge of
SYNC_NODE_SLICES (nn-network.cpp:537-569) and the root gather of SYNC_NODE_SLICES_EXCEPT_ROOT
(llm.cpp:432)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import distributed_llama_multiusers_amd as dl
    C = dl.native()
    return C.RcclComm(C.rccl_unique_id(), 0, 1, 0)


def test_rccl_collectives_eager(comm):
    x = np.arange(4096, dtype=np.float32) * 0.25 - 100.0
    assert comm.world == 1 and comm.rank == 0
    assert np.array_equal(comm.all_reduce(x), x)
    assert np.array_equal(comm.all_gather(x), x)
    assert np.array_equal(comm.gather_to_root(x), x)
    assert comm.broadcast_ints([3, 1, 4, 1, 5], 0) == [3, 1, 4, 1, 5]


@pytest.mark.parametrize("graph", [False, True])
def test_rccl_engine_schedule(comm, graph):
    """The engine's separate-collective schedule (Q80-rounded all-reduces per layer, root gather of
    the logits slices, all-gather of the argmax pairs), replayed from one captured hipGraph: exact."""
    err = comm.schedule_check(layers=8, rows=4, dim=4096, vocab0=128256, runs=4, graph=graph)
    assert err == 0.0


def test_rccl_schedule_large_rows(comm):
    """A prefill-sized exchange (1024 rows x dim) through the same captured schedule."""
    assert comm.schedule_check(layers=2, rows=1024, dim=4096, vocab0=4096, runs=2, graph=True) == 0.0
