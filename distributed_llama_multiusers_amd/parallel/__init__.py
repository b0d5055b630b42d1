"""Tensor-parallel helpers: shard plan, device-communicator bootstrap, local worker launcher.

The reference has exactly one parallelism strategy, 1-D Megatron tensor parallelism over 2^n
nodes (src/llm.cpp:131-142, src/nn/nn-core.cpp:198-266). Here a rank is one
process per MI355X. Two launch styles share the same native engine:

* `dllama` root + `dllama worker` processes (the reference's CLI roles, TCP control plane in
  csrc/net/tcp.cpp) - `start_local_workers` plays examples/n-workers.sh;
* `torch.distributed` ranks (bench.py, tests) - `init_device_comm` exchanges the xGMI IPC handles or
  the RCCL unique id over the process group (gloo: control plane only).

The per-token data plane is never Python: it is the engine's device communicator (csrc/hip/
xgmi_comm.cpp one-shot all-reduce over IPC-mapped peer HBM, or RCCL).
"""
from __future__ import annotations

import os
import subprocess
import sys
import time
from dataclasses import dataclass

from .. import REPO_DIR


@dataclass(frozen=True)
class ShardPlan:
    """One rank's slice of every tensor (mirror of csrc/core/plan.h)."""
    n_ranks: int
    rank: int
    dim: int
    head_size: int
    n_heads0: int
    n_kv_heads0: int
    kv_mul: int
    q0: int
    kv0: int
    hidden0: int
    vocab0: int

    # global start offsets of the row (Wq/Wk/Wv/W1/W3/Wcls) and column (Wo/W2) slices
    @property
    def q_start(self) -> int:
        return self.rank * self.q0

    @property
    def kv_start(self) -> int:
        return self.rank * self.kv0

    @property
    def hidden_start(self) -> int:
        return self.rank * self.hidden0

    @property
    def vocab_start(self) -> int:
        return self.rank * self.vocab0

    def weight_bytes_q40(self) -> int:
        """Q40 bytes of this rank's matmul shards (18 B per 32 weights), excluding the f32
        embedding and norms that every rank keeps."""
        per_layer = (self.q0 + 2 * self.kv0) * self.dim + self.dim * self.q0 + 3 * self.hidden0 * self.dim
        return (per_layer * self._layers + self.vocab0 * self.dim) * 18 // 32

    _layers: int = 0


def validate_world(header: dict, world: int) -> None:
    """The reference's constraints (app.cpp:237-238, README.md:40-41; nn-core.cpp slicer asserts):
    2^n ranks, at most nKvHeads, and every sharded dimension divisible."""
    if world < 1 or world & (world - 1):
        raise ValueError(f"the number of ranks must be a power of two, got {world}")
    if world > header["n_kv_heads"]:
        raise ValueError(f"{world} ranks > {header['n_kv_heads']} KV heads: not supported (one KV head per rank at most)")
    for key in ("n_kv_heads", "vocab_size"):
        if header[key] % world:
            raise ValueError(f"{key}={header[key]} is not divisible by {world} ranks")
    if header["hidden_dim"] % (32 * world):
        raise ValueError(f"hidden_dim={header['hidden_dim']} does not split into 32-aligned shards over {world} ranks")


def shard_plan(header: dict, world: int, rank: int) -> ShardPlan:
    validate_world(header, world)
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    hs = header["dim"] // header["n_heads"]
    n_heads0 = header["n_heads"] // world
    n_kv0 = header["n_kv_heads"] // world
    return ShardPlan(n_ranks=world, rank=rank, dim=header["dim"], head_size=hs, n_heads0=n_heads0,
                     n_kv_heads0=n_kv0, kv_mul=header["n_heads"] // header["n_kv_heads"], q0=n_heads0 * hs,
                     kv0=n_kv0 * hs, hidden0=header["hidden_dim"] // world, vocab0=header["vocab_size"] // world,
                     _layers=header["n_layers"])


def tp_degrees(header: dict, max_world: int = 8) -> list[int]:
    """Every valid tensor-parallel degree up to max_world (one node of 8 MI355X)."""
    out = []
    w = 1
    while w <= max_world:
        try:
            validate_world(header, w)
            out.append(w)
        except ValueError:
            pass
        w *= 2
    return out


def init_device_comm(C, dist, rank: int, world: int, max_floats: int, device: int, kind: str = "xgmi",
                     log=sys.stderr):
    """Set up the engine's device data plane for `world` torch.distributed ranks.

    kind "xgmi": every rank allocates its IPC-shared buffer, handles are all-gathered over `dist`,
    each rank maps its peers, then exact all-reduces run across the real GPUs as a pre-flight
    self-test (the low-latency push protocol, then both protocols). Every decision is agreed by all
    ranks (MIN all-reduce of a success flag): if the push protocol fails anywhere it is switched
    off on every rank; if the rest fails anywhere, every rank falls back to RCCL, so no rank ever
    waits on a peer that uses another data plane.
    kind "rccl" (or fallback): rank 0's ncclUniqueId is broadcast.
    Returns (comm or None, rccl uid or None, kind actually used)."""
    import numpy as np
    import torch
    comm, uid = None, None
    if world <= 1:
        return None, None, kind

    def agreed(ok: bool) -> bool:  # every rank calls this at the same points, whatever failed locally
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(int(flag[0]))

    def failed(stage, e):
        print(f"rank {rank}: xgmi comm unavailable at {stage} ({e}); falling back to rccl", file=log)
        return False

    if kind == "xgmi":
        ok, handle = True, None
        try:
            comm = C.XgmiComm(rank, world, max_floats, device)
            handle = comm.handle()
        except Exception as e:  # noqa: BLE001 - reported, then the agreed fallback
            ok = failed("allocation", e)
        handles = [None] * world
        dist.all_gather_object(handles, handle)  # every rank takes part, with None on failure
        ok = agreed(ok and all(h is not None for h in handles))
        if ok:
            try:
                comm.connect(handles)
            except Exception as e:  # noqa: BLE001
                ok = failed("peer mapping", e)
            ok = agreed(ok)

        def self_test(n, stage):
            try:
                got = comm.all_reduce(np.full(n, rank + 1, np.float32))
                want = world * (world + 1) / 2
                if comm.timed_out() or not np.all(got == want):
                    raise RuntimeError(f"got {got[:4]}, want {want}")
                return True
            except Exception as e:  # noqa: BLE001
                return failed(stage, e)

        if ok:
            # pre-flight: exact all-reduces across the real GPUs before trusting the path (device-
            # side collectives, so they only run once every rank has mapped its peers). First the
            # low-latency push protocol used for decode-size messages; if it fails anywhere, every
            # rank switches it off and the pull protocol is tested on its own.
            if not agreed(self_test(4096, "low-latency self-test")):
                comm.set_low_latency(False)
                comm.reset_error()
                dist.barrier()
            small = self_test(4096, "self-test")
            large = self_test(min(1 << 17, max_floats), "large self-test")  # the pull protocol
            ok = agreed(small and large)
        if not ok:
            comm, kind = None, "rccl"
        dist.barrier()
    if kind != "xgmi":
        obj = [C.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    return comm, uid, kind


# ----------------------------------------------------------------------------- CLI workers
def dllama_binary(name: str = "dllama") -> str:
    path = os.path.join(REPO_DIR, "build", name)
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: run `make` first")
    return path


def start_local_workers(n: int, base_port: int = 9999, gpu_indices=None, nthreads: int = 1, extra=(),
                        env=None) -> list[subprocess.Popen]:
    """Start n `dllama worker` processes on 127.0.0.1 (ports base_port, base_port-1, ... like
    examples/n-workers.sh). gpu_indices[i] pins worker i to a GPU (None: CPU backend)."""
    procs = []
    for i in range(n):
        cmd = [dllama_binary(), "worker", "--port", str(base_port - i), "--nthreads", str(nthreads), *extra]
        if gpu_indices is not None:
            cmd += ["--gpu-index", str(gpu_indices[i])]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env or os.environ.copy()))
    time.sleep(0.2)
    return procs


def worker_addresses(n: int, base_port: int = 9999) -> list[str]:
    return [f"127.0.0.1:{base_port - i}" for i in range(n)]


def stop_workers(procs, timeout: float = 10.0) -> None:
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


__all__ = ["ShardPlan", "validate_world", "shard_plan", "tp_degrees", "init_device_comm", "dllama_binary",
           "start_local_workers", "worker_addresses", "stop_workers"]
