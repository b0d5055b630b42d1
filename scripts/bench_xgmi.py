"""In-graph latency of the xGMI one-shot all-reduce (csrc/hip/xgmi_comm.cpp).

    python scripts/bench_xgmi.py --world 2 [--same-gpu]
With --same-gpu every rank runs on cuda:0 (protocol overhead only, no xGMI hop); on a multi-GPU
node rank r uses GPU r."""
import argparse
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, same, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import distributed_llama_multiusers_amd as dl
    C = dl.native()
    gpu = 0 if same else rank
    comm = C.XgmiComm(rank, world, 1 << 20, gpu)
    hs = [None] * world
    dist.all_gather_object(hs, comm.handle())
    comm.connect(hs)
    dist.barrier()
    res = {}
    for n in (4096, 16384, 65536, 262144):
        dist.barrier()
        res[n] = comm.bench_all_reduce(n, 200)
    dist.barrier()
    q.put((rank, res, comm.timed_out()))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--same-gpu", action="store_true")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.same_gpu, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join()
    for r, res, to in sorted(out):
        print(f"rank {r} timed_out={to} " + " ".join(f"n={n}: {us:.2f} us" for n, us in res.items()))
