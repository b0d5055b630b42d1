"""Same-GPU TP2 prefill diagnosis: a 1B-shape engine with max_batch 1024 on the xGMI comm, one
forward_argmax per row count (eager, then graph), per-rank wall time and comm state.
usage: python scripts/diag_tp_prefill.py  (spawns its two ranks)"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(rank, world, port, rows_list, q):
    try:
        _rank_main(rank, world, port, rows_list, q)
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, "error", repr(e)[:300]))


def _rank_main(rank, world, port, rows_list, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import distributed_llama_multiusers_amd as dl
    from distributed_llama_multiusers_amd.models.synthetic import LLAMA_SHAPES
    from distributed_llama_multiusers_amd.parallel import init_device_comm
    C = dl.native()
    shape = dict(LLAMA_SHAPES["llama3_2_1b"], seq_len=4200)
    comm, uid, kind = init_device_comm(C, dist, rank, world, 1024 * 2048 * 2, 0, os.environ.get("DL_TP_COMM", "xgmi"))
    eng = C.HipEngine("", "q80", max_seq_len=4200, max_batch=1024, n_slots=1, kv_bf16=True, gpu_index=0,
                      synthetic=shape, seed=1234, rank=rank, world=world, uid=uid, comm=comm)
    print(f"rank {rank}: engine ready", flush=True)
    dist.barrier()
    out = []
    for rows in rows_list:
        for rep in range(2):
            t = time.perf_counter()
            try:
                eng.forward_argmax(list(range(rows)), list(range(rows)), [0] * rows)
                err = ""
            except Exception as e:  # noqa: BLE001
                err = str(e)[:120]
            out.append((rows, rep, round((time.perf_counter() - t) * 1000, 2), err))
            print(f"rank {rank} {kind}: {out[-1]}", flush=True)
            dist.barrier()
            if err:
                q.put((rank, kind, out))
                return
    q.put((rank, kind, out))


if __name__ == "__main__":
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rows_list = [int(x) for x in (sys.argv[1:] or ["64", "128", "256", "512", "1024"])]
    ps = [ctx.Process(target=rank_main, args=(r, 2, port, rows_list, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in range(2):
        print(q.get(timeout=240), flush=True)
    for p in ps:
        p.join(timeout=30)
