"""world_size-2 gloo test of the bench's multi-rank aggregation (replicas: barrier, max time,
sum of iterations) — the N>1 path of bench.py, exercised on CPU."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    dt, iters = 0.5 + rank, 10 + rank          # rank-local timing and iteration count
    tot_dt, tot_it = bench.aggregate(dt, iters, dist, torch.device("cpu"))
    q.put((rank, tot_dt, tot_it))
    dist.destroy_process_group()


def test_two_rank_aggregation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, tot_dt, tot_it in res:
        assert tot_dt == pytest.approx(1.5)     # max over ranks
        assert tot_it == 21                     # sum over ranks
