"""world_size-2 gloo tests of the N>1 host logic of bench.py on CPU: the multi-rank aggregation
(max time; iterations of the one sharded solve, or summed over replicas) and the broadcast of the
RCCL unique id through the process group (RCCLComm.from_torch's protocol, without the GPU)."""
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
    tot_dt, tot_it, per_rank = bench.aggregate(dt, iters, dist, False)
    sh_dt, sh_it, _ = bench.aggregate(dt, 22, dist, True)
    box = [bytes(range(128)) if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    q.put((rank, tot_dt, tot_it, sh_dt, sh_it, box[0] == bytes(range(128)), per_rank))
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
    for rank, tot_dt, tot_it, sh_dt, sh_it, id_ok, per_rank in res:
        assert per_rank == pytest.approx([0.5, 1.5])  # every rank's own time, in rank order
        assert tot_dt == pytest.approx(1.5)     # max over ranks
        assert tot_it == 21                     # replicas: sum over ranks
        assert sh_dt == pytest.approx(1.5) and sh_it == 22  # sharded: one solve's iterations
        assert id_ok


def test_collective_volume():
    import bench
    assert bench.collective_volume({"xch_fact": 0, "xch_solve": 0}, []) is None
    warm = [{"name": "k_fact_tree", "launches": 3}, {"name": "k_bwd_tree", "launches": 9}]
    v = bench.collective_volume({"xch_fact": 1000, "xch_solve": 300, "xch_gather": 500}, warm, world=2)
    assert v["solves_per_fact"] == 3 and v["collectives_per_iter"] == 7
    assert v["fact_bytes"] == 8000 and v["solve_bytes"] == 6400 and v["bytes_per_iter"] == 8 * (1000 + 3 * 800)
    # ring model, P = 2: all-reduce m -> m doubles sent per rank, all-gather G -> G / 2
    assert v["wire_bytes_per_rank_per_iter"] == pytest.approx(8 * (1000 + 3 * (300 + 250)))
