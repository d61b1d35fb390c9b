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


class _FakeSolver:
    """Stands in for MPCSolver in bench.timed_leg (host logic only): rank r's loop takes 0.05 (r + 1) s."""

    def __init__(self, rank):
        self.rank, self.k = rank, 0

    def set_kernel_timing(self, mask=1):
        pass

    def kernel_stats(self):
        return [{"name": "k_fact_tree", "launches": 2, "time_ms": 0.4, "flops": 2e6, "alg_bytes": 8e6, "bytes": 1e7},
                {"name": "k_bwd_tree", "launches": 4, "time_ms": 0.2, "flops": 1e5, "alg_bytes": 4e6, "bytes": 5e6}]

    def set_max_iter(self, k):
        self.k = k

    def initialize(self):
        pass

    def solve(self, fetch_solution=True):
        import time
        import types
        time.sleep(0.05 * (self.rank + 1) if not fetch_solution else 0.0)
        return types.SimpleNamespace(iter=self.k)


def _leg_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    leg, warm, _ = bench.timed_leg(_FakeSolver(rank), 6, 2, dist, True, dist.barrier)
    q.put((rank, leg, [k["name"] for k in warm]))
    dist.destroy_process_group()


def test_two_rank_timed_leg():
    """bench.timed_leg (every leg's timed part; the 'neos' leg is sharded at N > 1): the time is the max over ranks, the
    iterations are the one sharded solve's, every rank's own time is reported."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_leg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, leg, warm in res:
        assert warm == ["k_fact_tree", "k_bwd_tree"]
        # (the closing barrier holds rank 0 until rank 1's slower loop is done: both see >= 0.1 s)
        assert len(leg["per_rank_s"]) == 2 and min(leg["per_rank_s"]) >= 0.1
        assert leg["steps"] == 6 and leg["iters_per_s"] == pytest.approx(6 / max(leg["per_rank_s"]))
        assert leg["ms_per_iter"] == pytest.approx(1e3 * max(leg["per_rank_s"]) / 6)
        # the dominant kind's roofline from the event statistics: (8 MB / 2) / (0.4 ms / 2) = 20 GB/s
        assert leg["roofline"]["kernel"] == "k_fact_tree" and leg["roofline"]["bound"] == "hbm"
        assert leg["roofline"]["achieved"] == pytest.approx(20.0)
