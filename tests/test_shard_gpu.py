"""Subtree-sharded LDL^T (SURVEY §8 e) on the GPU, checked against the unsharded factorisation and
the oracle.  One GPU: the shards run as a ShardGroup (local all-reduce) or as separate shard handles
driven phase by phase from Python (the protocol a multi-GPU host runs with RCCL).

Tolerances (fp64): the sharded factorisation sums each top-front entry as (external part,
all-reduced) + (top children), a different order than the unsharded assembly, so on well-conditioned
K2 (delta = 1e-2) pivots and solutions agree to 1e-12 relative; the MPC loop on a sharded solver
reaches the same status, iteration count (+-1) and objective (1e-8 relative) as the unsharded one.
"""
import numpy as np
import pytest

from helpers import block_angular_k2, dense_k2, random_k2
from oracle.ldl import OracleLDL

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


def _solve(ls, Lw, b):
    rc = ls.factorize(torch.from_numpy(Lw.data.copy()).to(DEV))
    x = torch.from_numpy(b.copy()).to(DEV)
    ls.solve(x)
    torch.cuda.synchronize()
    return rc, x.cpu().numpy()


@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("kind", ["block", "random"])
def test_sharded_group_matches_unsharded(P, kind):
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = (block_angular_k2(1200, 2400, 24, 3, well=True) if kind == "block"
             else random_k2(300, 600, 0.01, 4, well=True))
    N = K.shape[0]
    b = np.random.default_rng(P).standard_normal(N)
    ref = HIPLDLSolver(N, Lw.indptr, Lw.indices)
    rc0, x0 = _solve(ref, Lw, b)
    grp = HIPLDLSolver(N, Lw.indptr, Lw.indices, nshards=P)
    rc1, x1 = _solve(grp, Lw, b)
    assert rc0 == rc1 == 0 and grp.is_factorized()
    info = grp.shard_info()
    assert (info["owner"] == -1).any() or P == 1
    assert np.array_equal(ref.perm(), grp.perm())
    d0, d1 = ref.diag(), grp.diag()
    assert np.all(np.abs(d1 - d0) <= 1e-12 * np.abs(d0)), np.max(np.abs(d1 - d0) / np.abs(d0))
    assert np.max(np.abs(x1 - x0)) <= 1e-12 * np.max(np.abs(x0))
    assert grp.inertia() == ref.inertia()
    # oracle in the same order
    o = OracleLDL(K, ref.perm())
    assert o.factorize() == N
    xr = o.solve(b)
    assert np.max(np.abs(x1 - xr)) <= 1e-11 * np.max(np.abs(xr))
    # a second factorisation / solve reuses the buffers (epochs, counters, zeroed top region)
    rc2, x2 = _solve(grp, Lw, 2.0 * b)
    assert rc2 == 0 and np.max(np.abs(x2 - 2.0 * x1)) <= 1e-12 * np.max(np.abs(x1))


@pytest.mark.parametrize("P", [2, 3, 4])
def test_sharded_batched_leaves(P):
    """Dense-column K2 (diagonal H, dense A: every x_j a batched leaf under the y front) sharded P
    ways: the y front is the top, the x_j are dealt to the shards, each shard's MFMA SYRK adds its
    members' W D^-1 W^T to the top front's external part (all-reduced) and its GEMV forward sums to
    the exchanged top right-hand side.  Same pivots / solution as unsharded to 1e-12, and the
    oracle's."""
    from madipm_amd.linear_solver import HIPLDLSolver
    from madipm_amd._lib import Symbolic, default_ldl_opts
    K, Lw = dense_k2(150, 1000, 3)
    N = K.shape[0]
    b = np.random.default_rng(P).standard_normal(N)
    ref = HIPLDLSolver(N, Lw.indptr, Lw.indices, ordering=0)
    assert ref.info()["lb_members"] == 1000
    rc0, x0 = _solve(ref, Lw, b)
    # every member on exactly one shard
    mem = [Symbolic(N, Lw.indptr, Lw.indices, default_ldl_opts(ordering=0), nshards=P, shard=r).info()["lb_members"]
           for r in range(P)]
    assert sum(mem) == 1000 and min(mem) > 0
    grp = HIPLDLSolver(N, Lw.indptr, Lw.indices, ordering=0, nshards=P)
    rc1, x1 = _solve(grp, Lw, b)
    assert rc0 == rc1 == 0 and grp.is_factorized()
    d0, d1 = ref.diag(), grp.diag()
    assert np.all(np.abs(d1 - d0) <= 1e-12 * np.abs(d0)), np.max(np.abs(d1 - d0) / np.abs(d0))
    assert np.max(np.abs(x1 - x0)) <= 1e-12 * np.max(np.abs(x0))
    assert grp.inertia() == ref.inertia() == (1000, 0, 150)
    o = OracleLDL(K, ref.perm())
    assert o.factorize() == N
    xr = o.solve(b)
    assert np.max(np.abs(x1 - xr)) <= 1e-11 * np.max(np.abs(xr))
    rc2, x2 = _solve(grp, Lw, 2.0 * b)
    assert rc2 == 0 and np.max(np.abs(x2 - 2.0 * x1)) <= 1e-12 * np.max(np.abs(x1))


def test_phase_protocol_with_separate_shards():
    """P shard handles (madipm_ldl_analyze_shard) driven phase by phase with an explicit all-reduce —
    the multi-GPU protocol, with local_allreduce standing in for RCCL."""
    from madipm_amd.linear_solver import HIPLDLSolver, local_allreduce
    K, Lw = block_angular_k2(1200, 2400, 24, 7, well=True)
    N, P = K.shape[0], 4
    b = np.random.default_rng(1).standard_normal(N)
    ref = HIPLDLSolver(N, Lw.indptr, Lw.indices)
    _, x0 = _solve(ref, Lw, b)
    sh = [HIPLDLSolver(N, Lw.indptr, Lw.indices, nshards=P, shard=r) for r in range(P)]
    vals = torch.from_numpy(Lw.data.copy()).to(DEV)
    bufs = [s.factorize_phase(1, vals) for s in sh]
    assert len({ln for _, ln in bufs}) == 1 and bufs[0][1] > 0
    # the exchange carries only the top fronts' lower triangles + 4 status slots per shard
    from madipm_amd._lib import Symbolic, default_ldl_opts
    _, _, nrows = Symbolic(N, Lw.indptr, Lw.indices, default_ldl_opts(), nshards=P, shard=0).supernodes()
    r = nrows[sh[0].shard_info()["owner"] == -1].astype(np.int64)
    assert bufs[0][1] == (r * (r + 1) // 2).sum() + 4 * P == sh[0].info()["xch_fact"]
    # per solve: the top fronts' forward right-hand sides (all-reduce) + the subtree solution slices
    # (all-gather, P slices of the largest shard's column count): less than n + top rows together
    ntop = int(r.sum())
    assert sh[0].info()["xch_solve"] == ntop
    assert N - ntop <= sh[0].info()["xch_gather"] <= P * (N - ntop)
    local_allreduce([p for p, _ in bufs], bufs[0][1])
    for s in sh:
        s.factorize_phase(2)
    assert all(s.is_factorized() for s in sh)
    xs = [torch.from_numpy(b.copy()).to(DEV) for _ in range(P)]
    bufs = [s.solve_phase(1, x) for s, x in zip(sh, xs)]
    local_allreduce([p for p, _ in bufs], bufs[0][1])
    bufs = [s.solve_phase(2, x) for s, x in zip(sh, xs)]
    assert bufs[0][1] == sh[0].info()["xch_gather"]
    local_allreduce([p for p, _ in bufs], bufs[0][1])  # the all-gather (other slices are zero)
    # ABI 0.2 protocol guard: a 0.1-style caller (phase 2, then no phase 3) is refused at its next call
    with pytest.raises(Exception, match="phase 3"):
        sh[0].solve_phase(1, xs[0])
    with pytest.raises(Exception, match="pending"):
        sh[0].solve(xs[0])
    for s, x in zip(sh, xs):
        assert s.solve_phase(3, x) == (None, 0)
    torch.cuda.synchronize()
    for x in xs:
        assert np.max(np.abs(x.cpu().numpy() - x0)) <= 1e-12 * np.max(np.abs(x0))
    with pytest.raises(Exception, match="phase 1 expected"):
        sh[0].solve_phase(2, xs[0])


def test_sharded_pivot_failure_reaches_every_shard():
    """A zero pivot inside one shard's subtree fails the factorisation on every shard (status slots)."""
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = block_angular_k2(600, 1200, 12, 2, well=True)
    N = K.shape[0]
    Lw = Lw.copy()
    grp = HIPLDLSolver(N, Lw.indptr, Lw.indices, nshards=4)
    own = grp.shard_info()["owner"]
    # zero the diagonal of a column owned by a subtree of shard 2 that has no off-diagonal entries
    # in its column -> exact zero pivot
    from madipm_amd._lib import Symbolic, default_ldl_opts
    S = Symbolic(N, Lw.indptr, Lw.indices, default_ldl_opts(), nshards=4, shard=2)
    f, parent, _ = S.supernodes()
    perm = grp.perm()
    col = None
    for s in np.flatnonzero(own == 2):
        for k in range(f[s], f[s + 1]):
            j = perm[k]
            if Lw.indptr[j + 1] - Lw.indptr[j] == 1:  # diagonal only (empty column of A)
                col = j
                break
        if col is not None:
            break
    if col is None:  # no isolated column: make the first pivot of a shard-2 front exactly zero
        j = perm[f[np.flatnonzero(own == 2)[0]]]
        col = j
        Lw.data[Lw.indptr[j]:Lw.indptr[j + 1]] = 0.0
    else:
        Lw.data[Lw.indptr[col]] = 0.0
    rc = grp.factorize(torch.from_numpy(Lw.data.copy()).to(DEV))
    assert rc > 0 and not grp.is_factorized()


def _mpc_cases():
    import os
    from madipm_amd import read_mps, standard_form_qp
    from madipm_amd.instances import random_lp, ex10_standin
    gold = os.path.join(os.path.dirname(__file__), "golden", "afiro.mps")
    return {"afiro_std": lambda: standard_form_qp(read_mps(gold)),
            "random_lp": lambda: random_lp(200, 400, 0.02, 3, ineq_frac=0.3),
            "ex10_small": lambda: standard_form_qp(ex10_standin(scale=0.05)),
            "dense_qp": lambda: __import__("madipm_amd.instances", fromlist=["dense_qp"]).dense_qp(n=1200, m=200,
                                                                                                   seed=0)}


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("case", ["afiro_std", "random_lp", "ex10_small", "dense_qp"])
def test_mpc_on_sharded_solver(P, case):
    """The MPC loop on a sharded solver (dense_qp: batched leaves dealt to the shards) reaches the
    unsharded solve's status, iteration count and objective."""
    from madipm_amd import MPCSolver, FixedRegularization
    qp = _mpc_cases()[case]()
    kw = dict(regularization=FixedRegularization(1e-8, -1e-8), max_iter=300)
    if case == "dense_qp":
        kw["ordering"] = 0  # natural order: the x columns are the batched leaves
        assert MPCSolver(qp, nshards=P, **kw).ldl_info()["lb_members"] > 0
    a = MPCSolver(qp, **kw).solve()
    b = MPCSolver(qp, nshards=P, **kw).solve()
    assert a.status == b.status == 1
    assert abs(a.iter - b.iter) <= 1
    assert abs(a.objective - b.objective) <= 1e-8 * max(1.0, abs(a.objective))


def test_multiprocess_sharded_mpc():
    """Two processes, one shard each, collectives through torch.distributed (gloo, host-staged):
    the multi-process protocol of the sharded MPC solve (bench.py --gpus N uses RCCL instead)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29531", os.path.join(root, "tests", "_dist_shard_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["identical"], res
    assert res["status"] == res["ref_status"] == 1
    assert abs(res["iter"] - res["ref_iter"]) <= 1
    assert abs(res["objective"] - res["ref_objective"]) <= 1e-8 * max(1.0, abs(res["ref_objective"]))


def test_rccl_comm_single_rank():
    """RCCL links and runs in this image: a 1-rank communicator's in-place all-reduce is the identity."""
    import ctypes as C
    from madipm_amd import RCCLComm
    from madipm_amd import _lib as L
    comm = RCCLComm(0, 1, RCCLComm.unique_id())
    x = torch.arange(1000, dtype=torch.float64, device=DEV)
    L.check(L.lib.madipm_comm_allreduce(comm.h, C.c_void_p(x.data_ptr()), 1000,
                                        C.c_void_p(torch.cuda.current_stream().cuda_stream)), "allreduce")
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1000, dtype=torch.float64, device=DEV))
