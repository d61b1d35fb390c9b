"""The factorisation's root tail on a side stream (LDLSolver::root_async_, MADIPM_ROOT_ASYNC, default
on): when the launches after the tree launch assemble and factorise only elimination-tree roots that
k_root_solve solves (ex10's 120-column coupling root), they run on a second stream forked after
k_fact_tree, beside the next solve's right-hand side, forward leaves and tree fronts; k_root_solve
(or the root's own k_fwd_tree task), status(), the next factorisation and the MPC's state read-back
join it.  Same kernels, same operands:
pivots, solutions and the whole MPC trajectory must be BITWISE those of MADIPM_ROOT_ASYNC=0, and the
oracle's (K2 and the MPC of the ex10 and supportcase10 stand-ins)."""
import numpy as np
import pytest

from helpers import lp_k2
from oracle.ldl import OracleLDL

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _qp(name):
    """ex10 at 0.2: 27 blocks (a fan-in above k_fact_tree's 8) under a 120-row coupling root factorised
    after the tree launch and solved by k_root_solve; supportcase10 at full size (BASELINE configs[3];
    smaller stand-ins put big fronts after the tree launch): a 48-row root solved forward and backward
    by its own k_fwd_tree task."""
    from madipm_amd import standard_form_qp
    from madipm_amd.instances import ex10_standin, supportcase10_standin
    if name == "ex10":
        return standard_form_qp(ex10_standin(scale=0.2))
    return standard_form_qp(supportcase10_standin())


def _k2(name):
    return lp_k2(_qp(name), 0, well=True)


def _ldl_run(K, Lw, monkeypatch, flag, rounds=3):
    """factorize + solve `rounds` times on changing values (a factorisation the previous round never
    solved with included), then one more solve: pivots and every solution."""
    from madipm_amd.linear_solver import HIPLDLSolver
    monkeypatch.setenv("MADIPM_ROOT_ASYNC", flag)
    dev = torch.device("cuda:0")
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices)
    info = ls.info()
    rng = np.random.default_rng(7)
    xs = []
    for k in range(rounds):
        vals = Lw.data * (1.0 + 0.1 * k)
        if k == 1:  # factorised, never solved with, then factorised again
            from madipm_amd import _lib as L
            v1 = torch.from_numpy(vals.copy()).to(dev)
            assert L.lib.madipm_ldl_factorize_async(ls.h, v1.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        assert ls.factorize(torch.from_numpy(vals.copy()).to(dev)) == 0
        x = torch.from_numpy(rng.standard_normal(K.shape[0])).to(dev)
        ls.solve(x)
        xs.append(x.cpu().numpy())
    return info, ls.diag().copy(), xs, ls


@pytest.mark.parametrize("name", ["ex10", "supportcase10"])
def test_root_async_ldl_bitwise(name, monkeypatch):
    K, Lw = _k2(name)
    i1, d1, x1, ls1 = _ldl_run(K, Lw, monkeypatch, "1")
    i0, d0, x0, _ = _ldl_run(K, Lw, monkeypatch, "0")
    assert i1["root_tail_async"] == 1 and i0["root_tail_async"] == 0, (i1["root_tail_async"], i0["root_tail_async"])
    assert np.array_equal(d0.view(np.uint64), d1.view(np.uint64))
    for a, b in zip(x0, x1):
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
    if name != "ex10":
        return  # (the oracle's LDL^T of the full-size supportcase10 K2 is too slow for a test)
    Kk = K.copy()
    Kk.data = Kk.data * 1.2  # the last round's values
    ref = OracleLDL(Kk.tocsc(), ls1.perm())
    assert ref.factorize() == K.shape[0]
    dr = ref.diag()
    assert np.all(np.abs(d1 - dr) <= 1e-12 * np.abs(dr))


@pytest.mark.parametrize("name", ["ex10", "supportcase10"])
def test_root_async_mpc_bitwise(name, monkeypatch):
    """The MPC loop with the tail overlapped: the pivot check travels with the predictor's residual
    read-back (after the join) instead of its k_rhs; iterates, trace and objective bitwise."""
    from madipm_amd import MPCSolver, FixedRegularization
    qp = _qp(name)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("MADIPM_ROOT_ASYNC", flag)
        s = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), max_iter=300)
        assert s.ldl_info()["root_tail_async"] == (1 if flag == "1" else 0)
        st = s.solve()
        out[flag] = (st, s.trace())
    (a, ta), (b, tb) = out["1"], out["0"]
    assert a.status == b.status == 1 and a.iter == b.iter
    assert np.float64(a.objective).view(np.uint64) == np.float64(b.objective).view(np.uint64)
    assert len(ta) == len(tb)
    for p, q in zip(ta, tb):
        for key in ("obj", "inf_pr", "inf_du", "mu", "alpha_p", "alpha_d"):
            assert np.float64(p[key]).view(np.uint64) == np.float64(q[key]).view(np.uint64), (p["k"], key)


@pytest.mark.parametrize("name", ["ex10", "supportcase10"])
def test_root_async_pivot_failure_reaches_the_host(name, monkeypatch):
    """A failing pivot inside the root (factorised on the side stream) must still be reported by
    factorize(): a K2 whose last pivot (in the root) is NaN; then the good values factorise."""
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = _k2(name)
    monkeypatch.setenv("MADIPM_ROOT_ASYNC", "1")
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices)
    assert ls.info()["root_tail_async"] == 1
    perm = ls.perm()
    j = int(perm[-1])  # the last pivot: inside the root
    vals = Lw.data.copy()
    assert Lw.indices[Lw.indptr[j]] == j
    vals[Lw.indptr[j]] = np.nan  # its diagonal entry: a non-finite pivot
    assert ls.factorize(torch.from_numpy(vals).cuda()) != 0
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).cuda()) == 0


@pytest.mark.parametrize("var", ["ROCPROF_COUNTER_COLLECTION", "AMD_SERIALIZE_KERNEL", "HIP_LAUNCH_BLOCKING"])
def test_root_async_off_when_kernels_serialise(var, monkeypatch):
    """Counter collection (rocprofv3 --pmc) and the HIP serialisation knobs run one kernel at a time:
    the tail's kernel would wait on the device for a kernel that cannot start.  The solver then keeps
    the tail on the caller's stream (r6_ze: a --pmc pass ended in the hand-off timeout)."""
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = _k2("ex10")
    monkeypatch.setenv("MADIPM_ROOT_ASYNC", "1")
    monkeypatch.setenv(var, "1")
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices)
    assert ls.info()["root_tail_async"] == 0
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).cuda()) == 0
