"""GPU parity of the multifrontal LDL^T (HIP, libmadipm_hip) against the oracle's up-looking
sparse LDL^T (oracle/ldl_ref.c = LDLFactorizations.jl's algorithm) in the SAME pivot order.

Both factor the same quasi-definite K2 without pivoting, so they differ only by floating-point
summation order.  Two regimes, tolerances (fp64) written out:
  * well-conditioned K2 (delta = 1e-2, Sigma in [0.1, 10]: element growth O(1)) — exact parity of
    the algorithm:  |d_gpu - d_ref| <= 1e-12 |d_ref| per pivot,  ||x_gpu - x_ref|| / ||x_ref|| <= 1e-12;
  * IPM-like K2 (delta = 1e-8, Sigma in [1e-2, 1e2]): static pivoting has element growth ~1/delta
    (pivots reach 1e9), so pivots differ by up to ~1e-7 relative between ANY two summation orders
    (a dense no-pivot LDL^T in the same order differs from the oracle by 1.3e-7).  There the gate
    is stability parity: normwise backward error berr(x_gpu) <= 10 berr(x_ref) + 1e-15, and
    ||x_gpu - x_ref|| / ||x_ref|| <= 1e-6 (kappa(K2) ~1e10).
  * normwise backward error: berr(x_gpu) <= 10 * berr(x_ref) + 1e-15
    (static-pivot LDL^T on K2 with delta = 1e-8 has berr ~1e-10 in ANY implementation — the
     dense no-pivot LDL^T in the same order shows the same level)
  * inertia:                 (n, 0, m) for quasi-definite K2."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

from helpers import block_angular_k2, random_k2
from oracle.ldl import OracleLDL

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _berr(K, x, b):
    return np.max(np.abs(K @ x - b)) / (spla.norm(K, np.inf) * np.max(np.abs(x)) + np.max(np.abs(b)))


def _check_pivots(d_gpu, d_ref, K):
    tol = 1e-12 * np.abs(d_ref)
    bad = np.abs(d_gpu - d_ref) > tol
    k = int(np.argmax(np.abs(d_gpu - d_ref) / tol))
    assert not bad.any(), (f"{bad.sum()} pivots off; worst k={k} gpu={d_gpu[k]:.17e} ref={d_ref[k]:.17e}")


def _check_case(K, Lw, small_front_max=128, relax=1, seed=0, well=False):
    from madipm_amd.linear_solver import HIPLDLSolver
    N = K.shape[0]
    ls = HIPLDLSolver(N, Lw.indptr, Lw.indices, small_front_max=small_front_max, relax=relax)
    dev = torch.device("cuda:0")
    rc = ls.factorize(torch.from_numpy(Lw.data.copy()).to(dev))
    assert rc == 0 and ls.is_factorized()
    perm = ls.perm()
    ref = OracleLDL(K, perm)
    assert ref.factorize() == N
    d_gpu, d_ref = ls.diag(), ref.diag()
    if well:
        _check_pivots(d_gpu, d_ref, K)
    rng = np.random.default_rng(seed)
    b = rng.standard_normal(N)
    x = torch.from_numpy(b.copy()).to(dev)
    ls.solve(x)
    torch.cuda.synchronize()
    x = x.cpu().numpy()
    xr = ref.solve(b)
    ferr = np.max(np.abs(x - xr)) / np.max(np.abs(xr))
    assert ferr <= (1e-12 if well else 1e-6), f"forward difference {ferr:.3e}"
    bg, br = _berr(K, x, b), _berr(K, xr, b)
    assert bg <= 10 * br + 1e-15, f"backward error gpu {bg:.3e} vs oracle {br:.3e}"
    return ls


@pytest.mark.parametrize("m,n,dens,seed", [(1, 1, 1.0, 0), (5, 8, 0.3, 0), (30, 50, 0.05, 1),
                                           (200, 300, 0.01, 3), (400, 900, 0.004, 4)])
@pytest.mark.parametrize("sfm", [128, 16])
@pytest.mark.parametrize("well", [True, False])
def test_ldl_random_k2(m, n, dens, seed, sfm, well):
    K, Lw = random_k2(m, n, dens, seed, well=well)
    ls = _check_case(K, Lw, small_front_max=sfm, well=well)
    assert ls.inertia() == (n, 0, m)


@pytest.mark.parametrize("sfm,relax", [(128, 1), (32, 1), (128, 0)])
@pytest.mark.parametrize("well", [True, False])
def test_ldl_block_angular(sfm, relax, well):
    K, Lw = block_angular_k2(3000, 4000, 20, 7, well=well)
    ls = _check_case(K, Lw, small_front_max=sfm, relax=relax, well=well)
    assert ls.inertia() == (4000, 0, 3000)


@pytest.mark.parametrize("tree_fact,tree_solve", [("0", "0"), ("1", "0"), ("0", "1"), ("1", "1")])
@pytest.mark.parametrize("well", [True, False])
def test_ldl_tree_and_level_paths(tree_fact, tree_solve, well, monkeypatch):
    """The dependency-driven tree kernels (k_fact_tree, k_fwd_tree / k_bwd_tree) and the level-by-level
    kernels they replace give the oracle's pivots and solution on the same block-angular K2 (the bench's
    structure); MADIPM_TREE_FACT / MADIPM_TREE_SOLVE = 0 select the level path at analysis time."""
    monkeypatch.setenv("MADIPM_TREE_FACT", tree_fact)
    monkeypatch.setenv("MADIPM_TREE_SOLVE", tree_solve)
    K, Lw = block_angular_k2(3000, 4000, 20, 7, well=well)
    ls = _check_case(K, Lw, well=well)
    assert ls.inertia() == (4000, 0, 3000)


@pytest.mark.parametrize("sfm", [128, 192])
@pytest.mark.parametrize("well", [True, False])
def test_ldl_in_lds_fronts(sfm, well):
    """The in-LDS factorisation (16-pivot diagonal blocks factorised in registers — DPP row broadcasts
    + gfx950 permlane swaps, l = a * (1/d) with a Newton-refined v_rcp_f64 — panel and trailing update
    on f64 MFMA, the update block's Schur complement formed once after all pivots): the oracle's pivots
    to 1e-12 (well conditioned) and its solution, square (<= 128 rows) and packed (<= 192 rows)
    storage.  The block-angular K2 has fronts of 16 .. 150 columns (several diagonal blocks each) and a
    120-column root (k_small_blocked); the QP case a dense front."""
    K, Lw = block_angular_k2(3000, 4000, 20, 7, well=well)
    ls = _check_case(K, Lw, small_front_max=sfm, well=well)
    assert ls.inertia() == (4000, 0, 3000)
    K, Lw = _dense_k2(150, 1000, 5)
    _check_case(K, Lw, small_front_max=sfm, well=True)


def _factor_solve(K, Lw, sfm, seed=0):
    from madipm_amd.linear_solver import HIPLDLSolver
    N = K.shape[0]
    ls = HIPLDLSolver(N, Lw.indptr, Lw.indices, small_front_max=sfm)
    dev = torch.device("cuda:0")
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).to(dev)) == 0
    b = np.random.default_rng(seed).standard_normal(N)
    x = torch.from_numpy(b.copy()).to(dev)
    ls.solve(x)
    torch.cuda.synchronize()
    return ls.diag().copy(), x.cpu().numpy(), ls


@pytest.mark.parametrize("sfm", [128, 192])
@pytest.mark.parametrize("case", ["block_well", "block_ipm", "dense_front", "random"])
def test_ldl_fact_pipe_bitwise(case, sfm, monkeypatch):
    """The pipelined in-LDS schedule (blocked_factor_pipe: wave 0 runs the pivot chain, the other
    waves the panel and trailing update, LDS-counter hand-offs; MADIPM_FACT_PIPE=1, default) forms
    every tile with the same MFMA sequence from the same operands as the barrier schedule
    (blocked_factor_lds, MADIPM_FACT_PIPE=0): pivots and solution agree BITWISE, on k_fact_tree
    (8 waves) and k_small_blocked (4 waves; the 120-column root, dense fronts of 1-12 pivot blocks,
    square and packed storage) — and the oracle's to 1e-12."""
    if case.startswith("block"):
        K, Lw = block_angular_k2(3000, 4000, 20, 7, well=case == "block_well")
    elif case == "dense_front":
        K, Lw = _dense_k2(150, 1000, 5)
    else:
        K, Lw = random_k2(400, 900, 0.004, 4, well=True)
    out = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("MADIPM_FACT_PIPE", pipe)
        out[pipe] = _factor_solve(K, Lw, sfm)
    (d0, x0, _), (d1, x1, ls1) = out["0"], out["1"]
    assert np.array_equal(d0.view(np.uint64), d1.view(np.uint64)), \
        f"pivots differ at {np.flatnonzero(d0 != d1)[:8]}"
    assert np.array_equal(x0.view(np.uint64), x1.view(np.uint64))
    if case != "block_ipm":
        _check_case(K, Lw, small_front_max=sfm, well=True)


def test_ldl_pipe_lost_handoff_is_an_error(monkeypatch):
    """A hand-off of the pipelined in-LDS schedule that never arrives (MADIPM_DEBUG_PIPE_FAULT=1: the
    pivot-chain wave never publishes M_K) must not yield a silently wrong factor: the waits time out,
    the front raises the status block's sticky error and factorize() fails loudly."""
    from madipm_amd.linear_solver import HIPLDLSolver
    monkeypatch.setenv("MADIPM_DEBUG_PIPE_FAULT", "1")
    K, Lw = _dense_k2(150, 1000, 5)
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices, small_front_max=192)
    with pytest.raises(Exception, match="hand-off"):
        ls.factorize(torch.from_numpy(Lw.data.copy()).cuda())
    monkeypatch.setenv("MADIPM_DEBUG_PIPE_FAULT", "0")
    _factor_solve(K, Lw, 192)  # a fresh solver factorises normally


@pytest.mark.parametrize("shrink", ["8", "1048576"])
def test_ldl_fold_carve_overflow_is_an_error(shrink, monkeypatch):
    """k_fact_tree checks on the device that every front and each of its folded-leaf batches fit the
    launch's LDS carve (r4: a fold batch larger than its front's carve factorised silently wrong).
    MADIPM_DEBUG_LDS_SHRINK pretends the launch has fewer bytes — by 8 (the largest front alone
    overflows) or by 1 MB (every front) — so the check must fire: factorize() raises, never a silent
    wrong factor, and a fresh solver factorises normally."""
    from helpers import lp_k2
    from madipm_amd import standard_form_qp
    from madipm_amd.instances import ex10_standin
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = lp_k2(standard_form_qp(ex10_standin(scale=0.05)), 0, well=True)
    monkeypatch.setenv("MADIPM_DEBUG_LDS_SHRINK", shrink)
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices)
    with pytest.raises(Exception, match="LDS carve"):
        ls.factorize(torch.from_numpy(Lw.data.copy()).cuda())
    monkeypatch.delenv("MADIPM_DEBUG_LDS_SHRINK")
    _check_case(K, Lw, well=True)


@pytest.mark.parametrize("help_", ["1", "0"])
@pytest.mark.parametrize("well", [True, False])
def test_fold_helpers(help_, well, monkeypatch):
    """Fold helpers: a tree front with two or more leaf batches hands the first half to a helper
    ticket, which folds them into a zeroed LDS image of the front (their L and D written as the
    front's), stores it write-through and publishes a flag; the front folds the rest and adds the image
    after its waits.  The ex10 stand-in at 0.1 (level-1/2 fronts of 3-4 batches): the oracle's pivots
    (1e-12, well conditioned) and solution with helpers on and off (MADIPM_FOLD_HELP=0)."""
    from helpers import lp_k2
    from madipm_amd import standard_form_qp
    from madipm_amd.instances import ex10_standin
    monkeypatch.setenv("MADIPM_FOLD_HELP", help_)
    qp = standard_form_qp(ex10_standin(scale=0.1))
    K, Lw = lp_k2(qp, 1, well=well)
    ls = _check_case(K, Lw, well=well)
    assert ls.inertia() == (qp.nvar, 0, qp.ncon)


@pytest.mark.parametrize("case", ["block_well", "block_ipm", "random"])
def test_root_backward_in_forward(case):
    """An elimination-tree root (r == w) is solved backward by the forward tree kernel right after its
    forward substitution (panel already in LDS; k_bwd_tree skips its ticket): the oracle's solution."""
    if case.startswith("block"):
        K, Lw = block_angular_k2(3000, 4000, 20, 7, well=case == "block_well")
    else:
        K, Lw = random_k2(400, 900, 0.004, 4, well=True)
    _check_case(K, Lw, well=case != "block_ipm")


@pytest.mark.parametrize("well", [True, False])
def test_ldl_medium_tree_fronts(well):
    """Medium fronts (192 < r <= 256: the supportcase10 stand-in's block separators, r ~ 230) factorised
    inside the dependency-driven tree launch — F in HBM, one 64-column panel in LDS at a time, the
    trailing update on f64 MFMA in HBM, children's update blocks added in place — give the oracle's
    pivots (1e-12, well conditioned) and solution, chains of medium fronts included."""
    from helpers import lp_k2
    from madipm_amd import standard_form_qp
    from madipm_amd.instances import supportcase10_standin
    qp = standard_form_qp(supportcase10_standin(scale=0.05, block_scale=1.0))
    K, Lw = lp_k2(qp, 3, well=well)
    ls = _check_case(K, Lw, well=well)
    info = ls.info()
    assert info["tree_medium"] >= 3 and info["max_front"] > 192, info
    assert ls.inertia() == (qp.nvar, 0, qp.ncon)


@pytest.mark.parametrize("split", ["1", "0"])
@pytest.mark.parametrize("kpan", ["1", "2", "4"])
@pytest.mark.parametrize("n,m", [(320, 100), (130, 200)])
def test_big_front_panel_groups(kpan, n, m, split, monkeypatch):
    """A dense K2 (dense SPD H, dense A: one big front of n + m columns, several 64-column panels
    with a partial last one) on the big-front path with the deferred multi-panel trailing update in
    groups of MADIPM_BIG_KPAN panels (1 = right-looking per panel): pivots and solution of the oracle.
    Its 128-tile trailing launches have few tiles, so k_big_upd128 splits their K over 2-4 workgroups
    per tile (partials summed in part order by the tile's last part); MADIPM_UPD_SPLIT=0: unsplit."""
    import scipy.sparse as sp
    monkeypatch.setenv("MADIPM_BIG_KPAN", kpan)
    monkeypatch.setenv("MADIPM_UPD_SPLIT", split)
    rng = np.random.default_rng(11)
    B = rng.standard_normal((n, n))
    H = B @ B.T / n + np.eye(n)
    A = rng.standard_normal((m, n))
    K = sp.csc_matrix(np.block([[H, A.T], [A, -1e-2 * np.eye(m)]]))
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    _check_case(K, Lw, small_front_max=16, well=True)


@pytest.mark.parametrize("well", [True, False])
def test_ldl_tree_solves_repeated(well):
    """Tree solves (one task per front, flag epochs per solve) with the micro leaves under tree fronts
    solved from leaf records by the flat launches: the oracle's solution for several right-hand sides
    in a row."""
    K, Lw = block_angular_k2(3000, 4000, 20, 7, well=well)
    ls = _check_case(K, Lw, well=well)
    ref = OracleLDL(K, ls.perm())
    assert ref.factorize() == K.shape[0]
    rng = np.random.default_rng(5)
    for _ in range(3):
        b = rng.standard_normal(K.shape[0])
        x = torch.from_numpy(b.copy()).cuda()
        ls.solve(x)
        xr = ref.solve(b)
        assert np.max(np.abs(x.cpu().numpy() - xr)) <= (1e-12 if well else 1e-6) * np.max(np.abs(xr))


@pytest.mark.parametrize("fold", ["0", "1"])
@pytest.mark.parametrize("well", [True, False])
def test_ldl_leaf_folding(fold, well, monkeypatch):
    """Leaf folding (default; MADIPM_FOLD=0 turns it off): tree fronts factorise their micro-leaf
    children themselves and subtract the leaves' rank-1/2 updates in LDS through destination-sorted
    product lists — same pivots / solution as the oracle, with and without it."""
    monkeypatch.setenv("MADIPM_FOLD", fold)
    K, Lw = block_angular_k2(3000, 4000, 20, 7, well=well)
    ls = _check_case(K, Lw, well=well)
    assert ls.inertia() == (4000, 0, 3000)
    info = ls.info()
    if fold == "1":
        assert info["fold_fronts"] >= 1 and info["fold_leaves"] >= 100
    else:
        assert info["fold_fronts"] == 0


@pytest.mark.parametrize("well", [True, False])
def test_ldl_qp_dense_front(well):
    K, Lw = random_k2(150, 400, 0.05, 11, qp=True, well=well)
    ls = _check_case(K, Lw, small_front_max=128, well=well)
    assert ls.info()["nbig"] >= 1             # exercises the HBM panel + MFMA update path


def test_ldl_refactorize_new_values():
    """Only the diagonal changes between IPM iterations: refactorise in place."""
    K, Lw = random_k2(200, 300, 0.01, 5, well=True)
    from madipm_amd.linear_solver import HIPLDLSolver
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices)
    perm = ls.perm()
    for it in range(3):
        vals = Lw.data.copy()
        diag = Lw.indices == np.repeat(np.arange(K.shape[0]), np.diff(Lw.indptr))
        vals[diag] *= (1.0 + it)
        Kn = K.copy().tolil()
        Kn.setdiag(K.diagonal() * (1.0 + it))
        Kn = Kn.tocsc()
        assert ls.factorize(torch.from_numpy(vals).cuda()) == 0
        ref = OracleLDL(Kn, perm)
        ref.factorize()
        dr = ref.diag()
        _check_pivots(ls.diag(), dr, Kn)


def test_ldl_zero_pivot_reported():
    import scipy.sparse as sp
    from madipm_amd.linear_solver import HIPLDLSolver
    # [[1,.,1],[.,0,.],[1,.,2]] with an explicit structural zero on the diagonal
    Lw = sp.csc_matrix((np.array([1.0, 1.0, 0.0, 2.0]), np.array([0, 2, 1, 2]), np.array([0, 2, 3, 4])),
                       shape=(3, 3))
    ls = HIPLDLSolver(3, Lw.indptr, Lw.indices, ordering=0)
    rc = ls.factorize(torch.from_numpy(Lw.data.copy()).cuda())
    assert rc > 0 and not ls.is_factorized()


# ---------------------------------------------------------------- batched leaf columns (dense QP, config 3)
from helpers import dense_k2 as _dense_k2  # noqa: E402


@pytest.mark.parametrize("m,n,ordering,sfm", [(150, 1000, 0, 128), (200, 3000, 0, 128), (150, 1000, 1, 128),
                                               (128, 1000, 0, 128), (150, 1000, 0, 192), (100, 800, 0, 128)])
def test_batched_leaf_columns_parity(m, n, ordering, sfm):
    """K2 of a QP with diagonal H and dense A: the x_j are single-column leaves with m-row updates,
    eliminated as ONE group (W build + MFMA SYRK into the y front + GEMV solves).  Well conditioned:
    pivots and solution vs the oracle LDL^T in the same order to 1e-12 (relative)."""
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = _dense_k2(m, n, 3)
    N = K.shape[0]
    ls = HIPLDLSolver(N, Lw.indptr, Lw.indices, ordering=ordering, small_front_max=sfm)
    info = ls.info()
    if m >= 128:  # lb_min_rows (symbolic.hpp): shorter update columns are factorised one by one
        assert info["lb_groups"] >= 1 and info["lb_members"] >= n // 2
    else:
        assert info["lb_groups"] == 0
    dev = torch.device("cuda:0")
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).to(dev)) == 0
    ref = OracleLDL(K, ls.perm())
    assert ref.factorize() == N
    _check_pivots(ls.diag(), ref.diag(), K)
    assert ls.inertia() == (n, 0, m)
    b = np.random.default_rng(1).standard_normal(N)
    x = torch.from_numpy(b.copy()).to(dev)
    ls.solve(x)
    torch.cuda.synchronize()
    xr = ref.solve(b)
    assert np.max(np.abs(x.cpu().numpy() - xr)) <= 1e-11 * np.max(np.abs(xr))
    # refactorisation with new values reuses W's pattern
    Lw2 = Lw.copy()
    Lw2.data *= 1.5
    assert ls.factorize(torch.from_numpy(Lw2.data.copy()).to(dev)) == 0
    assert np.allclose(ls.diag(), 1.5 * ref.diag(), rtol=1e-12)


@pytest.mark.parametrize("sfm", [128, 192])
def test_small_front_storage_variants(sfm):
    """Fronts up to 192 rows can be factorised in LDS with packed lower storage (small_front_max=192)
    instead of the big-front panel path; both give the oracle's pivots (well conditioned, 1e-12)."""
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = block_angular_k2(900, 1800, 6, 11, well=True)
    N = K.shape[0]
    ls = HIPLDLSolver(N, Lw.indptr, Lw.indices, small_front_max=sfm, ordering=1)
    dev = torch.device("cuda:0")
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).to(dev)) == 0
    ref = OracleLDL(K, ls.perm())
    assert ref.factorize() == N
    _check_pivots(ls.diag(), ref.diag(), K)


@pytest.mark.parametrize("case", ["block", "qp_dense_front", "batched_leaves"])
def test_alg_bytes_sum_to_survey_counts(case):
    """bench.py's roofline prices a launch by SURVEY 8(d)'s algorithmic bytes (madipm_kstat.alg_bytes):
    over one factorisation the launches' alg_bytes add up to exactly 8 nnzL + 12 nnzK, and over one solve
    to 2 x 8 nnzL (every column factorised / substituted once, by exactly one launch)."""
    from madipm_amd.linear_solver import HIPLDLSolver
    if case == "block":
        K, Lw = block_angular_k2(3000, 4000, 20, 7)
        kw = {}
    elif case == "qp_dense_front":
        K, Lw = random_k2(150, 400, 0.05, 11, qp=True)
        kw = {}
    else:
        K, Lw = _dense_k2(150, 1000, 5)
        kw = {"ordering": 0}
    N = K.shape[0]
    ls = HIPLDLSolver(N, Lw.indptr, Lw.indices, **kw)
    info = ls.info()
    if case == "batched_leaves":
        assert info["lb_members"] >= 500
    dev = torch.device("cuda:0")
    vals = torch.from_numpy(Lw.data.copy()).to(dev)
    solve_kinds = {"k_fwd_small", "k_fwd_gather", "k_fwd_big", "k_bwd_below", "k_bwd_big", "k_bwd_small",
                   "k_fwd_tiny", "k_bwd_tiny", "k_lb_gemv", "k_fwd_tree", "k_bwd_tree"}
    ls.set_kernel_timing()
    assert ls.factorize(vals) == 0
    st = ls.kernel_stats()
    fact = sum(k["alg_bytes"] for k in st if k["name"] not in solve_kinds)
    assert fact == pytest.approx(8.0 * info["nnzL"] + 12.0 * info["nnzK"], rel=1e-12), (case, fact)
    ls.set_kernel_timing()
    x = torch.ones(N, dtype=torch.float64, device=dev)
    ls.solve(x)
    st = ls.kernel_stats()
    sol = sum(k["alg_bytes"] for k in st if k["name"] in solve_kinds)
    assert sol == pytest.approx(16.0 * info["nnzL"], rel=1e-12), (case, sol)


@pytest.mark.parametrize("n", [1300, 2500])
def test_fold_many_leaves(n):
    """One tree front folding > 1024 two-row micro leaves: the planner cuts batches of at
    most kFoldLeavesMax leaves, so k_fact_tree folds them without a carve error — the oracle's pivots
    (1e-12) and solution."""
    from helpers import many_leaf_k2
    K, Lw = many_leaf_k2(n)
    ls = _check_case(K, Lw, well=True)
    info = ls.info()
    assert info["fold_fronts"] == 1 and info["fold_leaves"] > 1024, info
    assert ls.inertia() == (n, 0, 1)


def _dense_kkt(n, m, seed=11):
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    B = rng.standard_normal((n, n))
    H = B @ B.T / n + np.eye(n)
    A = rng.standard_normal((m, n))
    K = sp.csc_matrix(np.block([[H, A.T], [A, -1e-2 * np.eye(m)]]))
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


@pytest.mark.parametrize("kpan", ["1", "2", "4"])
@pytest.mark.parametrize("case", ["dense_320_100", "dense_130_200", "dense_700_60", "qp_dense_front", "neos_0.1"])
def test_big_dag_bitwise(case, kpan, monkeypatch):
    """k_big_dag (default, r6): every big front of a level in ONE persistent launch — first diagonal
    blocks, trsm tiles, local updates, the next group's columns as 64 x 64 trailing tiles and the rest as
    128 x 128 tiles — as dependency-ordered tasks (sc1 hand-offs, per-panel M_K slots, dependencies = the
    earlier writers of every rectangle a task reads or rewrites) instead of one launch per panel step and
    kind (MADIPM_BIG_DAG=0).  Same operands and MFMA order as the per-step launches with K unsplit
    (MADIPM_UPD_SPLIT=0): the pivots and the solution agree BITWISE, and with the oracle (1e-12, well
    conditioned).  Dense K2s with partial last panels and groups (420, 330 and 760 columns: misaligned
    trsm rows, trailing tiles straddling the previous group's tiles), a QP with a dense front, and the
    neos stand-in at 0.1 (many big fronts per level, fused fronts)."""
    from helpers import lp_k2
    monkeypatch.setenv("MADIPM_BIG_KPAN", kpan)
    if case.startswith("dense"):
        n, m = map(int, case.split("_")[1:])
        K, Lw = _dense_kkt(n, m)
        sfm = 16
    elif case == "qp_dense_front":
        K, Lw = random_k2(150, 400, 0.05, 11, qp=True, well=True)
        sfm = 128
    else:
        from madipm_amd import standard_form_qp
        from madipm_amd import instances as I
        K, Lw = lp_k2(standard_form_qp(I.neos5052403_standin(scale=0.1)), 2, well=True)
        sfm = 128
    out = {}
    for dag in ("0", "1"):
        monkeypatch.setenv("MADIPM_BIG_DAG", dag)
        monkeypatch.setenv("MADIPM_UPD_SPLIT", "0")
        out[dag] = _factor_solve(K, Lw, sfm)
    (d0, x0, ls0), (d1, x1, _) = out["0"], out["1"]
    assert ls0.info()["nbig"] >= 1
    bad = np.flatnonzero(d0.view(np.uint64) != d1.view(np.uint64))
    assert bad.size == 0, f"{bad.size} pivots differ, first {bad[:8]}"
    assert np.array_equal(x0.view(np.uint64), x1.view(np.uint64))
    ref = OracleLDL(K, ls0.perm())
    assert ref.factorize() == K.shape[0]
    _check_pivots(d1, ref.diag(), K)
