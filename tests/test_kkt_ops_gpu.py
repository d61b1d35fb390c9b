"""Array-type overrides (csrc/kkt.hip, the ROCArray counterparts of ext/MadIPMCUDAExt) through the
C-ABI against the oracle's restatement of the reference's CPU methods (oracle/kkt_ops.py).

Tolerances: transfer!, compress_jacobian!, coo_to_csr, fill_structure and assemble_normal_system!
follow the reference CPU loops' order and rounding: BIT-EXACT.  The SpMV operator and the QP
evaluators sum rows in a fixed order of their own (cuSPARSE's order is unspecified in the
reference): 1e-14 relative to the row's absolute sum.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = torch.device("cuda:0")


def _t(a, dtype=None):
    a = np.ascontiguousarray(a)
    t = torch.from_numpy(a.copy())
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def _np(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _random_csr(m, n, dens, seed):
    rng = np.random.default_rng(seed)
    A = sp.random(m, n, density=dens, format="csr", random_state=rng, data_rvs=rng.standard_normal)
    A.sort_indices()
    return A


@pytest.mark.parametrize("nsrc,ndest,seed", [(0, 5, 0), (1, 1, 1), (1000, 300, 2), (200_000, 50_000, 3)])
def test_transfer_bitexact(nsrc, ndest, seed):
    from madipm_amd.rocm_wrapper import Transfer
    from oracle import kkt_ops as O
    rng = np.random.default_rng(seed)
    mp = rng.integers(0, ndest, nsrc).astype(np.int64)        # duplicates: scatter-ADD
    src = rng.standard_normal(nsrc) * 10.0 ** rng.integers(-8, 8, nsrc)
    ref = O.transfer(ndest, src, mp.tolist()) if nsrc <= 1000 else None
    if ref is None:  # large case: the same ascending-k sums, vectorised per destination
        order = np.argsort(mp, kind="stable")
        ref = np.zeros(ndest)
        for k in order:
            ref[mp[k]] += src[k]
    dest = torch.full((ndest,), 7.0, dtype=torch.float64, device=DEV)   # stale values are overwritten
    for dev_map in (False, True):
        T = Transfer(_t(mp) if dev_map else mp, ndest)
        T(dest, _t(src))
        assert np.array_equal(_np(dest), ref)


def test_compress_jacobian_bitexact():
    from madipm_amd.rocm_wrapper import compress_jacobian
    from oracle import kkt_ops as O
    rng = np.random.default_rng(0)
    nnz, ns = 5000, 300
    AV = rng.standard_normal(nnz)
    cmap = rng.permutation(nnz).astype(np.int64)
    refAV, refAT = O.compress_jacobian(AV, ns, cmap)
    dAV, dAT = _t(AV), torch.zeros(nnz, dtype=torch.float64, device=DEV)
    compress_jacobian(dAV, ns, _t(cmap), dAT)
    assert np.array_equal(_np(dAV), refAV) and np.array_equal(_np(dAT), refAT)


@pytest.mark.parametrize("m,n,nnz,seed", [(1, 1, 0, 0), (5, 7, 12, 1), (300, 200, 4000, 2), (20000, 30000, 400_000, 3)])
def test_coo_to_csr_bitexact(m, n, nnz, seed):
    from madipm_amd.rocm_wrapper import coo_to_csr
    from oracle import kkt_ops as O
    rng = np.random.default_rng(seed)
    Ai = rng.integers(0, m, nnz).astype(np.int32)
    Aj = rng.integers(0, n, nnz).astype(np.int32)
    Ax = rng.standard_normal(nnz)
    if nnz <= 4000:
        Rp, Rj, Rx = O.coo_to_csr(m, n, Ai.tolist(), Aj.tolist(), Ax)
    else:  # stable counting sort by row == a stable argsort by row
        o = np.argsort(Ai, kind="stable")
        Rp = np.r_[0, np.cumsum(np.bincount(Ai, minlength=m))].astype(np.int32)
        Rj, Rx = Aj[o], Ax[o]
    Bp, Bj, Bx = coo_to_csr(m, n, _t(Ai), _t(Aj), _t(Ax))
    assert np.array_equal(_np(Bp), Rp) and np.array_equal(_np(Bj), Rj) and np.array_equal(_np(Bx), Rx)
    # sort_cols: the rows' entries by ascending column, ties in input order (cuSPARSE layout)
    o = np.lexsort((np.arange(nnz), Aj, Ai))
    Bp, Bj, Bx = coo_to_csr(m, n, _t(Ai), _t(Aj), _t(Ax), sort_cols=True)
    assert np.array_equal(_np(Bp), Rp) and np.array_equal(_np(Bj), Aj[o]) and np.array_equal(_np(Bx), Ax[o])


def test_coo_to_csr_rejects_out_of_range():
    """An index outside [0, n_rows) x [0, n_cols) is reported, not turned into a corrupt CSR."""
    from madipm_amd.rocm_wrapper import coo_to_csr
    Ax = np.ones(3)
    for Ai, Aj in (([0, 5, 1], [0, 1, 2]), ([0, 1, 1], [0, -1, 2]), ([0, 1, 1], [0, 1, 3])):
        with pytest.raises(Exception, match="out of range"):
            coo_to_csr(4, 3, _t(np.array(Ai, np.int32)), _t(np.array(Aj, np.int32)), _t(Ax))


def test_fill_structure_exact():
    from madipm_amd.rocm_wrapper import fill_structure
    from oracle import kkt_ops as O
    A = _random_csr(500, 300, 0.02, 1)
    rows = torch.zeros(A.nnz, dtype=torch.int32, device=DEV)
    cols = torch.zeros(A.nnz, dtype=torch.int32, device=DEV)
    fill_structure(500, _t(A.indptr.astype(np.int32)), _t(A.indices.astype(np.int32)), rows, cols)
    rr, rc = O.fill_structure(500, A.indptr, A.indices)
    assert np.array_equal(_np(rows), rr) and np.array_equal(_np(cols), rc)


@pytest.mark.parametrize("m,n,dens,seed", [(40, 60, 0.1, 0), (400, 900, 0.01, 1), (3000, 8000, 0.002, 2)])
def test_assemble_normal_system_bitexact(m, n, dens, seed):
    from madipm_amd.rocm_wrapper import build_normal_system, assemble_normal_system
    from oracle import kkt_ops as O
    A = _random_csr(m, n, dens, seed)
    Cp, Cj = build_normal_system(m, n, A.indptr, A.indices)
    D = np.random.default_rng(seed).uniform(0.1, 10.0, n)
    Cx = torch.full((len(Cj),), np.nan, dtype=torch.float64, device=DEV)
    assemble_normal_system(m, n, _t(A.indptr.astype(np.int32)), _t(A.indices.astype(np.int32)), _t(A.data),
                           _t(Cp), _t(Cj), Cx, _t(D))
    got = _np(Cx)
    if m <= 400:
        ref = O.assemble_normal_system(m, n, A.indptr.tolist(), A.indices.tolist(), A.data.tolist(),
                                       Cp.tolist(), Cj.tolist(), D)
        assert np.array_equal(got, ref)
    # and it is A D A' on the lower pattern
    C = sp.tril(A @ sp.diags(D) @ A.T).tocsc()
    ref2 = np.asarray(C[Cj, np.repeat(np.arange(m), np.diff(Cp))]).ravel()
    assert np.allclose(got, ref2, rtol=1e-13, atol=1e-13 * np.abs(ref2).max())


@pytest.mark.parametrize("transa,symmetric", [("N", False), ("T", False), ("N", True)])
def test_operator_mul(transa, symmetric):
    from madipm_amd.rocm_wrapper import MadIPMOperator
    from oracle import kkt_ops as O
    rng = np.random.default_rng(3)
    m, n = (700, 700) if symmetric else (700, 1100)
    A = _random_csr(m, n, 0.01, 4)
    if symmetric:
        A = sp.tril(A).tocsr()
        A.sort_indices()
    dp, dj, dx = _t(A.indptr.astype(np.int32)), _t(A.indices.astype(np.int32)), _t(A.data)
    op = MadIPMOperator(m, n, dp, dj, dx, transa=transa, symmetric=symmetric)
    assert op.shape == (m, n) and op.nnz() == A.nnz
    M = O.operator_matrix(m, n, A.indptr, A.indices, A.data, transa, symmetric)
    x = rng.standard_normal(M.shape[1])
    y0 = rng.standard_normal(M.shape[0])
    scale = abs(M) @ abs(x) + abs(y0) + 1e-300
    for alpha, beta in ((1.0, 0.0), (1.0, -1.0), (-0.5, 2.0)):
        y = _t(y0)
        op.mul(y, _t(x), alpha, beta)
        ref = alpha * (M @ x) + beta * y0
        assert np.all(np.abs(_np(y) - ref) <= 1e-14 * scale * max(1.0, abs(alpha), abs(beta)))
    if not symmetric:  # 'N' and 'T' read the caller's values live (cuSPARSE descriptors do too)
        dx.mul_(2.0)
        y = torch.zeros(M.shape[0], dtype=torch.float64, device=DEV)
        op.mul(y, _t(x))
        assert np.all(np.abs(_np(y) - 2.0 * (M @ x)) <= 2e-14 * scale)


def test_qp_obj_grad():
    from madipm_amd.rocm_wrapper import MadIPMOperator, qp_obj, qp_grad
    from oracle import kkt_ops as O
    rng = np.random.default_rng(5)
    n = 5000
    H = sp.tril(_random_csr(n, n, 0.001, 6) + sp.eye(n)).tocsr()
    H.sort_indices()
    Hop = MadIPMOperator(n, n, _t(H.indptr.astype(np.int32)), _t(H.indices.astype(np.int32)), _t(H.data),
                         symmetric=True)
    Hm = O.operator_matrix(n, n, H.indptr, H.indices, H.data, "N", True)
    c, x = rng.standard_normal(n), rng.standard_normal(n)
    v = torch.zeros(n, dtype=torch.float64, device=DEV)
    obj = qp_obj(Hop, _t(c), 1.25, _t(x), v)
    ref = O.qp_obj(Hm, c, 1.25, x)
    assert abs(obj - ref) <= 1e-13 * (abs(c) @ abs(x) + abs(Hm) @ abs(x) @ abs(x) + 1.25)
    g = torch.zeros(n, dtype=torch.float64, device=DEV)
    qp_grad(Hop, _t(c), _t(x), g)
    assert np.allclose(_np(g), O.qp_grad(Hm, c, x), rtol=1e-13, atol=1e-13)


def test_normal_kkt_constructor_pipeline():
    """NormalKKTSystem's construction on device arrays (src/KKT/normalkkt.jl:69-111): A_coo with
    values 1..nnz -> coo_to_csr -> A_csr_map; build_normal_system; compress_jacobian!; build_kkt!
    (assemble_normal_system! with D = 1 ./ pr_diag); then the LDL^T of C through the plugin
    boundary — the normal-equations solve equals the dense one."""
    from madipm_amd.rocm_wrapper import (coo_to_csr, build_normal_system, compress_jacobian,
                                         assemble_normal_system)
    from madipm_amd.linear_solver import HIPLDLSolver
    rng = np.random.default_rng(7)
    m, nx, ns = 300, 700, 40
    A = sp.random(m, nx, density=0.02, format="coo", random_state=rng, data_rvs=rng.standard_normal)
    ind_ineq = np.sort(rng.choice(m, ns, replace=False)).astype(np.int32)
    I = np.r_[A.row, ind_ineq].astype(np.int32)
    J = np.r_[A.col, nx + np.arange(ns)].astype(np.int32)
    ntot, nnz = nx + ns, A.nnz + ns
    # A_coo.V .= 1:nnz (0-based here); coo_to_csr; A_csr_map = convert.(Int, Ax)
    Ap, Aj, Ax = coo_to_csr(m, ntot, _t(I), _t(J), _t(np.arange(nnz, dtype=np.float64)), sort_cols=True)
    csr_map = Ax.to(torch.int64)
    Cp, Cj = build_normal_system(m, ntot, _np(Ap), _np(Aj))
    # jac values + compress_jacobian! (slack entries -1)
    V = _t(np.r_[A.data, np.zeros(ns)])
    ATnz = torch.zeros(nnz, dtype=torch.float64, device=DEV)
    compress_jacobian(V, ns, csr_map, ATnz)
    pr = rng.uniform(0.5, 5.0, ntot)
    Cx = torch.zeros(len(Cj), dtype=torch.float64, device=DEV)
    assemble_normal_system(m, ntot, Ap, Aj, ATnz, _t(Cp), _t(Cj), Cx, _t(1.0 / pr))
    Afull = sp.csr_matrix((np.r_[A.data, -np.ones(ns)], (I, J)), shape=(m, ntot))
    Cd = (Afull @ sp.diags(1.0 / pr) @ Afull.T).toarray()
    ls = HIPLDLSolver(m, Cp.astype(np.int64), Cj)
    assert ls.factorize(Cx) == 0
    b = rng.standard_normal(m)
    xb = _t(b)
    ls.solve(xb)
    xr = np.linalg.solve(Cd, b)
    assert np.max(np.abs(_np(xb) - xr)) <= 1e-10 * np.max(np.abs(xr))


@pytest.mark.parametrize("which", ["upper", "mixed"])
def test_ldl_either_triangle(which):
    """madipm_ldl_analyze / factorize on the upper triangle (LDLFactorizations' input) or a mixed
    one gives the lower-triangle factorisation's pivots and solution."""
    from helpers import random_k2
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw = random_k2(200, 300, 0.02, 9, well=True)
    N = K.shape[0]
    if which == "upper":
        M = sp.triu(K).tocsc()
    else:
        T = sp.tril(K, -1).tocoo()
        flip = np.arange(T.nnz) % 3 == 0
        M = sp.csc_matrix((np.r_[T.data, K.diagonal()],
                           (np.r_[np.where(flip, T.col, T.row), np.arange(N)],
                            np.r_[np.where(flip, T.row, T.col), np.arange(N)])), shape=(N, N))
    M.sort_indices()
    low = HIPLDLSolver(N, Lw.indptr, Lw.indices)
    oth = HIPLDLSolver(N, M.indptr, M.indices)
    assert low.factorize(_t(Lw.data)) == 0 and oth.factorize(_t(M.data)) == 0
    if which == "upper":  # same adjacency order -> same ordering and pivots (a mixed input may break
        assert np.array_equal(low.perm(), oth.perm())  # AMD's ties differently: same solution only)
        assert np.allclose(low.diag(), oth.diag(), rtol=1e-13, atol=0)
    b = np.random.default_rng(1).standard_normal(N)
    x1, x2 = _t(b), _t(b)
    low.solve(x1)
    oth.solve(x2)
    r1, r2 = _np(x1), _np(x2)
    if which == "upper":
        assert np.max(np.abs(r1 - r2)) <= 1e-12 * np.max(np.abs(r1))
    # both are backward stable solves of K x = b (a different pivot order rounds differently)
    nK = abs(K).sum(axis=1).max()
    for r_ in (r1, r2):
        assert np.max(np.abs(K @ r_ - b)) <= 1e-13 * nK * np.max(np.abs(r_))
    assert low.inertia() == oth.inertia()
