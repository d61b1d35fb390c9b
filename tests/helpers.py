"""Shared test helpers: seeded KKT matrices and problem generators (test data only)."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def random_k2(m, n, density, seed, delta=1e-8, qp=False, well=False):
    """K2 = [H + Sigma, A^T; A, -delta I] with Sigma in [1e-2, 1e2]: quasi-definite.
    well=True: delta = 1e-2, Sigma in [0.1, 10] (O(1) element growth)."""
    rng = np.random.default_rng(seed)
    A = sp.random(m, n, density=density, random_state=rng, format="csr")
    A.data[:] = rng.standard_normal(A.nnz)
    sig = 10.0 ** rng.uniform(-1, 1, n) if well else 10.0 ** rng.uniform(-2, 2, n)
    if well:
        delta = 1e-2
    H = sp.diags(sig)
    if qp:
        B = sp.random(n, n, density=min(1.0, 3.0 / n), random_state=rng)
        H = H + B @ B.T
    K = sp.bmat([[H, A.T], [A, -delta * sp.eye(m)]]).tocsc()
    K.sum_duplicates()
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


def block_angular_k2(m, n, nblocks, seed, coupling=0.02, delta=1e-8, well=False):
    """Structured stand-in: block-angular A with a few coupling rows."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    bn = n // nblocks
    for i in range(m):
        b = (i * nblocks) // m
        c = rng.integers(b * bn, (b + 1) * bn, size=6)
        if rng.random() < coupling:
            c = np.concatenate([c, rng.integers(0, n, size=20)])
        rows += [i] * len(c)
        cols += list(c)
    A = sp.csr_matrix((rng.standard_normal(len(rows)), (rows, cols)), shape=(m, n))
    A.sum_duplicates()
    sig = 10.0 ** rng.uniform(-1, 1, n) if well else 10.0 ** rng.uniform(-2, 2, n)
    if well:
        delta = 1e-2
    K = sp.bmat([[sp.diags(sig), A.T], [A, -delta * sp.eye(m)]]).tocsc()
    K.sum_duplicates()
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


def dense_k2(m, n, seed, delta=1e-2):
    """K2 of a QP with diagonal H and dense A (m x n): the x_j are single-column leaves with m-row
    updates (batched leaves); returns (K, lower CSC with sorted indices)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((m, n))
    sig = 10.0 ** rng.uniform(-1, 1, n)
    K = sp.bmat([[sp.diags(sig), sp.csr_matrix(A.T)], [sp.csr_matrix(A), -delta * sp.eye(m)]]).tocsc()
    K.sum_duplicates()
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


def lp_k2(qp, seed, well=False, delta=1e-8):
    """K2 = [Sigma, A^T; A, -delta I] on the constraint matrix of a QuadraticModel (the benchmark
    stand-ins' structure: their fronts), Sigma as random_k2; returns (K, lower CSC sorted)."""
    rng = np.random.default_rng(seed)
    m, n = qp.ncon, qp.nvar
    A = sp.csr_matrix((np.asarray(qp.Avals, float), (np.asarray(qp.Arows), np.asarray(qp.Acols))), shape=(m, n))
    A.sum_duplicates()
    sig = 10.0 ** rng.uniform(-1, 1, n) if well else 10.0 ** rng.uniform(-2, 2, n)
    if well:
        delta = 1e-2
    K = sp.bmat([[sp.diags(sig), A.T], [A, -delta * sp.eye(m)]]).tocsc()
    K.sum_duplicates()
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


def kkt_properties(qp, st):
    """Optimality measures of (x, y, zl, zu) for min/max c'x + x'Hx/2 + c0, Ax = b, l <= x <= u
    (unscaled).  The multipliers are those of the problem the solver minimises, sigma f with
    sigma = +1 (minimise) / -1 (maximise) (MadNLP's objective sign [EXT]; the reference flips only the
    reported objective back, /root/reference/src/utils.jl:150-156): stationarity
    sigma (c + Hx) + A'y - zl + zu = 0, and the dual bound of min sigma f,
    sigma c0 - y'b + zl'l - zu'u - sigma x'Hx/2 (src/kernels.jl:408-430), is reported in the
    problem's own sense (times sigma) so that it compares with the primal objective."""
    import scipy.sparse as sp
    n, m = qp.nvar, qp.ncon
    sg = 1.0 if getattr(qp, "minimize", True) else -1.0
    A = sp.csr_matrix((qp.Avals, (qp.Arows, qp.Acols)), shape=(m, n))
    x, y, zl, zu = st.solution, st.multipliers, st.multipliers_L, st.multipliers_U
    hx = np.zeros(n)
    np.add.at(hx, qp.Hrows, qp.Hvals * x[qp.Hcols])
    off = qp.Hrows != qp.Hcols
    np.add.at(hx, qp.Hcols[off], qp.Hvals[off] * x[qp.Hrows[off]])
    b = qp.lcon
    pr = np.max(np.abs(A @ x - b)) / (1.0 + np.max(np.abs(b)))
    g = sg * (qp.c + hx)
    du = np.max(np.abs(g + A.T @ y - zl + zu)) / (1.0 + np.max(np.abs(qp.c)))
    lo, hi = np.isfinite(qp.lvar), np.isfinite(qp.uvar)
    compl = max(np.max(np.abs((x - qp.lvar)[lo] * zl[lo]), initial=0.0),
                np.max(np.abs((qp.uvar - x)[hi] * zu[hi]), initial=0.0))
    pobj = qp.c0 + qp.c @ x + 0.5 * x @ hx
    dobj = sg * (sg * qp.c0 - y @ b + zl[lo] @ qp.lvar[lo] - zu[hi] @ qp.uvar[hi] - sg * 0.5 * x @ hx)
    return dict(pr=pr, du=du, compl=compl, pobj=pobj, dobj=dobj,
                bounds=max(np.max((qp.lvar - x)[lo], initial=-1.0), np.max((x - qp.uvar)[hi], initial=-1.0)),
                zmin=min(np.min(zl[lo], initial=0.0), np.min(zu[hi], initial=0.0)))


def many_leaf_k2(n, seed=0):
    """K2 of an LP with one constraint row over n columns (delta = 1e-2, well conditioned): every x_j is
    a two-row micro leaf (x_j, y) under the one tree front y, which folds all n of them — more than
    k_fact_tree's fold_leaves holds per batch (2 x 512 leaf-table registers) once n > 1024."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    A = sp.csr_matrix(rng.uniform(0.5, 1.5, (1, n)))
    K = sp.bmat([[sp.diags(10.0 ** rng.uniform(-1, 1, n)), A.T], [A, -1e-2 * sp.eye(1)]]).tocsc()
    K.sum_duplicates()
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw
