"""Seeded synthetic instances (host side; data generators, not solver code).

No MIPLIB/netlib MPS files exist in this environment, so the benchmark configs of
BASELINE.json are served by seeded, *structured* stand-ins with the catalogue shapes, built to be
primal feasible and dual bounded: b = A x0 with x0 interior, c = A^T y0 + z0 with z0 >= 0.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp

from .qp import QuadraticModel

INF = math.inf


def random_lp(m, n, density=0.05, seed=0, ub_frac=0.5, ineq_frac=0.0, free_frac=0.0) -> QuadraticModel:
    """Feasible, bounded random sparse LP: min c'x, lcon <= Ax <= ucon, lvar <= x <= uvar."""
    rng = np.random.default_rng(seed)
    A = sp.random(m, n, density=density, random_state=rng, format="coo")
    A.data[:] = rng.standard_normal(A.nnz)
    # every row / column non-empty
    rows = np.concatenate([A.row, np.arange(m), rng.integers(0, m, n)])
    cols = np.concatenate([A.col, rng.integers(0, n, m), np.arange(n)])
    vals = np.concatenate([A.data, rng.standard_normal(m), rng.standard_normal(n)])
    A = sp.coo_matrix((vals, (rows, cols)), shape=(m, n)).tocsr().tocoo()
    lvar = np.zeros(n)
    uvar = np.where(rng.random(n) < ub_frac, rng.uniform(1.0, 5.0, n), INF)
    free = rng.random(n) < free_frac
    lvar[free] = -INF
    uvar[free] = INF
    x0 = np.where(np.isfinite(uvar), uvar * rng.uniform(0.2, 0.8, n), rng.uniform(0.5, 2.0, n))
    x0[free] = rng.standard_normal(free.sum())
    b = A @ x0
    y0 = rng.standard_normal(m)
    z0 = rng.uniform(0.0, 1.0, n)
    z0[free] = 0.0
    c = A.T @ y0 + z0
    lcon, ucon = b.copy(), b.copy()
    ineq = rng.random(m) < ineq_frac
    lcon[ineq] = b[ineq] - rng.uniform(0.1, 1.0, ineq.sum())
    ucon[ineq] = np.where(rng.random(ineq.sum()) < 0.5, INF, b[ineq] + rng.uniform(0.1, 1.0, ineq.sum()))
    return QuadraticModel(c=c, Hrows=[], Hcols=[], Hvals=[], Arows=A.row, Acols=A.col, Avals=A.data,
                          lcon=lcon, ucon=ucon, lvar=lvar, uvar=uvar, name=f"random_lp_{m}x{n}_s{seed}")


def random_qp(m, n, density=0.05, seed=0, hdens=None, box=True) -> QuadraticModel:
    """Convex QP: H = diag(U[1e-2,1]) + sparse B B^T (PSD), box-bounded, b = A x0."""
    rng = np.random.default_rng(seed)
    base = random_lp(m, n, density, seed, ub_frac=1.0 if box else 0.0)
    hd = hdens if hdens is not None else min(1.0, 2.0 / n)
    B = sp.random(n, max(1, n // 4), density=hd, random_state=rng)
    H = sp.diags(rng.uniform(1e-2, 1.0, n)) + (B @ B.T)
    H = sp.tril(H).tocoo()
    return QuadraticModel(c=base.c, Hrows=H.row, Hcols=H.col, Hvals=H.data, Arows=base.Arows, Acols=base.Acols,
                          Avals=base.Avals, lcon=base.lcon, ucon=base.ucon, lvar=base.lvar, uvar=base.uvar,
                          name=f"random_qp_{m}x{n}_s{seed}")


def dense_dummy_qp(n, m, seed=1, fixed=(), eq=()) -> QuadraticModel:
    """Structural stand-in for MadNLPTests.DenseDummyQP (test/runtests.jl:10-27): dense PSD Hessian
    P P^T, dense random A, x in [0, 1], constraints in [-1, 1] (rows in `eq` become equalities,
    variables in `fixed` are fixed).  Julia's RNG stream cannot be reproduced, so values differ."""
    rng = np.random.default_rng(seed)
    P = rng.standard_normal((n, n))
    q = rng.standard_normal(n)
    Hd = P @ P.T
    A = rng.standard_normal((m, n))
    Hl = np.tril(Hd)
    r, c = np.nonzero(Hl)
    ar, ac = np.nonzero(A)
    lvar, uvar = np.zeros(n), np.ones(n)
    lcon, ucon = -np.ones(m), np.ones(m)
    x0 = np.full(n, 0.5)
    g = A @ x0
    lcon = np.minimum(lcon, g - 0.5)
    ucon = np.maximum(ucon, g + 0.5)
    for i in eq:
        lcon[i] = ucon[i] = g[i]
    for i in fixed:
        lvar[i] = uvar[i] = 0.5
    return QuadraticModel(c=q, Hrows=r, Hcols=c, Hvals=Hl[r, c], Arows=ar, Acols=ac, Avals=A[ar, ac],
                          lcon=lcon, ucon=ucon, lvar=lvar, uvar=uvar, x0=np.zeros(n), name=f"densedummy_{n}_{m}")


def block_angular_lp(nblocks, rows_per_block, cols_per_block, ncoupling, nnz_per_row, seed=0,
                     ub_frac=1.0, coupling_density=0.02, name="block_angular") -> QuadraticModel:
    """Block-angular LP (independent diagonal blocks + dense-ish coupling rows), equality form."""
    rng = np.random.default_rng(seed)
    m = nblocks * rows_per_block + ncoupling
    n = nblocks * cols_per_block
    R, Cc = [], []
    for b in range(nblocks):
        r0, c0 = b * rows_per_block, b * cols_per_block
        rr = np.repeat(np.arange(rows_per_block) + r0, nnz_per_row)
        cc = rng.integers(c0, c0 + cols_per_block, rows_per_block * nnz_per_row)
        R.append(rr)
        Cc.append(cc)
        # make every column of the block appear
        R.append(rng.integers(r0, r0 + rows_per_block, cols_per_block))
        Cc.append(np.arange(cols_per_block) + c0)
    k = max(1, int(coupling_density * n))
    for j in range(ncoupling):
        R.append(np.full(k, nblocks * rows_per_block + j))
        Cc.append(rng.choice(n, k, replace=False))
    rows = np.concatenate(R)
    cols = np.concatenate(Cc)
    vals = np.where(rng.random(len(rows)) < 0.5, rng.choice([-1.0, 1.0], len(rows)), rng.standard_normal(len(rows)))
    A = sp.coo_matrix((vals, (rows, cols)), shape=(m, n)).tocsr().tocoo()
    lvar = np.zeros(n)
    uvar = np.where(rng.random(n) < ub_frac, 1.0, INF)
    x0 = np.where(np.isfinite(uvar), rng.uniform(0.2, 0.8, n), rng.uniform(0.5, 2.0, n))
    b = A @ x0
    y0 = rng.standard_normal(m)
    z0 = rng.uniform(0.0, 1.0, n)
    c = A.T @ y0 + z0
    return QuadraticModel(c=c, Hrows=[], Hcols=[], Hvals=[], Arows=A.row, Acols=A.col, Avals=A.data,
                          lcon=b, ucon=b.copy(), lvar=lvar, uvar=uvar, name=name)


def packing_lp(nblocks, rows_per_block, cols_per_block, ncoupling, nnz_per_row, seed=0,
               coupling_density=0.01, name="packing") -> QuadraticModel:
    """Set-packing-like LP relaxation: max w'x s.t. A x <= b (0/1 A, small integer b), 0 <= x <= 1.

    Rows are grouped in diagonal blocks with a few long coupling rows.  Feasible (x = 0) and
    bounded (box), with a non-trivial optimal face because b is tight for a random x0."""
    rng = np.random.default_rng(seed)
    m = nblocks * rows_per_block + ncoupling
    n = nblocks * cols_per_block
    R, Cc = [], []
    for b in range(nblocks):
        r0, c0 = b * rows_per_block, b * cols_per_block
        R.append(np.repeat(np.arange(rows_per_block) + r0, nnz_per_row))
        Cc.append(rng.integers(c0, c0 + cols_per_block, rows_per_block * nnz_per_row))
        R.append(rng.integers(r0, r0 + rows_per_block, cols_per_block))
        Cc.append(np.arange(cols_per_block) + c0)
    k = max(2, int(coupling_density * n))
    for j in range(ncoupling):
        R.append(np.full(k, nblocks * rows_per_block + j))
        Cc.append(rng.choice(n, k, replace=False))
    rows = np.concatenate(R)
    cols = np.concatenate(Cc)
    A = sp.coo_matrix((np.ones(len(rows)), (rows, cols)), shape=(m, n)).tocsr()
    A.data[:] = 1.0                       # duplicates collapse to a 0/1 matrix
    A = A.tocoo()
    x0 = rng.uniform(0.0, 0.15, n)
    b = np.ceil(A @ x0)
    w = rng.uniform(0.5, 1.5, n)
    return QuadraticModel(c=w, Hrows=[], Hcols=[], Hvals=[], Arows=A.row, Acols=A.col, Avals=A.data,
                          lcon=np.full(m, -INF), ucon=b, lvar=np.zeros(n), uvar=np.ones(n),
                          minimize=False, name=name)


def ex10_standin(seed=0, scale=1.0) -> QuadraticModel:
    """MIPLIB ex10 LP-relaxation stand-in (BASELINE.json configs[1]): ~69.6k rows x 17.7k binary
    columns, ~1.16M nnz, 0/1 coefficients (catalogue shape, recalled).  136 blocks of
    511 rows x 130 columns at 16 nnz/row, plus 120 coupling rows.  After standard_form_qp:
    ~105k variables, ~87k constraints (K2 of order ~192k)."""
    nblocks = max(2, int(round(136 * scale)))
    return packing_lp(nblocks=nblocks, rows_per_block=511, cols_per_block=130, ncoupling=120,
                      nnz_per_row=16, seed=seed, coupling_density=0.004, name=f"ex10_standin_s{seed}")


def dense_qp(n=50_000, m=10_000, seed=0) -> QuadraticModel:
    """BASELINE.json configs[2]: random dense convex QP, A dense N(0,1) (m x n), H = diag(U[1e-2,1]),
    0 <= x <= 10, b = A x0 with x0 ~ U[0,10] (feasible), c ~ N(0,1).  Generated in float64 with int32
    COO indices, column-major (A's columns contiguous), so the full size (5e8 entries) stays ~8 GB."""
    rng = np.random.default_rng(seed)
    x0 = rng.uniform(0.0, 10.0, n)
    h = rng.uniform(1e-2, 1.0, n)
    c = rng.standard_normal(n)
    vals = np.empty(m * n)
    b = np.zeros(m)
    cb = max(1, (1 << 24) // m)                       # columns per generation block
    for j0 in range(0, n, cb):
        j1 = min(n, j0 + cb)
        blk = rng.standard_normal((j1 - j0, m))       # rows = columns of A
        vals[j0 * m:j1 * m] = blk.ravel()
        b += blk.T @ x0[j0:j1]
    ar = np.tile(np.arange(m, dtype=np.int32), n)
    ac = np.repeat(np.arange(n, dtype=np.int32), m)
    return QuadraticModel(c=c, Hrows=np.arange(n, dtype=np.int32), Hcols=np.arange(n, dtype=np.int32), Hvals=h,
                          Arows=ar, Acols=ac, Avals=vals, lcon=b, ucon=b.copy(), lvar=np.zeros(n),
                          uvar=np.full(n, 10.0), name=f"dense_qp_{n}x{m}")


def supportcase10_standin(seed=0, scale=1.0, block_scale=1.0) -> QuadraticModel:
    """MIPLIB supportcase10 LP-relaxation stand-in (BASELINE.json configs[3]): ~165.7k rows x 14.8k
    [0,1] columns, ~555k nnz (catalogue shape, recalled) — many short rows.  64 blocks of
    2589 rows x 231 columns at 3 nnz/row + 48 coupling rows.  After standard_form_qp: ~180k variables,
    ~166k constraints (K2 of order ~346k): the large, HBM-bound KKT of the north star."""
    nblocks = max(2, int(round(64 * scale)))
    return packing_lp(nblocks=nblocks, rows_per_block=max(8, int(2589 * block_scale)),
                      cols_per_block=max(4, int(231 * block_scale)), ncoupling=max(2, int(48 * block_scale)),
                      nnz_per_row=3, seed=seed, coupling_density=0.002, name=f"supportcase10_standin_s{seed}")


def neos5052403_standin(seed=0, scale=1.0, block_scale=1.0) -> QuadraticModel:
    """MIPLIB neos-5052403-cygnet LP-relaxation stand-in (BASELINE.json configs[4]): ~38.3k rows x
    32.9k columns, ~4.9M nnz (catalogue shape, recalled) — dense rows, wide separators: the config the
    north star shards across GPUs.  16 blocks of 2370 rows x 2054 columns at 120 nnz/row + 348
    coupling rows (1% dense)."""
    nblocks = max(2, int(round(16 * scale)))
    return packing_lp(nblocks=nblocks, rows_per_block=max(8, int(2370 * block_scale)),
                      cols_per_block=max(8, int(2054 * block_scale)), ncoupling=max(2, int(348 * block_scale)),
                      nnz_per_row=max(4, int(120 * block_scale)), seed=seed, coupling_density=0.01,
                      name=f"neos5052403_standin_s{seed}")
