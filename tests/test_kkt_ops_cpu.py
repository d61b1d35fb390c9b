"""Host-side parts of the array-type overrides (csrc/kkt.hip) against the oracle's restatement
(oracle/kkt_ops.py): `build_normal_system` runs on the host in the reference's GPU path too
(src/KKT/normalkkt.jl:104), so it is checked here bit for bit; the symbolic analysis accepts either
triangle of K (LDLFactorizations takes the upper one, MadNLP's aug_com the lower one)."""
import numpy as np
import pytest
import scipy.sparse as sp

from helpers import random_k2


def _random_csr(m, n, dens, seed, dense_rows=0):
    rng = np.random.default_rng(seed)
    A = sp.random(m, n, density=dens, format="csr", random_state=rng)
    if dense_rows:
        D = sp.lil_matrix((m, n))
        for r in rng.choice(m, dense_rows, replace=False):
            D[r, :] = rng.standard_normal(n)
        A = (A + D.tocsr()).tocsr()
    A.sort_indices()
    return A


@pytest.mark.parametrize("m,n,dens,seed,dr", [(1, 1, 1.0, 0, 0), (7, 5, 0.3, 1, 0), (60, 90, 0.05, 2, 0),
                                              (120, 80, 0.02, 3, 2), (50, 40, 0.0, 4, 0)])
def test_build_normal_system_matches_reference_loop(m, n, dens, seed, dr):
    from madipm_amd.rocm_wrapper import build_normal_system
    from oracle import kkt_ops as O
    A = _random_csr(m, n, dens, seed, dr)
    Cp, Cj = build_normal_system(m, n, A.indptr, A.indices)
    Rp, Rj = O.build_normal_system(m, n, A.indptr.tolist(), A.indices.tolist())
    assert np.array_equal(Cp, Rp) and np.array_equal(Cj, Rj)
    # it is the lower pattern of A A'
    S = sp.tril((abs(A) @ abs(A).T) != 0).tocsc()
    S.sort_indices()
    assert np.array_equal(S.indptr, Cp) and np.array_equal(S.indices, Cj)


def test_build_normal_system_capacity_error():
    from madipm_amd import _lib as L
    import ctypes as C
    A = _random_csr(10, 10, 0.3, 0)
    Jp, Jj = A.indptr.astype(np.int32), A.indices.astype(np.int32)
    Cp = np.zeros(11, np.int32)
    Cj = np.zeros(1, np.int32)
    nnz = C.c_int64()
    from madipm_amd import rocm_wrapper  # noqa: F401  (declares the signatures)
    rc = L.lib.madipm_build_normal_system(10, 10, L.ptr(Jp, C.c_int32), L.ptr(Jj, C.c_int32), L.ptr(Cp, C.c_int32),
                                          L.ptr(Cj, C.c_int32), 1, C.byref(nnz))
    assert rc == -4 and nnz.value > 1 and b"cap" in L.madipm_last_error()


@pytest.mark.parametrize("ordering", [0, 1, 3])
def test_symbolic_upper_triangle_same_plan(ordering):
    """The upper triangle (and a mixed one) of K gives the same ordering and nnz(L) as the lower."""
    from madipm_amd._lib import Symbolic, default_ldl_opts
    K, Lw = random_k2(60, 90, 0.05, 5)
    N = K.shape[0]
    U = sp.triu(K).tocsc()
    U.sort_indices()
    low = Symbolic(N, Lw.indptr, Lw.indices, default_ldl_opts(ordering=ordering))
    up = Symbolic(N, U.indptr, U.indices, default_ldl_opts(ordering=ordering))
    assert np.array_equal(low.perm(), up.perm())
    assert low.info()["nnzL"] == up.info()["nnzL"]
    # mixed: every other off-diagonal pair moved to the other triangle
    T = sp.tril(K, -1).tocoo()
    flip = np.arange(T.nnz) % 2 == 1
    r = np.where(flip, T.col, T.row)
    c = np.where(flip, T.row, T.col)
    M = sp.csc_matrix((np.r_[T.data, K.diagonal()], (np.r_[r, np.arange(N)], np.r_[c, np.arange(N)])), shape=(N, N))
    M.sort_indices()
    mix = Symbolic(N, M.indptr, M.indices, default_ldl_opts(ordering=ordering))
    assert mix.info()["nnzL"] == low.info()["nnzL"]
