"""CPU tests of host logic and of the C-ABI library (no GPU compute calls).

* every function declared in include/madipm_hip.h is exported by libmadipm_hip.so;
* host-side symbolic analysis (AMD, etree, column counts, supernodes) against the oracle's
  up-looking LDL^T (same order => identical nnz(L)) and a brute-force elimination;
* MPS reader, standard_form_qp (src/utils.jl:373-505), scale_qp, option parsing.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.sparse as sp

from helpers import block_angular_k2, random_k2

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    from madipm_amd import _lib
    header = open(os.path.join(ROOT, "include", "madipm_hip.h")).read()
    header = re.sub(r"/\*.*?\*/", "", header, flags=re.S)
    names = set(re.findall(r"\b(madipm_[a-z0-9_]+)\s*\(", header))
    assert len(names) >= 25
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    assert _lib.madipm_version() == 203


def test_library_reports_errors_without_gpu():
    from madipm_amd import _lib
    o = _lib.default_ldl_opts()
    h = ctypes.c_void_p()
    colptr = np.array([0, 2, 3], np.int64)
    rowval = np.array([1, 0, 1], np.int32)     # (1,0) then (0,0): row 0 in col 0 ok, but unsorted fine
    rc = _lib.madipm_symbolic_analyze(2, _lib.ptr(colptr, ctypes.c_int64), _lib.ptr(rowval, ctypes.c_int32),
                                      ctypes.byref(o), None, ctypes.byref(h))
    assert rc == 0
    _lib.madipm_symbolic_destroy(h)
    rowval2 = np.array([0, 0, 1], np.int32)     # upper triangle (0,0), (0,1), (1,1): accepted
    rc = _lib.madipm_symbolic_analyze(2, _lib.ptr(np.array([0, 1, 3], np.int64), ctypes.c_int64),
                                      _lib.ptr(rowval2, ctypes.c_int32), ctypes.byref(o), None, ctypes.byref(h))
    assert rc == 0
    _lib.madipm_symbolic_destroy(h)
    rowval3 = np.array([0, 1, 0, 1], np.int32)  # full symmetric: (1,0) and (0,1) -> rejected
    rc = _lib.madipm_symbolic_analyze(2, _lib.ptr(np.array([0, 2, 4], np.int64), ctypes.c_int64),
                                      _lib.ptr(rowval3, ctypes.c_int32), ctypes.byref(o), None, ctypes.byref(h))
    assert rc < 0 and b"both triangles" in _lib.madipm_last_error()
    rowval4 = np.array([0, 5], np.int32)        # out of range
    rc = _lib.madipm_symbolic_analyze(2, _lib.ptr(np.array([0, 1, 2], np.int64), ctypes.c_int64),
                                      _lib.ptr(rowval4, ctypes.c_int32), ctypes.byref(o), None, ctypes.byref(h))
    assert rc < 0 and b"out of range" in _lib.madipm_last_error()


def _brute_nnzL(K, perm):
    Kp = (K[perm][:, perm].toarray() != 0)
    N = Kp.shape[0]
    cnt = 0
    for j in range(N):
        rows = np.flatnonzero(Kp[j + 1:, j]) + j + 1
        cnt += 1 + len(rows)
        if len(rows):
            Kp[np.ix_(rows, rows)] = True
    return cnt


@pytest.mark.parametrize("m,n,dens,seed", [(5, 8, 0.3, 0), (30, 50, 0.05, 1), (80, 120, 0.03, 2)])
@pytest.mark.parametrize("ordering", [0, 1])
def test_symbolic_nnzL_brute_force(m, n, dens, seed, ordering):
    from madipm_amd._lib import Symbolic, default_ldl_opts
    K, Lw = random_k2(m, n, dens, seed)
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=ordering))
    perm = S.perm()
    assert sorted(perm.tolist()) == list(range(K.shape[0]))
    assert S.info()["nnzL"] == _brute_nnzL(K, perm)


@pytest.mark.parametrize("relax", [0, 1])
def test_symbolic_matches_oracle_ldl(relax):
    from madipm_amd._lib import Symbolic, default_ldl_opts
    from oracle.ldl import OracleLDL
    K, Lw = block_angular_k2(2000, 3000, 15, 3)
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(relax=relax))
    info = S.info()
    F = OracleLDL(K, S.perm())
    assert F.factorize() == K.shape[0]
    assert F.nnzL() == info["nnzL"]
    assert info["nnzL_stored"] >= info["nnzL"]
    first, parent, nrows = S.supernodes()
    ns = info["nsuper"]
    assert first[0] == 0 and first[-1] == K.shape[0] and np.all(np.diff(first) > 0)
    assert np.all((parent == -1) | (parent > np.arange(ns)))      # postordered front tree
    assert np.all(nrows >= np.diff(first))


def test_amd_beats_natural_order():
    from madipm_amd._lib import Symbolic, default_ldl_opts
    K, Lw = block_angular_k2(3000, 4000, 20, 7)
    nat = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=0)).info()["nnzL"]
    amd = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=1)).info()["nnzL"]
    assert amd < nat / 3


def test_symbolic_rejects_duplicates():
    from madipm_amd._lib import Symbolic, MadIPMError
    with pytest.raises(MadIPMError, match="duplicate"):
        Symbolic(2, np.array([0, 3, 4]), np.array([0, 1, 1, 1]))


def test_read_afiro():
    from madipm_amd import read_mps
    qp = read_mps(os.path.join(ROOT, "tests", "golden", "afiro.mps"))
    assert (qp.ncon, qp.nvar) == (27, 32)
    # netlib lists AFIRO with 88 nonzeros including the 4 objective coefficients
    assert qp.nnzj == 84 and np.count_nonzero(qp.c) == 4
    assert np.all(qp.lvar == 0) and np.all(np.isinf(qp.uvar))


def test_standard_form_shapes():
    """standard_form_qp (src/utils.jl:373-505): slacks for inequality rows, w for range bounds."""
    from madipm_amd import QuadraticModel, standard_form_qp
    inf = np.inf
    qp = QuadraticModel(c=[1.0, 2.0, 3.0], Hrows=[], Hcols=[], Hvals=[], Arows=[0, 0, 1, 2], Acols=[0, 1, 1, 2],
                        Avals=[1.0, 1.0, 1.0, 1.0], lcon=[1.0, -inf, 0.0], ucon=[1.0, 4.0, 2.0],
                        lvar=[0.0, 0.0, -1.0], uvar=[inf, 5.0, 1.0])
    s = standard_form_qp(qp)
    # ineq rows: 1 (only ub), 2 (range) -> ns = 2; range bounds: x1 (0..5), x2 (-1..1), s_row2 (0..2) -> nw = 3
    assert s.nvar == 3 + 2 + 3 and s.ncon == 3 + 3
    assert np.all(s.lcon == s.ucon)                         # all equalities
    assert np.all(s.lvar[5:] == 0) and np.all(np.isinf(s.uvar[5:]))
    assert s.nnzj == qp.nnzj + 2 + 2 * 3


def test_scale_qp_equilibrates():
    from madipm_amd import scale_qp
    from madipm_amd.instances import random_lp
    qp = random_lp(50, 80, 0.1, 0)
    qp.Avals[:] *= np.exp(np.random.default_rng(0).uniform(-5, 5, qp.nnzj))
    s = scale_qp(qp)
    A = sp.coo_matrix((np.abs(s.Avals), (s.Arows, s.Acols)), shape=(s.ncon, s.nvar)).tocsr()
    assert np.allclose(A.max(axis=1).toarray().ravel(), 1.0, atol=1e-3)
    assert np.allclose(A.max(axis=0).toarray().ravel(), 1.0, atol=1e-3)


def test_options_parsing():
    from madipm_amd.solver import (load_options, FixedRegularization, MehrotraAdaptiveStep, NormalKKTSystem,
                                   ScaledSparseKKTSystem, SparseKKTSystem)
    o = load_options(max_iter=300, regularization=FixedRegularization(1e-8, -1e-8),
                     step_rule=MehrotraAdaptiveStep(0.9), tol=1e-7)
    assert (o.max_iter, o.regularization, o.delta_p, o.delta_d, o.step_rule, o.step_tau, o.tol) == \
        (300, 1, 1e-8, -1e-8, 2, 0.9, 1e-7)
    d = load_options()
    assert (d.tol, d.max_iter, d.mu_init, d.mu_min, d.bound_push, d.delta_p) == (1e-8, 3000, 0.1, 1e-12, 1e-2, 1e-10)
    # unknown options are printed as ignored (MadNLP.print_ignored_options, src/utils.jl:140-142)
    assert load_options(not_an_option=1).max_iter == 3000
    assert [load_options(kkt_system=k).kkt_system for k in (SparseKKTSystem, ScaledSparseKKTSystem, NormalKKTSystem)] \
        == [0, 1, 2]
    with pytest.raises(TypeError):
        load_options(kkt_system=int)


@pytest.mark.parametrize("ordering", [3, 4])
def test_nested_dissection_orderings(ordering):
    """ND (csrc/nd.cpp) is a valid permutation with exact nnz(L) (oracle LDL^T in the same order); on
    a block-angular K2 it beats AMD by a wide margin, and `auto` keeps the cheaper of the two."""
    from madipm_amd._lib import Symbolic, default_ldl_opts
    from oracle.ldl import OracleLDL
    K, Lw = block_angular_k2(2000, 3000, 15, 3)
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=ordering))
    perm = S.perm()
    assert sorted(perm.tolist()) == list(range(K.shape[0]))
    F = OracleLDL(K, perm)
    assert F.factorize() == K.shape[0]
    assert F.nnzL() == S.info()["nnzL"]
    amd = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=1)).info()["flops"]
    nd = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=3)).info()["flops"]
    if ordering == 4:
        assert S.info()["flops"] <= min(amd, nd) * 1.0001


@pytest.mark.parametrize("m,n,dens,seed", [(30, 50, 0.05, 1), (80, 120, 0.03, 2)])
def test_nd_nnzL_brute_force(m, n, dens, seed):
    from madipm_amd._lib import Symbolic, default_ldl_opts
    K, Lw = random_k2(m, n, dens, seed)
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=3))
    assert S.info()["nnzL"] == _brute_nnzL(K, S.perm())


# ---------------------------------------------------------------- presolve_qp (src/utils.jl:319-343)
def test_presolve_simple_lp_flag():
    """test/runtests.jl:154-157: presolve_qp(simple_lp) returns flag == true."""
    from madipm_amd import presolve_qp, simple_lp
    new, flag = presolve_qp(simple_lp())
    assert flag and new.nvar == 2 and new.ncon == 1


def _presolve_case():
    """LP with a fixed variable, an empty row, a singleton row and an empty column."""
    import numpy as np
    from madipm_amd.qp import QuadraticModel
    inf = float("inf")
    # x0 + x1 + x2 = 4 ; x3 fixed = 1 appears in row 0 (x0 + x1 + x2 + x3 = 5) ; row 1 empty ;
    # row 2: 2 x1 <= 6 (singleton) ; x4 empty column with c4 = -1, 0 <= x4 <= 2
    return QuadraticModel(
        c=np.array([1.0, 2.0, 3.0, 5.0, -1.0]), Hrows=[], Hcols=[], Hvals=[],
        Arows=[0, 0, 0, 0, 2], Acols=[0, 1, 2, 3, 1], Avals=[1.0, 1.0, 1.0, 1.0, 2.0],
        lcon=np.array([5.0, -1.0, -inf]), ucon=np.array([5.0, 1.0, 6.0]),
        lvar=np.array([0.0, 0.0, 0.0, 1.0, 0.0]), uvar=np.array([inf, inf, inf, 1.0, 2.0]))


def test_presolve_reductions_and_postsolve():
    import numpy as np
    from madipm_amd import presolve_qp, postsolve
    from oracle.mpc import OracleMPC, OracleOptions
    qp = _presolve_case()
    new, flag = presolve_qp(qp)
    assert flag
    info = new.meta["presolve"]
    assert list(info.keep_var) == [0, 1, 2] and list(info.keep_con) == [0]
    assert new.uvar[1] == 3.0                       # singleton row 2 x1 <= 6 became x1 <= 3
    assert new.lcon[0] == new.ucon[0] == 4.0        # fixed x3 = 1 moved into the row
    ref = OracleMPC(qp, OracleOptions(max_iter=300)).solve()
    sol = OracleMPC(new, OracleOptions(max_iter=300)).solve()
    assert ref.status == sol.status == 1
    assert abs((sol.objective) - ref.objective) <= 1e-7 * max(1.0, abs(ref.objective))
    xo, _ = postsolve(info, sol.solution, sol.multipliers)
    assert np.allclose(xo, ref.solution, atol=1e-6)
    assert xo[3] == 1.0 and xo[4] == 2.0


def test_presolve_detects_infeasible_and_unbounded():
    import numpy as np
    from madipm_amd import presolve_qp
    from madipm_amd.qp import QuadraticModel
    inf = float("inf")
    infeas = QuadraticModel(c=np.ones(1), Hrows=[], Hcols=[], Hvals=[], Arows=[0], Acols=[0], Avals=[1.0],
                            lcon=np.array([5.0]), ucon=np.array([5.0]), lvar=np.zeros(1), uvar=np.array([1.0]))
    assert presolve_qp(infeas)[1] is False
    unb = QuadraticModel(c=np.array([-1.0, 1.0]), Hrows=[], Hcols=[], Hvals=[], Arows=[0], Acols=[1], Avals=[1.0],
                         lcon=np.array([1.0]), ucon=np.array([1.0]), lvar=np.zeros(2), uvar=np.array([inf, inf]))
    assert presolve_qp(unb)[1] is False


def test_presolve_afiro_same_optimum():
    """AFIRO through presolve -> standard form (scripts/benchmarks_cpu.jl:26-41 order): same optimum."""
    import os
    from madipm_amd import presolve_qp, read_mps, standard_form_qp
    from oracle.mpc import OracleMPC, OracleOptions
    qp = read_mps(os.path.join(os.path.dirname(__file__), "golden", "afiro.mps"))
    new, flag = presolve_qp(qp)
    assert flag
    st = OracleMPC(standard_form_qp(new), OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=300)).solve()
    assert st.status == 1 and abs(st.objective + 464.75314286) <= 1e-6 * 464.75


def _presolve_case2():
    """min x0 + 2 x1 + x2^2/2 ... with a free row, a free column singleton in an equality row and an
    unconstrained quadratic variable:
       row 0:  x0 + x1 + x3 = 4        (x3 free, column singleton, cost 3)
       row 1:  x0 - x1 <= 1
       row 2:  -inf <= x0 + x2 <= inf  (free row)
       x4: no A entries, H_44 = 2, c4 = -2, bounds [0, 0.5]  -> x4 = 0.5
    """
    import numpy as np
    from madipm_amd.qp import QuadraticModel
    inf = np.inf
    return QuadraticModel(
        c=np.array([1.0, 2.0, 0.5, 3.0, -2.0]), c0=0.25,
        Hrows=np.array([2, 4]), Hcols=np.array([2, 4]), Hvals=np.array([1.0, 2.0]),
        Arows=np.array([0, 0, 0, 1, 1, 2, 2]), Acols=np.array([0, 1, 3, 0, 1, 0, 2]),
        Avals=np.array([1.0, 1.0, 1.0, 1.0, -1.0, 1.0, 1.0]),
        lcon=np.array([4.0, -inf, -inf]), ucon=np.array([4.0, 1.0, inf]),
        lvar=np.array([0.0, 0.0, 0.0, -inf, 0.0]), uvar=np.array([3.0, 3.0, 2.0, inf, 0.5]))


def test_presolve_free_rows_singleton_columns_unconstrained_quadratic():
    import numpy as np
    from madipm_amd import presolve_qp, postsolve
    from oracle.mpc import OracleMPC, OracleOptions
    qp = _presolve_case2()
    new, flag = presolve_qp(qp)
    assert flag
    info = new.meta["presolve"]
    assert 2 not in info.keep_con                      # free row dropped
    assert 0 not in info.keep_con and 3 not in info.keep_var   # free column singleton + its row
    assert 4 not in info.keep_var and info.xfix[4] == 0.5      # unconstrained quadratic variable
    assert len(info.free_singletons) == 1
    ref = OracleMPC(qp, OracleOptions(max_iter=300)).solve()
    sol = OracleMPC(new, OracleOptions(max_iter=300)).solve()
    assert ref.status == sol.status == 1
    assert abs(sol.objective - ref.objective) <= 1e-7 * max(1.0, abs(ref.objective))
    xo, yo = postsolve(info, sol.solution, sol.multipliers)
    assert np.allclose(xo, ref.solution, atol=1e-6)
    # the recovered row multiplier: stationarity of the free x3 is c3 + a03 y0 = 0
    assert abs(yo[0] - (-3.0)) <= 1e-12
    A = np.zeros((3, 5))
    A[qp.Arows, qp.Acols] = qp.Avals
    assert abs(A[0] @ xo - 4.0) <= 1e-8


def test_presolve_maximize_model():
    """A MAX model (max -f == min f, case2 negated) presolves to the negated min model: same optimum
    (sign-flipped), same postsolved x, and the recovered multipliers in the solver's convention (those of
    min -f: the oracle's multipliers of the original MAX model)."""
    import numpy as np
    from madipm_amd import presolve_qp, postsolve
    from madipm_amd.qp import QuadraticModel
    from oracle.mpc import OracleMPC, OracleOptions
    q = _presolve_case2()
    qmax = QuadraticModel(c=-q.c, c0=-q.c0, Hrows=q.Hrows, Hcols=q.Hcols, Hvals=-q.Hvals, Arows=q.Arows,
                          Acols=q.Acols, Avals=q.Avals, lcon=q.lcon, ucon=q.ucon, lvar=q.lvar, uvar=q.uvar,
                          minimize=False)
    nmin, _ = presolve_qp(q)
    new, flag = presolve_qp(qmax)
    assert flag and not new.minimize
    assert np.array_equal(new.c, -nmin.c) and new.c0 == -nmin.c0 and np.array_equal(new.Hvals, -nmin.Hvals)
    info = new.meta["presolve"]
    assert info.xfix[4] == 0.5                          # the maximiser of -x4^2 + 2 x4 on [0, 0.5]
    ref = OracleMPC(qmax, OracleOptions(max_iter=300)).solve()
    sol = OracleMPC(new, OracleOptions(max_iter=300)).solve()
    assert ref.status == sol.status == 1
    assert abs(sol.objective - ref.objective) <= 1e-7 * max(1.0, abs(ref.objective))
    xo, yo = postsolve(info, sol.solution, sol.multipliers)
    assert np.allclose(xo, ref.solution, atol=1e-6)
    assert abs(yo[0] - (-3.0)) <= 1e-12                 # y of min -f: same as the MIN model's
    assert np.allclose(yo[info.keep_con], ref.multipliers[info.keep_con], atol=1e-5)
    refmin = OracleMPC(q, OracleOptions(max_iter=300)).solve()
    assert np.allclose(ref.multipliers, refmin.multipliers, atol=1e-6)


@pytest.mark.parametrize("ordering", [1, 3, 4])
def test_dense_block_orderings_defer_constraint_vertices(ordering):
    """K2 of a QP with a dense A (m x n, m < n) and a diagonal H: every ordering must eliminate the
    x columns first (batched leaves) and the m constraint vertices last, the optimal fill
    n (m + 1) + m (m + 1) / 2.  Nested dissection defers the dense vertices (csrc/nd.cpp) like AMD."""
    from madipm_amd._lib import Symbolic, default_ldl_opts
    n, m = 300, 40
    N = n + m
    colptr = np.concatenate([np.arange(n + 1, dtype=np.int64) * (m + 1),
                             n * (m + 1) + np.arange(1, m + 1, dtype=np.int64)])
    blk = np.empty((n, m + 1), np.int32)
    blk[:, 0] = np.arange(n)
    blk[:, 1:] = n + np.arange(m)[None, :]
    rows = np.concatenate([blk.ravel(), n + np.arange(m, dtype=np.int32)])
    S = Symbolic(N, colptr, rows, default_ldl_opts(ordering=ordering))
    assert S.info()["nnzL"] == n * (m + 1) + m * (m + 1) // 2
    assert sorted(S.perm()[-m:].tolist()) == list(range(n, N))


def _twin_k2(seed):
    """K2 of an LP-like QP whose x columns come in groups with identical A columns (twin leaves of the
    etree) next to unique ones, a few H couplings (non-leaves) and an empty column."""
    rng = np.random.default_rng(seed)
    n, m = 90, 25
    A = np.zeros((m, n))
    base = [rng.random(m) < 0.3 for _ in range(6)]
    for j in range(n):
        if j % 3 == 0:
            A[:, j] = base[j % 6] * rng.standard_normal(m)         # twins: 6 shared row sets
        elif j != 7:
            A[:, j] = (rng.random(m) < 0.15) * rng.standard_normal(m)
    H = np.diag(rng.random(n) + 0.1)
    for _ in range(5):                                               # couplings: these are not leaves
        a, b = rng.choice(n, 2, replace=False)
        H[a, b] = H[b, a] = 0.01
    K = sp.csc_matrix(np.block([[H, A.T], [A, -1e-8 * np.eye(m)]]))
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("ordering", [0, 1, 4])
def test_symbolic_twin_leaves(seed, ordering):
    """Twin leaves (symbolic.cpp find_twins: leaves with identical column sets, skipped by the etree
    and the column counts) give the same nnz(L) as brute-force elimination and the oracle LDL^T."""
    from madipm_amd._lib import Symbolic, default_ldl_opts
    from oracle.ldl import OracleLDL
    K, Lw = _twin_k2(seed)
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=ordering))
    perm = S.perm()
    assert S.info()["nnzL"] == _brute_nnzL(K, perm)
    F = OracleLDL(K, perm)
    assert F.factorize() == K.shape[0]
    assert F.nnzL() == S.info()["nnzL"]


def _sibling_k2(seed, nblk=4, bw=20, border=300):
    """K of `nblk` diagonal blocks (bw columns each, sparse inside) all coupled to a border of `border`
    variables (dense clique): the blocks are etree siblings under the border, each with an update block
    of ~border rows (HBM-sized: > big_merge_rows)."""
    rng = np.random.default_rng(seed)
    N = nblk * bw + border
    K = np.zeros((N, N))
    for b in range(nblk):
        s = slice(b * bw, (b + 1) * bw)
        K[s, s] = (rng.random((bw, bw)) < 0.3) * rng.standard_normal((bw, bw))
        K[s, nblk * bw:] = (rng.random((bw, border)) < 0.9) * rng.standard_normal((bw, border))
    K[nblk * bw:, nblk * bw:] = rng.standard_normal((border, border))
    K = K + K.T + 4 * N * np.eye(N)
    K = sp.csc_matrix(K)
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    return K, Lw


@pytest.mark.parametrize("seed", [0, 1])
def test_symbolic_sibling_merge(seed, monkeypatch):
    """Cost-based amalgamation of HBM-sized fronts (symbolic.cpp step 2b + step 4's big_merge rule):
    sibling children with large update blocks are moved next to their parent and merged into it.  The
    moved order is an elimination order of the same etree: the same nnz(L) (brute force and the oracle
    LDL^T on it), a postordered front tree, and fewer fronts than without the rule.  relax=0: the
    zero-fraction amalgamation off, the cost rule alone."""
    from madipm_amd._lib import Symbolic, default_ldl_opts
    from oracle.ldl import OracleLDL
    K, Lw = _sibling_k2(seed)
    monkeypatch.setenv("MADIPM_BIG_MERGE", "0")
    S0 = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=1, relax=0))
    monkeypatch.setenv("MADIPM_BIG_MERGE", "6")
    S1 = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=1, relax=0))
    i0, i1 = S0.info(), S1.info()
    perm = S1.perm()
    assert sorted(perm.tolist()) == list(range(K.shape[0]))
    assert i1["nnzL"] == i0["nnzL"] == _brute_nnzL(K, perm)
    F = OracleLDL(K, perm)
    assert F.factorize() == K.shape[0]
    assert F.nnzL() == i1["nnzL"]
    first, parent, nrows = S1.supernodes()
    ns = i1["nsuper"]
    assert np.all((parent == -1) | (parent > np.arange(ns)))
    assert np.all(nrows >= np.diff(first))
    # the siblings merged: no front with more than 256 rows has a parent any more
    p0 = S0.supernodes()[1]
    assert np.sum((S0.supernodes()[2] > 256) & (p0 >= 0)) >= 2
    assert np.sum((nrows > 256) & (parent >= 0)) == 0
    assert ns < i0["nsuper"] and i1["nnzL_stored"] >= i0["nnzL_stored"]


_THREADS_PROBE = r"""
import sys, hashlib
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/madipm.jl_amd', sys.argv[1] + '/tests']
import numpy as np
from helpers import lp_k2
from madipm_amd import standard_form_qp
from madipm_amd import instances as I
from madipm_amd._lib import Symbolic, default_ldl_opts
qp = standard_form_qp(I.ex10_standin(scale=0.1))
K, Lw = lp_k2(qp, 0)
for ordering in (3, 4):
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=ordering))
    first, parent, nrows = S.supernodes()
    h = hashlib.sha256(S.perm().tobytes() + first.tobytes() + parent.tobytes() + nrows.tobytes()).hexdigest()
    print(ordering, S.info()["nnzL"], h)
"""


def test_analysis_independent_of_thread_count():
    """Nested dissection runs its independent subgraphs, bisection tries and seeds on host threads
    (csrc/nd.cpp, symbolic.cpp step 1), the fold tables and the assembly plan per front on threads
    (step 10): the order, the fronts and the plan must not depend on MADIPM_ANALYSIS_THREADS (read
    once per process, hence the subprocesses)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for t in ("1", "3", "8"):
        env = dict(os.environ, MADIPM_ANALYSIS_THREADS=t)
        r = subprocess.run([sys.executable, "-c", _THREADS_PROBE, root], env=env, capture_output=True,
                           text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout)
    assert outs[0] == outs[1] == outs[2], outs


@pytest.mark.parametrize("n", [1300, 2500])
def test_fold_batches_hold_at_most_1024_leaves(n):
    """A tree front with more than 2 x 512 micro leaves still folds them (fold_leaves keeps a
    batch's leaf table in two registers per thread, so the planner caps a batch at kFoldLeavesMax
    leaves and cuts more batches; the GPU side is test_ldl_gpu.py::test_fold_many_leaves)."""
    from helpers import many_leaf_k2
    from madipm_amd._lib import Symbolic, default_ldl_opts
    K, Lw = many_leaf_k2(n)
    info = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=4)).info()
    assert info["fold_fronts"] == 1 and info["fold_leaves"] > 1024, info


# SHA-1 (16 hex digits) of the nested-dissection order (ordering 3) of seeded stand-ins, as produced by
# the round-5 ND code and unchanged by r6's speed-ups (threaded contraction, refinement scans and
# induced subgraphs, uninitialised level arrays, the unit-weight matching shortcut): checked against a
# build of the r5 sources (tools/perm_hash.py for the full-size configs).  A deliberate change of the
# ordering updates these values.
_ND_PINNED = {("ex10", 0.2): "d5c08eaa5e16e99c", ("neos", 0.1): "609901f70409cd1a",
              ("supportcase10", 0.1): "328a57c1bc0e6381"}


@pytest.mark.parametrize("name,scale", sorted(_ND_PINNED))
def test_nd_order_pinned(name, scale):
    import hashlib
    from helpers import lp_k2
    from madipm_amd import standard_form_qp
    from madipm_amd import instances as I
    from madipm_amd._lib import Symbolic, default_ldl_opts
    make = {"ex10": I.ex10_standin, "neos": I.neos5052403_standin, "supportcase10": I.supportcase10_standin}[name]
    K, Lw = lp_k2(standard_form_qp(make(scale=scale)), 0, well=True)
    S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(ordering=3))
    assert hashlib.sha1(S.perm().tobytes()).hexdigest()[:16] == _ND_PINNED[(name, scale)]
