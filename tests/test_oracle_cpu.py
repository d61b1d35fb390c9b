"""CPU tests of the oracle (test infrastructure): pinned against the reference's own answers and HiGHS.

* simple_lp (test/runtests.jl:29-60): objective exactly 1 with NoRegularization;
  standard_form_qp gives the same objective (test/runtests.jl:159-164).
* AFIRO (BASELINE.json configs[0]): netlib optimum -464.75314286 (HiGHS: -464.7531428571).
* seeded LPs: objective within 1e-6 relative of HiGHS (fp64; IPM tol 1e-8).
* golden traces (tests/golden/oracle_traces.json, made by tools/make_golden.py): the oracle
  reproduces its committed per-iteration trace to 1e-10 relative (regression pin).
"""
import json
import os

import numpy as np
import pytest

from oracle.mpc import OracleMPC, OracleOptions, SOLVE_SUCCEEDED

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load_case(name):
    from madipm_amd import read_mps, simple_lp, standard_form_qp
    from madipm_amd.instances import random_lp
    afiro = lambda: read_mps(os.path.join(GOLD, "afiro.mps"))  # noqa: E731
    return {
        "simple_lp_noreg": simple_lp, "simple_lp_std": lambda: standard_form_qp(simple_lp()),
        "afiro_fixed": afiro, "afiro_std_fixed": lambda: standard_form_qp(afiro()),
        "random_lp_60x120_s0": lambda: random_lp(60, 120, 0.05, 0, ineq_frac=0.3, free_frac=0.05),
        "random_lp_100x200_s1": lambda: random_lp(100, 200, 0.03, 1, ineq_frac=0.2),
    }[name]()


def _opts(d):
    return OracleOptions(**{k: tuple(v) if isinstance(v, list) else v for k, v in d.items()})


def test_simple_lp_objective_is_one():
    from madipm_amd import simple_lp
    st = OracleMPC(simple_lp(), OracleOptions(regularization=("none",))).solve()
    assert st.status == SOLVE_SUCCEEDED
    assert st.objective == pytest.approx(1.0, abs=1e-10)


def test_simple_lp_standard_form_same_objective():
    from madipm_amd import simple_lp, standard_form_qp
    a = OracleMPC(simple_lp(), OracleOptions(regularization=("none",))).solve()
    b = OracleMPC(standard_form_qp(simple_lp()), OracleOptions()).solve()
    assert abs(a.objective - b.objective) <= 1e-10


@pytest.mark.parametrize("std", [False, True])
def test_afiro_netlib_optimum(std):
    from madipm_amd import read_mps, standard_form_qp
    qp = read_mps(os.path.join(GOLD, "afiro.mps"))
    if std:
        qp = standard_form_qp(qp)
    st = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=300)).solve()
    assert st.status == SOLVE_SUCCEEDED
    assert st.objective == pytest.approx(-464.75314286, rel=1e-9)


with open(os.path.join(GOLD, "oracle_traces.json")) as _f:
    GOLDEN = json.load(_f)


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_golden_traces(name):
    g = GOLDEN[name]
    qp = _load_case(name)
    st = OracleMPC(qp, _opts(g["options"])).solve()
    assert st.status == g["status"] and st.iter == g["iter"]
    assert st.objective == pytest.approx(g["objective"], rel=1e-10, abs=1e-12)
    assert st.objective == pytest.approx(g["highs_objective"], rel=1e-6, abs=1e-8)
    for a, b in zip(st.trace, g["trace"]):
        for k in ("obj", "inf_pr", "inf_du", "inf_compl", "mu", "alpha_p", "alpha_d"):
            assert a[k] == pytest.approx(b[k], rel=1e-10, abs=1e-14), (name, a["k"], k)


@pytest.mark.parametrize("rule", [("adaptive", 0.99), ("conservative", 0.99), ("mehrotra", 0.99)])
def test_step_rules_converge(rule):
    from madipm_amd.instances import dense_dummy_qp
    st = OracleMPC(dense_dummy_qp(10, 5), OracleOptions(step_rule=rule)).solve()
    assert st.status == SOLVE_SUCCEEDED


def test_gondzio_and_regularizations_agree():
    """test/runtests.jl:67-78,122-140: variants reach the same solution (atol 1e-6)."""
    from madipm_amd.instances import dense_dummy_qp
    qp = dense_dummy_qp(20, 15, eq=[1, 2, 3, 8])
    ref = OracleMPC(qp, OracleOptions(regularization=("none",))).solve()
    for o in (OracleOptions(max_ncorr=5), OracleOptions(regularization=("fixed", 1e-8, -1e-9)),
              OracleOptions(regularization=("adaptive", 1e-8, -1e-9, 1e-9))):
        st = OracleMPC(qp, o).solve()
        assert st.status == SOLVE_SUCCEEDED
        assert st.objective == pytest.approx(ref.objective, abs=1e-6)
        assert np.allclose(st.solution, ref.solution, atol=1e-5)


def test_oracle_ldl_linear_solver_matches_superlu():
    """The oracle's C LDL^T path (used as CPU baseline) gives the same MPC result as SuperLU."""
    from madipm_amd import read_mps, standard_form_qp
    qp = standard_form_qp(read_mps(os.path.join(GOLD, "afiro.mps")))
    a = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8))).solve()
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8)))
    o.linear_solver = "ldl"
    b = o.solve()
    assert a.status == b.status == SOLVE_SUCCEEDED
    assert b.objective == pytest.approx(a.objective, rel=1e-9)


def test_maximize_sign():
    """update_solution! flips the objective of maximisation problems (src/utils.jl:150-156)."""
    from madipm_amd.instances import ex10_standin
    from madipm_amd import standard_form_qp
    qp = standard_form_qp(ex10_standin(scale=0.02))
    assert not qp.minimize
    st = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=100)).solve()
    assert st.status == SOLVE_SUCCEEDED and st.objective > 0


# ---------------------------------------------------------------- KKT formulations (oracle)
# test/runtests.jl:107-120 (K2.5 == K2 within 1e-6) and :182-196 (NormalKKTSystem == K2 within 1e-6)
def _cmp_sol(a, b, tol=1e-6, ytol=1e-6):
    """objective / solution / multipliers within `tol` (the reference's atol 1e-6, scaled by the
    magnitude); `ytol` for multipliers of problems with a degenerate dual face (AFIRO, random LPs:
    the IPM stops at tol 1e-8 before the multipliers settle to 1e-6)."""
    assert a.status == b.status == SOLVE_SUCCEEDED
    assert abs(a.objective - b.objective) <= tol * max(1.0, abs(b.objective))
    assert np.max(np.abs(a.solution - b.solution)) <= tol * max(1.0, np.max(np.abs(b.solution)))
    assert np.max(np.abs(a.multipliers - b.multipliers)) <= ytol * max(1.0, np.max(np.abs(b.multipliers)))


@pytest.mark.parametrize("kkt", ["K25", "normal"])
@pytest.mark.parametrize("case", ["simple_lp", "afiro", "random_lp_60x120_s0"])
def test_oracle_kkt_formulations_agree(kkt, case):
    from madipm_amd import read_mps, simple_lp
    from madipm_amd.instances import random_lp
    qp = {"simple_lp": simple_lp, "afiro": lambda: read_mps(os.path.join(GOLD, "afiro.mps")),
          "random_lp_60x120_s0": lambda: random_lp(60, 120, 0.05, 0, ineq_frac=0.3)}[case]()
    reg = ("fixed", 1e-8, -1e-8)
    ref = OracleMPC(qp, OracleOptions(regularization=reg, max_iter=300)).solve()
    st = OracleMPC(qp, OracleOptions(regularization=reg, max_iter=300, kkt_system=kkt)).solve()
    _cmp_sol(st, ref, ytol=1e-6 if case == "simple_lp" else 1e-5)
    assert abs(st.iter - ref.iter) <= 1


def test_oracle_k25_qp_agrees():
    from madipm_amd.instances import random_qp
    qp = random_qp(40, 80, 0.08, 3)
    ref = OracleMPC(qp, OracleOptions(max_iter=300)).solve()
    st = OracleMPC(qp, OracleOptions(max_iter=300, kkt_system="K25")).solve()
    _cmp_sol(st, ref, ytol=1e-5)


@pytest.mark.skipif(not __import__("oracle.pardiso", fromlist=["available"]).available(), reason="MKL absent")
def test_oracle_pardiso_linear_solver_matches_superlu():
    """bench.py's CPU baseline (oracle MPC + MKL PARDISO) reaches the same answer as the oracle's
    default SuperLU solve: AFIRO's netlib optimum and the same iteration count; and the failure-path
    semantics (pivot_tol, unfactorized solve) hold for the LDL^T oracle."""
    from madipm_amd import read_mps, standard_form_qp
    from oracle import pardiso
    qp = standard_form_qp(read_mps(os.path.join(os.path.dirname(__file__), "golden", "afiro.mps")))
    pardiso.set_threads(2)
    a = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8)))
    a.linear_solver = "pardiso"
    sa = a.solve()
    sb = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8))).solve()
    assert sa.status == sb.status == SOLVE_SUCCEEDED and sa.iter == sb.iter
    assert abs(sa.objective + 464.7531428571) <= 1e-7 * 464.75
    assert a._pardiso.nperturbed == 0 and a._pardiso.nfactor == sa.iter + 1


def test_oracle_failed_factorization_is_internal_error():
    """Every trial of factorize_regularized_system! failing (del_w = 0 on a free LP column) makes the
    next solve throw an exception that is no LinearSolverException: solve!'s catch-all sets
    INTERNAL_ERROR (src/solver.jl:398-403; oracle semantics the GPU tests compare against)."""
    from madipm_amd.qp import QuadraticModel
    from oracle.mpc import INTERNAL_ERROR, EXC_UNFACTORIZED
    inf = np.inf
    qp = QuadraticModel(c=np.array([1.0, 1.0, 0.0]), Hrows=[], Hcols=[], Hvals=[], Arows=[0, 0, 1, 1, 1],
                        Acols=[0, 1, 0, 1, 2], Avals=[1.0, 1.0, 1.0, -1.0, 1.0], lcon=[1.0, 0.0], ucon=[1.0, 0.0],
                        lvar=[0.0, 0.0, -inf], uvar=[inf, inf, inf])
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 0.0, -1e-8)))
    o.linear_solver = "ldl"
    o.ldl_perm = np.array([2, 4, 3, 1, 0])
    st = o.solve()
    assert st.status == INTERNAL_ERROR and st.exception == EXC_UNFACTORIZED
    assert st.iter == 0 and len(st.trace) == 1
    # pivot_tol: del_w = 1e-12 and 1e-10 rejected, 1e-8 accepted -> the retry path converges
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-12, -1e-8)))
    o.linear_solver = "ldl"
    o.ldl_perm = np.array([2, 4, 3, 1, 0])
    o.pivot_tol = 1e-9
    st = o.solve()
    assert st.status == SOLVE_SUCCEEDED and abs(st.objective - 1.0) <= 1e-7
    assert all(abs(t["del_w"] - 1e-8) <= 1e-20 for t in st.trace[1:])


@pytest.mark.skipif(not __import__("oracle.pardiso", fromlist=["available"]).available(), reason="MKL absent")
def test_kkt_properties_maximisation_stand_in():
    """The optimality measures the full-size GPU tests threshold (helpers.kkt_properties), pinned on a
    maximisation stand-in (every MIPLIB stand-in is minimize=False) where the oracle runs: with the
    solver's objective sign sigma = -1 the returned (x, y, zl, zu) satisfy the KKT conditions to the
    IPM's tolerance and the dual bound equals the primal objective; HiGHS gives the same optimum."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import bench
    from helpers import kkt_properties
    from oracle import pardiso
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    from make_golden_fullsize import highs_standard_form
    qp, _ = bench.build_problem("ex10@0.05")
    assert not qp.minimize
    pardiso.set_threads(1)
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), step_rule=("adaptive", 0.99),
                                    max_iter=300, tol=1e-8), record_trace=False)
    o.linear_solver = "pardiso"
    st = o.solve()
    assert st.status == SOLVE_SUCCEEDED
    p = kkt_properties(qp, st)
    assert p["pr"] <= 1e-6 and p["du"] <= 1e-6, p
    assert abs(p["pobj"] - p["dobj"]) <= 1e-6 * max(1.0, abs(p["pobj"])), p
    assert abs(p["pobj"] - st.objective) <= 1e-9 * max(1.0, abs(p["pobj"]))
    h = highs_standard_form(qp)
    assert abs(st.objective - h["objective"]) <= 1e-6 * max(1.0, abs(h["objective"])), (st.objective, h)


def test_fullsize_highs_fixture_present():
    """tests/golden/fullsize_highs.json (tools/make_golden_fullsize.py) pins the full-size stand-ins'
    optima for the GPU tests (tests/test_fullsize_gpu.py)."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "fullsize_highs.json")) as f:
        g = json.load(f)
    for c in ("ex10", "supportcase10", "neos"):
        assert g[c]["status"] == 0 and not g[c]["minimize"] and np.isfinite(g[c]["objective"]), g[c]
