"""GPU tests of the scheduling / analysis variants behind environment knobs:

* MADIPM_TAIL_OVERLAP=1 — the launches after k_fact_tree (root assembly + root front) on a side stream
  beside the next solve's leaf and tree launches, joined before the root solve, the status read-back,
  the inertia count and the next factorisation (csrc/ldl.hip LDLSolver::fact1_tail_).  The same
  kernels run on the same data in a different stream placement, so the MPC trajectory must be BITWISE
  the default one: status, iteration count, every trace entry, objective and solution bits — a race on
  the fork/join would show up as a changed bit (or a stale pivot status).
* MADIPM_BIG_MERGE=<flop/B> — cost-based sibling merges of HBM-sized fronts (csrc/symbolic.cpp step
  2b/4): a different elimination order of the same etree, so parity is against the oracle (status,
  iterations +-1, objective 1e-6), and the analysis must have merged something.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cases():
    from madipm_amd import read_mps, standard_form_qp
    from madipm_amd import instances as I
    gold = os.path.join(os.path.dirname(__file__), "golden", "afiro.mps")
    return {
        "afiro_std": lambda: standard_form_qp(read_mps(gold)),
        "random_lp": lambda: I.random_lp(120, 250, 0.03, 1, ineq_frac=0.3, free_frac=0.05),
        "ex10_small": lambda: standard_form_qp(I.ex10_standin(scale=0.05)),
        "supportcase10_small": lambda: standard_form_qp(I.supportcase10_standin(scale=0.05, block_scale=1.0)),
    }


def _solve(qp, env, monkeypatch, timing=False, **kw):
    from madipm_amd import MPCSolver, FixedRegularization
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    try:
        s = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), max_iter=300, **kw)
    finally:
        for k in env:
            monkeypatch.delenv(k, raising=False)
    if timing:
        s.set_kernel_timing()
    st = s.solve()
    return s, st


@pytest.mark.parametrize("case", ["afiro_std", "random_lp", "ex10_small", "supportcase10_small"])
@pytest.mark.parametrize("timing", [False, True])
def test_tail_overlap_bitwise(case, timing, monkeypatch):
    qp = _cases()[case]()
    s0, a = _solve(qp, {"MADIPM_TAIL_OVERLAP": "0"}, monkeypatch, timing=timing)
    s1, b = _solve(qp, {"MADIPM_TAIL_OVERLAP": "1"}, monkeypatch, timing=timing)
    assert a.status == b.status == 1, (a.status_name, b.status_name)
    assert a.iter == b.iter
    assert a.objective == b.objective, (a.objective, b.objective)
    assert np.array_equal(a.solution, b.solution)
    assert np.array_equal(a.multipliers, b.multipliers)
    assert len(a.trace) == len(b.trace)
    for ta, tb in zip(a.trace, b.trace):
        assert ta == tb, (ta, tb)
    if timing:
        ka = {k["name"]: k["launches"] for k in s0.kernel_stats()}
        kb = {k["name"]: k["launches"] for k in s1.kernel_stats()}
        assert ka == kb, (ka, kb)
        assert all(k["time_ms"] > 0 for k in s1.kernel_stats() if k["launches"]), s1.kernel_stats()


def test_tail_overlap_vs_oracle(monkeypatch):
    """The overlapped path against the oracle on the ex10 stand-in (small scale)."""
    from oracle.mpc import OracleMPC, OracleOptions
    qp = _cases()["ex10_small"]()
    _, g = _solve(qp, {"MADIPM_TAIL_OVERLAP": "1"}, monkeypatch)
    ref = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=300)).solve()
    assert g.status == ref.status == 1
    assert abs(g.iter - ref.iter) <= 1
    assert abs(g.objective - ref.objective) <= 1e-6 * max(1.0, abs(ref.objective))


@pytest.mark.parametrize("merge", ["6", "12"])
def test_big_merge_vs_oracle(merge, monkeypatch):
    """neos stand-in at a scale whose fronts exceed big_merge_rows (256): the merged order vs the oracle."""
    from madipm_amd import standard_form_qp
    from madipm_amd import instances as I
    from oracle.mpc import OracleMPC, OracleOptions
    from oracle import pardiso
    qp = standard_form_qp(I.neos5052403_standin(scale=0.1))
    s0, a = _solve(qp, {}, monkeypatch)
    s1, b = _solve(qp, {"MADIPM_BIG_MERGE": merge}, monkeypatch)
    i0, i1 = s0.ldl_info(), s1.ldl_info()
    print("default", {k: i0[k] for k in ("nsuper", "nnzL_stored", "flops", "nlevels")},
          "merge", merge, {k: i1[k] for k in ("nsuper", "nnzL_stored", "flops", "nlevels")})
    assert i1["nsuper"] < i0["nsuper"]
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), step_rule=("adaptive", 0.99),
                                    max_iter=300, tol=1e-8), record_trace=False)
    if pardiso.available():
        o.linear_solver = "pardiso"
    ref = o.solve()
    assert a.status == b.status == ref.status == 1
    assert abs(b.iter - ref.iter) <= 1, (b.iter, ref.iter)
    assert abs(b.objective - ref.objective) <= 1e-6 * max(1.0, abs(ref.objective))
    assert abs(b.objective - a.objective) <= 1e-6 * max(1.0, abs(a.objective))
