"""GPU test of the cost-based sibling merges of HBM-sized fronts (csrc/symbolic.cpp steps 2b / 4,
SymbolicOptions::big_merge; default 6 flop/B since r5 — neos 31.5 -> 35.9 iters/s, profiles/r5_a_*;
MADIPM_BIG_MERGE overrides, 0 disables): the merged order is another elimination order of the same
etree, so parity is against the oracle (status, iterations +-1, objective 1e-6) and against the
unmerged factorisation, and the analysis must have merged something.

(The r4 opt-in tail overlap — the fronts after k_fact_tree on a side stream beside the next solve —
measured slower on the GPU, ex10 1683 -> 1653 and supportcase10 1157 -> 1111 iters/s, profiles/r5_a_*,
and was deleted with its code.)
"""
import pytest

pytestmark = pytest.mark.gpu


def _solve(qp, env, monkeypatch):
    from madipm_amd import MPCSolver, FixedRegularization
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    try:
        s = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), max_iter=300)
    finally:
        for k in env:
            monkeypatch.delenv(k, raising=False)
    return s, s.solve()


@pytest.mark.parametrize("merge", ["6", "12"])
def test_big_merge_vs_oracle(merge, monkeypatch):
    """neos stand-in at a scale whose fronts exceed big_merge_rows (256): the merged order vs the
    unmerged one (MADIPM_BIG_MERGE=0) and vs the oracle."""
    from madipm_amd import standard_form_qp
    from madipm_amd import instances as I
    from oracle.mpc import OracleMPC, OracleOptions
    from oracle import pardiso
    qp = standard_form_qp(I.neos5052403_standin(scale=0.1))
    s0, a = _solve(qp, {"MADIPM_BIG_MERGE": "0"}, monkeypatch)
    s1, b = _solve(qp, {"MADIPM_BIG_MERGE": merge}, monkeypatch)
    i0, i1 = s0.ldl_info(), s1.ldl_info()
    print("unmerged", {k: i0[k] for k in ("nsuper", "nnzL_stored", "flops", "nlevels")},
          "merge", merge, {k: i1[k] for k in ("nsuper", "nnzL_stored", "flops", "nlevels")})
    assert i1["nsuper"] < i0["nsuper"] and i1["nnzL"] == i0["nnzL"]
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), step_rule=("adaptive", 0.99),
                                    max_iter=300, tol=1e-8), record_trace=False)
    if pardiso.available():
        o.linear_solver = "pardiso"
    ref = o.solve()
    assert a.status == b.status == ref.status == 1
    assert abs(b.iter - ref.iter) <= 1, (b.iter, ref.iter)
    assert abs(b.objective - ref.objective) <= 1e-6 * max(1.0, abs(ref.objective))
    assert abs(b.objective - a.objective) <= 1e-6 * max(1.0, abs(a.objective))


def test_big_merge_default_is_on(monkeypatch):
    """The default analysis merges (big_merge = 6): same plan as MADIPM_BIG_MERGE=6."""
    from madipm_amd import standard_form_qp
    from madipm_amd import instances as I
    qp = standard_form_qp(I.neos5052403_standin(scale=0.1))
    monkeypatch.delenv("MADIPM_BIG_MERGE", raising=False)
    sd, _ = _solve(qp, {}, monkeypatch)
    s6, _ = _solve(qp, {"MADIPM_BIG_MERGE": "6"}, monkeypatch)
    idf, i6 = sd.ldl_info(), s6.ldl_info()
    for k in ("nsuper", "nnzL_stored", "flops", "nlevels"):
        assert idf[k] == i6[k], (k, idf[k], i6[k])
