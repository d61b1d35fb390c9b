"""MOI-style front end on the GPU: Optimizer.copy_to -> optimize -> results (MOI_wrapper.jl:89-188).

The translated model is solved by the HIP MPC and by the oracle (tests/test_mpc_gpu.py::_compare
tolerances); the simple_lp answer is the reference's own (test/runtests.jl:29-60: objective 1).
"""
import numpy as np
import pytest

from madipm_amd import moi
from madipm_amd.moi import (EqualTo, GreaterThan, Interval, LessThan, Nonnegatives,
                            ScalarAffineFunction as SAF, ScalarAffineTerm as SAT,
                            ScalarQuadraticFunction as SQF, ScalarQuadraticTerm as SQT,
                            VectorAffineFunction as VAF, VectorAffineTerm as VAT)
from test_mpc_gpu import _compare

pytestmark = pytest.mark.gpu


def test_optimizer_simple_lp():
    m = moi.Model()
    x = m.add_variables(2)
    for v in x:
        m.add_constraint(v, GreaterThan(0.0))
        m.set_start(v, 1.0)
    m.add_constraint(SAF([SAT(1.0, x[0]), SAT(1.0, x[1])]), EqualTo(1.0))
    m.set_objective(moi.MIN_SENSE, SAF([SAT(1.0, x[0]), SAT(1.0, x[1])]))
    opt = moi.Optimizer()
    opt.set_silent(True)
    imap = opt.copy_to(m)
    opt.optimize()
    assert opt.termination_status() == "OPTIMAL" and opt.primal_status() == "FEASIBLE_POINT"
    assert abs(opt.objective_value() - 1.0) < 1e-7
    xs = [opt.variable_primal(imap[v]) for v in x]
    assert abs(sum(xs) - 1.0) < 1e-7 and min(xs) > -1e-8
    assert opt.raw_status_string() == "SOLVE_SUCCEEDED" and opt.solve_time_sec() > 0


def _qp_model(sense, seed=3, n=40, nrow=12):
    rng = np.random.default_rng(seed)
    m = moi.Model()
    x = m.add_variables(n)
    for i, v in enumerate(x):
        k = i % 4
        if k == 0:
            m.add_constraint(v, Interval(-1.0, 3.0))
        elif k == 1:
            m.add_constraint(v, GreaterThan(-0.5))
        elif k == 2:
            m.add_constraint(v, LessThan(2.0))
    x0 = rng.uniform(-0.4, 1.5, n)                                   # strictly inside every bound
    for r in range(nrow):
        cols = rng.choice(n, 6, replace=False)
        a = rng.standard_normal(6)
        f = SAF([SAT(float(a[t]), x[c]) for t, c in enumerate(cols)], float(rng.uniform(-1, 1)))
        val = float(a @ x0[cols]) + f.constant
        # every row holds at x0 (f(x0) = val)
        s = [EqualTo(val), LessThan(val + 1.0), GreaterThan(val - 1.0), Interval(val - 0.5, val + 0.5)][r % 4]
        m.add_constraint(f, s)
    m.add_constraint(VAF([VAT(0, SAT(1.0, x[1])), VAT(1, SAT(1.0, x[5]))], [1.0, 1.0]), Nonnegatives(2))
    sign = 1.0 if sense == moi.MIN_SENSE else -1.0
    quad = [SQT(sign * float(rng.uniform(0.5, 2.0)), v, v) for v in x]
    quad += [SQT(sign * 0.1, x[i + 1], x[i]) for i in range(0, n - 1, 3)]
    aff = [SAT(sign * float(rng.standard_normal()), v) for v in x]
    m.set_objective(sense, SQF(quad, aff, sign * 2.0))
    return m


@pytest.mark.parametrize("sense", [moi.MIN_SENSE, moi.MAX_SENSE])
def test_optimizer_qp_against_oracle(sense):
    from madipm_amd import madipm
    m = _qp_model(sense)
    opt = moi.Optimizer()
    opt.set_silent(True)
    opt.set_attribute("max_iter", 200)
    opt.copy_to(m)
    opt.optimize()
    assert opt.termination_status() == "OPTIMAL"
    qp, _ = moi.qp_model(_qp_model(sense))
    direct = madipm(qp, max_iter=200)
    assert opt.objective_value() == direct.objective and opt.stats.iter == direct.iter
    _compare(qp, max_iter=200)
    if sense == moi.MAX_SENSE:   # max -f = -(min f): same optimum up to the sign
        mq, _ = moi.qp_model(_qp_model(moi.MIN_SENSE))
        assert abs(opt.objective_value() + madipm(mq, max_iter=200).objective) <= 1e-6 * max(1.0, abs(opt.objective_value()))
