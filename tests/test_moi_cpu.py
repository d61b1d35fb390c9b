"""MOI-style front end (madipm_amd.moi): model -> QuadraticModel translation.

Checks the translation rules of the reference's `parse_moi.jl` (ext/MadIPMMathOptInterfaceExt):
variable bounds from VariableIndex-in-set constraints (:37-45), affine rows with the constant moved
into the bounds (:73-96), vector-affine rows per set (:97-114), canonicalised quadratic objective in
the lower triangle (:145-164, :173-180), sense (:182); and that the oracle solves the translated
model to the same optimum as the hand-built QuadraticModel.
"""
import math

import numpy as np
import pytest

from madipm_amd import moi
from madipm_amd.moi import (EqualTo, GreaterThan, Interval, LessThan, Nonnegatives, Nonpositives, Zeros,
                            ScalarAffineFunction as SAF, ScalarAffineTerm as SAT,
                            ScalarQuadraticFunction as SQF, ScalarQuadraticTerm as SQT,
                            VectorAffineFunction as VAF, VectorAffineTerm as VAT)


def _simple_lp_model():
    """test/runtests.jl:29-60 simple_lp through the model API: min x1 + x2, x1 + x2 = 1, x >= 0."""
    m = moi.Model()
    x = m.add_variables(2)
    for v in x:
        m.add_constraint(v, GreaterThan(0.0))
        m.set_start(v, 1.0)
    m.add_constraint(SAF([SAT(1.0, x[0]), SAT(1.0, x[1])], 0.0), EqualTo(1.0))
    m.set_objective(moi.MIN_SENSE, SAF([SAT(1.0, x[0]), SAT(1.0, x[1])], 0.0))
    return m, x


def test_simple_lp_translation_equals_reference_problem():
    from madipm_amd import simple_lp
    m, _ = _simple_lp_model()
    qp, imap = moi.qp_model(m)
    ref = simple_lp()
    for k in ("c", "Avals", "lcon", "ucon", "lvar", "uvar", "x0"):
        np.testing.assert_array_equal(getattr(qp, k), getattr(ref, k), err_msg=k)
    np.testing.assert_array_equal(qp.Arows, ref.Arows)
    np.testing.assert_array_equal(qp.Acols, ref.Acols)
    assert qp.minimize and qp.nnzh == 0 and qp.c0 == 0.0
    assert imap[moi.VariableIndex(1)] == moi.VariableIndex(1)


def _mixed_model():
    m = moi.Model()
    x = m.add_variables(4)
    m.add_constraint(x[0], Interval(-1.0, 2.0))
    m.add_constraint(x[1], GreaterThan(0.5))
    m.add_constraint(x[1], LessThan(3.0))
    m.add_constraint(x[2], EqualTo(1.25))
    # rows: affine with constants, every ALS set
    m.add_constraint(SAF([SAT(1.0, x[0]), SAT(2.0, x[1])], 0.5), LessThan(4.0))      # row 0: (-inf, 3.5]
    m.add_constraint(SAF([SAT(1.0, x[1]), SAT(-1.0, x[3])], -1.0), GreaterThan(0.0))  # row 1: [1, inf)
    m.add_constraint(SAF([SAT(1.0, x[0]), SAT(1.0, x[3])], 0.0), Interval(-2.0, 5.0))  # row 2
    m.add_constraint(SAF([SAT(3.0, x[2])], 1.0), EqualTo(4.75))                        # row 3: = 3.75
    # vector rows
    m.add_constraint(VAF([VAT(0, SAT(1.0, x[3])), VAT(1, SAT(1.0, x[0])), VAT(1, SAT(1.0, x[1]))],
                         [0.0, -1.0]), Nonnegatives(2))                                 # rows 4,5
    m.add_constraint(VAF([VAT(0, SAT(1.0, x[3]))], [-6.0]), Nonpositives(1))            # row 6: x3 <= 6
    m.add_constraint(VAF([VAT(0, SAT(1.0, x[0])), VAT(0, SAT(-1.0, x[2]))], [0.25]), Zeros(1))  # row 7
    # quadratic objective with duplicates in both orders, an affine duplicate and a constant
    obj = SQF([SQT(2.0, x[0], x[0]), SQT(0.5, x[1], x[0]), SQT(0.5, x[0], x[1]), SQT(1.0, x[3], x[3]),
               SQT(0.0, x[2], x[2])],
              [SAT(1.0, x[0]), SAT(-2.0, x[1]), SAT(0.5, x[0]), SAT(1.0, x[3])], 7.0)
    m.set_objective(moi.MIN_SENSE, obj)
    return m, x


def test_translation_rules():
    m, x = _mixed_model()
    qp, imap = moi.qp_model(m)
    inf = math.inf
    np.testing.assert_array_equal(qp.lvar, [-1.0, 0.5, 1.25, -inf])
    np.testing.assert_array_equal(qp.uvar, [2.0, 3.0, 1.25, inf])
    np.testing.assert_array_equal(qp.lcon, [-inf, 1.0, -2.0, 3.75, 0.0, 1.0, -inf, -0.25])
    np.testing.assert_array_equal(qp.ucon, [3.5, inf, 5.0, 3.75, inf, inf, 6.0, -0.25])
    A = np.zeros((8, 4))
    np.add.at(A, (qp.Arows, qp.Acols), qp.Avals)
    np.testing.assert_array_equal(A, [[1, 2, 0, 0], [0, 1, 0, -1], [1, 0, 0, 1], [0, 0, 3, 0],
                                      [0, 0, 0, 1], [1, 1, 0, 0], [0, 0, 0, 1], [1, 0, -1, 0]])
    np.testing.assert_array_equal(qp.c, [1.5, -2.0, 0.0, 1.0])
    assert qp.c0 == 7.0
    assert np.all(qp.Hrows >= qp.Hcols)                   # lower triangle
    H = np.zeros((4, 4))
    np.add.at(H, (qp.Hrows, qp.Hcols), qp.Hvals)
    np.testing.assert_array_equal(H, [[2, 0, 0, 0], [1.0, 0, 0, 0], [0, 0, 0, 0], [0, 0, 0, 1]])
    assert qp.nnzh == 3                                    # merged duplicate, zero dropped
    # constraint index map: VariableIndex constraints map to their variable, rows to their row
    cis = [ci for (F, S) in m.list_of_constraint_types_present() for ci, _, _ in m.constraints(F, S)]
    rows = sorted(imap[ci].value for ci in cis if ci.function_type is not moi.VariableIndex)
    assert rows == [0, 1, 2, 3, 4, 6, 7]                   # vector blocks map to their first row


def test_objective_value_semantics():
    """1/2 x'Hx + c'x + c0 of the translation equals the MOI function evaluated term by term."""
    m, x = _mixed_model()
    f = m.objective
    pt = np.array([0.3, -1.2, 2.0, 0.7])
    direct = f.constant + sum(t.coefficient * pt[t.variable.value] for t in f.affine_terms)
    for t in f.quadratic_terms:
        i, j = t.variable_1.value, t.variable_2.value
        direct += (0.5 if i == j else 1.0) * t.coefficient * pt[i] * pt[j]
    qp, _ = moi.qp_model(m)
    H = np.zeros((4, 4))
    np.add.at(H, (qp.Hrows, qp.Hcols), qp.Hvals)
    H = H + np.tril(H, -1).T
    assert abs((qp.c0 + qp.c @ pt + 0.5 * pt @ H @ pt) - direct) < 1e-12


def test_maximize_and_objective_kinds():
    m = moi.Model()
    x = m.add_variables(2)
    m.set_objective(moi.MAX_SENSE, x[1])
    qp, _ = moi.qp_model(m)
    assert not qp.minimize and list(qp.c) == [0.0, 1.0] and qp.ncon == 0
    with pytest.raises(TypeError):
        m.add_constraint(x[0], Zeros(1))
    with pytest.raises(TypeError):
        m.set_objective(moi.MIN_SENSE, 3.0)


def test_optimizer_attributes_without_solving():
    opt = moi.Optimizer()
    assert opt.is_empty() and opt.solver_name == "MadIPM"
    assert opt.termination_status() == "OPTIMIZE_NOT_CALLED"
    assert opt.primal_status() == "NO_SOLUTION" and opt.dual_status() == "NO_SOLUTION"
    opt.set_attribute("max_iter", 50)
    opt.set_attribute("array_type", "ROCArray")
    assert opt.get_attribute("max_iter") == 50 and "array_type" not in opt.options
    opt.set_silent(True)
    assert opt.get_silent()
    assert opt.supports("ObjectiveFunction", moi.ScalarQuadraticFunction)
    assert opt.supports("VariablePrimalStart")
    assert opt.supports_constraint(moi.VectorAffineFunction, Zeros)
    assert not opt.supports_constraint(moi.VectorAffineFunction, EqualTo)
    m, _ = _simple_lp_model()
    opt.copy_to(m)
    assert not opt.is_empty()
    opt.empty()
    assert opt.is_empty()
    with pytest.raises(ValueError):
        opt.objective_value()
    # every MadNLP status this build reports has a termination-status mapping
    from madipm_amd.qp import QuadraticModel  # noqa: F401  (host import only)
    for name in ("SOLVE_SUCCEEDED", "INFEASIBLE_PROBLEM_DETECTED", "MAXIMUM_ITERATIONS_EXCEEDED",
                 "MAXIMUM_WALLTIME_EXCEEDED", "DIVERGING_ITERATES", "ERROR_IN_STEP_COMPUTATION", "INTERNAL_ERROR"):
        assert name in moi.TERMINATION_STATUS


def test_oracle_solves_translation_like_hand_built():
    """The oracle MPC on the translated simple_lp and on the reference's own simple_lp: same answer."""
    from madipm_amd import simple_lp
    from oracle.mpc import OracleMPC, OracleOptions
    m, _ = _simple_lp_model()
    qp, _ = moi.qp_model(m)
    a = OracleMPC(qp, OracleOptions()).solve()
    b = OracleMPC(simple_lp(), OracleOptions()).solve()
    assert a.status == b.status and a.iter == b.iter
    assert abs(a.objective - 1.0) < 1e-7 and a.objective == b.objective
