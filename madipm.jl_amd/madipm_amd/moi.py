"""MathOptInterface-style front end: model objects -> QuadraticModel -> MPCSolver.

Mirrors the reference's MOI extension (klamike/MadIPM.jl `ext/MadIPMMathOptInterfaceExt/`):
* `qp_model` with `parse_variable` / `parse_constraints` / `parse_objective`
  (`parse_moi.jl:22-215`, itself adapted from NLPModelsJuMP): variable bounds from VariableIndex-in-set
  constraints, ScalarAffineFunction-in-{EqualTo, GreaterThan, LessThan, Interval} and
  VectorAffineFunction-in-{Nonnegatives, Nonpositives, Zeros} rows with the function constant moved
  into the bounds, a VariableIndex / ScalarAffineFunction / ScalarQuadraticFunction objective whose
  quadratic terms are canonicalised (duplicates merged) and stored in the lower triangle;
* `Optimizer` (`MOI_wrapper.jl:1-188`): raw attributes (options forwarded to `MPCSolver`,
  "array_type" recorded — every array of this build lives in HBM), `Silent` -> print level,
  `supports` / `supports_constraint`, `copy_to` returning the index map, `optimize`, and the result
  attributes (termination status through the reference's `TERMINATION_STATUS` table, primal status,
  objective value, variable primal, solve time, raw status string, result count).

Julia's MOI is not available to a Python host, so the model side is a small stand-in with MOI's
names and semantics (`Model`, function and set types).  Indices are 0-based here.
ScalarQuadraticFunction follows MOI's convention: a diagonal term (c, x_i, x_i) is 1/2 c x_i^2, an
off-diagonal term (c, x_i, x_j) is c x_i x_j — i.e. exactly the entry H_ij of 1/2 x'Hx.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .qp import QuadraticModel


# ---------------------------------------------------------------- functions
@dataclass(frozen=True)
class VariableIndex:
    value: int


@dataclass(frozen=True)
class ConstraintIndex:
    function_type: type
    set_type: type
    value: int


@dataclass
class ScalarAffineTerm:
    coefficient: float
    variable: VariableIndex


@dataclass
class ScalarAffineFunction:
    terms: list
    constant: float = 0.0


@dataclass
class ScalarQuadraticTerm:
    coefficient: float
    variable_1: VariableIndex
    variable_2: VariableIndex


@dataclass
class ScalarQuadraticFunction:
    quadratic_terms: list
    affine_terms: list
    constant: float = 0.0


@dataclass
class VectorAffineTerm:
    output_index: int
    scalar_term: ScalarAffineTerm


@dataclass
class VectorAffineFunction:
    terms: list
    constants: list


# ---------------------------------------------------------------- sets
@dataclass(frozen=True)
class EqualTo:
    value: float


@dataclass(frozen=True)
class GreaterThan:
    lower: float


@dataclass(frozen=True)
class LessThan:
    upper: float


@dataclass(frozen=True)
class Interval:
    lower: float
    upper: float


@dataclass(frozen=True)
class Nonnegatives:
    dimension: int


@dataclass(frozen=True)
class Nonpositives:
    dimension: int


@dataclass(frozen=True)
class Zeros:
    dimension: int


ALS = (EqualTo, GreaterThan, LessThan, Interval)   # parse_moi.jl:14-19
VLS = (Nonnegatives, Nonpositives, Zeros)          # parse_moi.jl:20
MIN_SENSE, MAX_SENSE, FEASIBILITY_SENSE = "MIN_SENSE", "MAX_SENSE", "FEASIBILITY_SENSE"


def canonicalize(f: ScalarQuadraticFunction) -> ScalarQuadraticFunction:
    """MOI.Utilities.canonicalize!: duplicate terms merged (the pair is unordered), zeros dropped."""
    aff: dict = {}
    for t in f.affine_terms:
        aff[t.variable] = aff.get(t.variable, 0.0) + t.coefficient
    quad: dict = {}
    for t in f.quadratic_terms:
        a, b = t.variable_1, t.variable_2
        key = (a, b) if a.value <= b.value else (b, a)
        quad[key] = quad.get(key, 0.0) + t.coefficient
    f.affine_terms = [ScalarAffineTerm(c, v) for v, c in sorted(aff.items(), key=lambda kv: kv[0].value) if c != 0.0]
    f.quadratic_terms = [ScalarQuadraticTerm(c, a, b) for (a, b), c in
                         sorted(quad.items(), key=lambda kv: (kv[0][0].value, kv[0][1].value)) if c != 0.0]
    return f


# ---------------------------------------------------------------- the model (MOI.ModelLike stand-in)
class Model:
    """A minimal MOI.ModelLike: variables, constraints (function-in-set), objective, primal starts."""

    def __init__(self):
        self._nvar = 0
        self._cons: dict = {}                 # (F, S) -> list of (ConstraintIndex, func, set)
        self._ncons = 0
        self.sense = FEASIBILITY_SENSE
        self.objective = ScalarAffineFunction([], 0.0)
        self.primal_start: dict = {}

    def add_variable(self) -> VariableIndex:
        v = VariableIndex(self._nvar)
        self._nvar += 1
        return v

    def add_variables(self, n: int) -> list:
        return [self.add_variable() for _ in range(n)]

    def add_constraint(self, func, s) -> ConstraintIndex:
        F, S = type(func), type(s)
        if not supports_constraint(F, S):
            raise TypeError(f"unsupported constraint {F.__name__}-in-{S.__name__}")
        if F is VariableIndex and not (0 <= func.value < self._nvar):
            raise ValueError("unknown variable")
        ci = ConstraintIndex(F, S, self._ncons)
        self._ncons += 1
        self._cons.setdefault((F, S), []).append((ci, func, s))
        return ci

    def set_objective(self, sense: str, func) -> None:
        if not isinstance(func, (VariableIndex, ScalarAffineFunction, ScalarQuadraticFunction)):
            raise TypeError("objective must be a VariableIndex, ScalarAffineFunction or ScalarQuadraticFunction")
        self.sense, self.objective = sense, func

    def set_start(self, v: VariableIndex, value) -> None:
        self.primal_start[v] = value

    # MOI.get equivalents used by qp_model
    def list_of_variable_indices(self) -> list:
        return [VariableIndex(i) for i in range(self._nvar)]

    def list_of_constraint_types_present(self) -> list:
        return list(self._cons.keys())

    def constraints(self, F, S) -> list:
        return list(self._cons.get((F, S), []))

    def all_bounds(self):
        """MOI.Utilities.get_bounds for every variable at once: the intersection of the
        VariableIndex-in-set constraints on each, in ONE pass over those constraints."""
        lo = [-math.inf] * self._nvar
        hi = [math.inf] * self._nvar
        for (F, S), lst in self._cons.items():
            if F is not VariableIndex:
                continue
            for _, f, s in lst:
                i = f.value
                if S is EqualTo:
                    lo[i], hi[i] = max(lo[i], s.value), min(hi[i], s.value)
                elif S is GreaterThan:
                    lo[i] = max(lo[i], s.lower)
                elif S is LessThan:
                    hi[i] = min(hi[i], s.upper)
                elif S is Interval:
                    lo[i], hi[i] = max(lo[i], s.lower), min(hi[i], s.upper)
        return lo, hi

    def get_bounds(self, v: VariableIndex):
        """MOI.Utilities.get_bounds: the intersection of the VariableIndex-in-set constraints on v."""
        lo, hi = self.all_bounds()
        return lo[v.value], hi[v.value]


def supports_constraint(F, S) -> bool:
    """MOI_wrapper.jl:85-87."""
    if F in (VariableIndex, ScalarAffineFunction):
        return S in ALS
    if F is VectorAffineFunction:
        return S in VLS
    return False


# ---------------------------------------------------------------- model -> QuadraticModel
def parse_variable(model: Model):
    """parse_moi.jl:22-48: index map, bounds, primal start."""
    vars_ = model.list_of_variable_indices()
    nvar = len(vars_)
    lvar, uvar, x0 = np.zeros(nvar), np.zeros(nvar), np.zeros(nvar)
    index_map = {vi: VariableIndex(i) for i, vi in enumerate(vars_)}
    lo, hi = model.all_bounds()  # one pass over the bound constraints (not one per variable)
    for i, vi in enumerate(vars_):
        lvar[i], uvar[i] = lo[vi.value], hi[vi.value]
        val = model.primal_start.get(vi)
        if val is not None:
            x0[i] = val
    return index_map, nvar, lvar, uvar, x0


def parse_constraints(model: Model, index_map: dict):
    """parse_moi.jl:50-118: linear rows in the order the constraint types are listed."""
    nlin = 0
    rows, cols, vals, lcon, ucon = [], [], [], [], []
    for (F, S) in model.list_of_constraint_types_present():
        for cidx, fun, s in model.constraints(F, S):
            if F is VariableIndex:
                index_map[cidx] = ConstraintIndex(F, S, fun.value)
                continue
            index_map[cidx] = ConstraintIndex(F, S, nlin)
            if F is ScalarAffineFunction:
                for t in fun.terms:
                    rows.append(nlin)
                    cols.append(index_map[t.variable].value)
                    vals.append(t.coefficient)
                if S in (Interval, GreaterThan):
                    lcon.append(-fun.constant + s.lower)
                elif S is EqualTo:
                    lcon.append(-fun.constant + s.value)
                else:
                    lcon.append(-math.inf)
                if S in (Interval, LessThan):
                    ucon.append(-fun.constant + s.upper)
                elif S is EqualTo:
                    ucon.append(-fun.constant + s.value)
                else:
                    ucon.append(math.inf)
                nlin += 1
            elif F is VectorAffineFunction:
                if len(fun.constants) != s.dimension:
                    raise ValueError("VectorAffineFunction constants do not match the set dimension")
                for t in fun.terms:
                    if not (0 <= t.output_index < s.dimension):
                        raise ValueError("VectorAffineTerm output_index out of range")
                    rows.append(nlin + t.output_index)
                    cols.append(index_map[t.scalar_term.variable].value)
                    vals.append(t.scalar_term.coefficient)
                neg = [-c for c in fun.constants]
                lcon.extend(neg if S in (Nonnegatives, Zeros) else [-math.inf] * s.dimension)
                ucon.extend(neg if S in (Nonpositives, Zeros) else [math.inf] * s.dimension)
                nlin += s.dimension
    return rows, cols, vals, lcon, ucon


def parse_objective(model: Model, index_map: dict, nvar: int):
    """parse_moi.jl:120-166: c, the constant and the (row >= col) quadratic terms."""
    constant = 0.0
    vect = np.zeros(nvar)
    rows, cols, vals = [], [], []
    f = model.objective
    if isinstance(f, VariableIndex):
        vect[index_map[f].value] = 1.0
    elif isinstance(f, ScalarAffineFunction):
        constant = f.constant
        for t in f.terms:
            vect[index_map[t.variable].value] += t.coefficient
    elif isinstance(f, ScalarQuadraticFunction):
        canonicalize(f)
        constant = f.constant
        for t in f.affine_terms:
            vect[index_map[t.variable].value] += t.coefficient
        for t in f.quadratic_terms:
            i, j = index_map[t.variable_1].value, index_map[t.variable_2].value
            rows.append(max(i, j))
            cols.append(min(i, j))
            vals.append(t.coefficient)
    return rows, cols, vals, vect, constant


def qp_model(model: Model):
    """parse_moi.jl:168-215: the QuadraticModel and the index map."""
    index_map, nvar, lvar, uvar, x0 = parse_variable(model)
    Ai, Aj, Ax, lb, ub = parse_constraints(model, index_map)
    Qi, Qj, Qx, c, d = parse_objective(model, index_map, nvar)
    ncon = len(lb)
    qp = QuadraticModel(c=c, Hrows=np.asarray(Qi, np.int64), Hcols=np.asarray(Qj, np.int64),
                        Hvals=np.asarray(Qx, np.float64), Arows=np.asarray(Ai, np.int64),
                        Acols=np.asarray(Aj, np.int64), Avals=np.asarray(Ax, np.float64),
                        lcon=np.asarray(lb, np.float64), ucon=np.asarray(ub, np.float64), lvar=lvar, uvar=uvar,
                        c0=float(d), x0=x0, y0=np.zeros(ncon), minimize=model.sense == MIN_SENSE, name="moi")
    return qp, index_map


# ---------------------------------------------------------------- the optimizer
# MOI.TerminationStatusCode per MadNLP status (MOI_wrapper.jl:131-151), by the status names of
# madipm_amd.solver (MadNLP.Status values)
TERMINATION_STATUS = {
    "SOLVE_SUCCEEDED": "OPTIMAL",
    "SOLVED_TO_ACCEPTABLE_LEVEL": "ALMOST_OPTIMAL",
    "SEARCH_DIRECTION_BECOMES_TOO_SMALL": "SLOW_PROGRESS",
    "DIVERGING_ITERATES": "INFEASIBLE_OR_UNBOUNDED",
    "INFEASIBLE_PROBLEM_DETECTED": "INFEASIBLE",
    "MAXIMUM_ITERATIONS_EXCEEDED": "ITERATION_LIMIT",
    "MAXIMUM_WALLTIME_EXCEEDED": "TIME_LIMIT",
    "INITIAL": "OPTIMIZE_NOT_CALLED",
    "RESTORATION_FAILED": "NUMERICAL_ERROR",
    "INVALID_NUMBER_DETECTED": "INVALID_MODEL",
    "ERROR_IN_STEP_COMPUTATION": "NUMERICAL_ERROR",
    "NOT_ENOUGH_DEGREES_OF_FREEDOM": "INVALID_MODEL",
    "USER_REQUESTED_STOP": "INTERRUPTED",
    "INTERNAL_ERROR": "OTHER_ERROR",
    "INVALID_NUMBER_OBJECTIVE": "INVALID_MODEL",
    "INVALID_NUMBER_GRADIENT": "INVALID_MODEL",
    "INVALID_NUMBER_CONSTRAINTS": "INVALID_MODEL",
    "INVALID_NUMBER_JACOBIAN": "INVALID_MODEL",
    "INVALID_NUMBER_HESSIAN_LAGRANGIAN": "INVALID_MODEL",
}


class Optimizer:
    """MadIPM.Optimizer (MOI_wrapper.jl:2-15) over the GPU MPCSolver."""

    def __init__(self):
        self.options: dict = {}
        self.silent = False
        self.solver = None
        self.qp: QuadraticModel | None = None
        self.array_type = "HBM"
        self.stats = None

    # MOI.SolverName / is_empty / empty! (MOI_wrapper.jl:17-26)
    solver_name = "MadIPM"

    def is_empty(self) -> bool:
        return self.solver is None and self.qp is None

    def empty(self) -> None:
        self.solver = self.qp = self.stats = None

    # RawOptimizerAttribute (:32-43) and Silent (:49-56)
    def set_attribute(self, name: str, value) -> None:
        if name == "array_type":
            self.array_type = value      # recorded only: every solver array is device-resident here
        else:
            self.options[name] = value

    def get_attribute(self, name: str):
        return self.options[name]

    def set_silent(self, value: bool) -> None:
        self.silent = bool(value)

    def get_silent(self) -> bool:
        return self.silent

    @staticmethod
    def supports(attr: str, typ=None) -> bool:
        """ObjectiveSense, ObjectiveFunction{VI|SAF|SQF}, Silent, VariablePrimalStart (:49, :62-79)."""
        if attr == "ObjectiveFunction":
            return typ in (VariableIndex, ScalarAffineFunction, ScalarQuadraticFunction)
        return attr in ("ObjectiveSense", "Silent", "VariablePrimalStart")

    supports_constraint = staticmethod(supports_constraint)

    def copy_to(self, src: Model) -> dict:
        """MOI.copy_to (:89-97)."""
        self.qp, index_map = qp_model(src)
        return index_map

    def optimize(self) -> None:
        """MOI.optimize! (:99-111): options forwarded to MPCSolver, Silent -> print level."""
        from .solver import MPCSolver
        if self.qp is None:
            raise RuntimeError("optimize: no model (call copy_to first)")
        opts = {k: v for k, v in self.options.items() if k != "solver"}
        opts["print_level"] = 0 if self.silent else 1
        self.solver = MPCSolver(self.qp, **opts)
        self.stats = self.solver.solve()

    # result attributes (:113-188)
    def solve_time_sec(self) -> float:
        return self.stats.counters.total_time

    def raw_status_string(self) -> str:
        return self.stats.status_name

    def raw_status(self, name: str):
        return getattr(self.stats, name)

    def termination_status(self) -> str:
        if self.stats is None:
            return "OPTIMIZE_NOT_CALLED"
        return TERMINATION_STATUS[self.stats.status_name]

    def result_count(self) -> int:
        return 1

    def _check_result_index(self, result_index: int) -> None:
        if self.stats is None or not (1 <= result_index <= self.result_count()):
            raise ValueError(f"result index {result_index} out of bounds (MOI.check_result_index_bounds)")

    def objective_value(self, result_index: int = 1) -> float:
        self._check_result_index(result_index)
        return self.stats.objective

    def primal_status(self, result_index: int = 1) -> str:
        if result_index > self.result_count() or self.stats is None:
            return "NO_SOLUTION"
        ts = self.termination_status()
        if ts == "OPTIMAL":
            return "FEASIBLE_POINT"
        if ts == "INFEASIBLE":
            return "INFEASIBLE_POINT"
        return "UNKNOWN_RESULT_STATUS"

    def dual_status(self, result_index: int = 1) -> str:
        return "NO_SOLUTION"          # as the reference (MOI_wrapper.jl:178-181)

    def variable_primal(self, vi: VariableIndex, result_index: int = 1) -> float:
        self._check_result_index(result_index)
        return float(self.stats.solution[vi.value])
