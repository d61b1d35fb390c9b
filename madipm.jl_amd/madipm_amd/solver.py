"""Host-side mirror of MadIPM's public interface over the native (HIP) solver.

Same names and argument meaning as the reference (src/MadIPM.jl exports `MPCSolver`, `madipm`;
options are IPMOptions fields, src/utils.jl:69-105; types src/utils.jl:10-48):

    solver = MPCSolver(qp; tol=1e-8, max_iter=300, linear_solver=HIPLDLSolver,
                       regularization=FixedRegularization(1e-8, -1e-8), step_rule=AdaptiveStep(0.99))
    stats = solver.solve()          # solve!(solver)
    stats = madipm(qp; kwargs...)   # madipm(m; kwargs...)

Every computation of the solve runs in libmadipm_hip on the GPU; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .linear_solver import HIPLDLSolver
from .qp import QuadraticModel


# ---------------------------------------------------------------- option types (src/utils.jl:10-48)
class AbstractBarrierUpdate: ...


class Mehrotra(AbstractBarrierUpdate): ...


@dataclass
class ConservativeStep:
    tau: float = 0.995


@dataclass
class AdaptiveStep:
    tau_min: float = 0.99


@dataclass
class MehrotraAdaptiveStep:
    gamma_f: float = 0.99


@dataclass
class NoRegularization: ...


@dataclass
class FixedRegularization:
    delta_p: float
    delta_d: float


@dataclass
class AdaptiveRegularization:
    delta_p: float
    delta_d: float
    delta_min: float


class SparseKKTSystem: ...          # K2 (MadNLP.SparseKKTSystem)


class ScaledSparseKKTSystem: ...    # K2.5 (MadNLP.ScaledSparseKKTSystem; src/kernels.jl:139-149)


class NormalKKTSystem: ...          # src/KKT/normalkkt.jl (LPs only; A Sigma^-1 A^T, Cholesky semantics)


_KKT_CODES = {SparseKKTSystem: 0, ScaledSparseKKTSystem: 1, NormalKKTSystem: 2}


# MadNLP.Status
STATUS_NAMES = {
    0: "REGULAR", 1: "SOLVE_SUCCEEDED", 2: "INFEASIBLE_PROBLEM_DETECTED",
    -1: "MAXIMUM_ITERATIONS_EXCEEDED", -2: "MAXIMUM_WALLTIME_EXCEEDED", -3: "DIVERGING_ITERATES",
    -4: "ERROR_IN_STEP_COMPUTATION", -5: "INTERNAL_ERROR",
}
SOLVE_SUCCEEDED = 1
INFEASIBLE_PROBLEM_DETECTED = 2
MAXIMUM_ITERATIONS_EXCEEDED = -1
MAXIMUM_WALLTIME_EXCEEDED = -2
DIVERGING_ITERATES = -3
ERROR_IN_STEP_COMPUTATION = -4
INTERNAL_ERROR = -5


class Options(C.Structure):
    _fields_ = [("tol", C.c_double), ("max_iter", C.c_int32), ("max_wall_time", C.c_double),
                ("divergence_tol", C.c_double), ("scaling", C.c_int32), ("bound_push", C.c_double),
                ("bound_fac", C.c_double), ("bound_relax_factor", C.c_double), ("regularization", C.c_int32),
                ("delta_p", C.c_double), ("delta_d", C.c_double), ("delta_min", C.c_double),
                ("step_rule", C.c_int32), ("step_tau", C.c_double), ("max_ncorr", C.c_int32),
                ("mu_init", C.c_double), ("mu_min", C.c_double), ("tol_linear_solve", C.c_double),
                ("check_residual", C.c_int32), ("kkt_system", C.c_int32), ("print_level", C.c_int32),
                ("ldl", L.LDLOpts)]


class QPStruct(C.Structure):
    _fields_ = [("nvar", C.c_int32), ("ncon", C.c_int32), ("nnzh", C.c_int64), ("nnzj", C.c_int64),
                ("c", L.f64p), ("c0", C.c_double), ("Hrows", L.i32p), ("Hcols", L.i32p), ("Hvals", L.f64p),
                ("Arows", L.i32p), ("Acols", L.i32p), ("Avals", L.f64p), ("lcon", L.f64p), ("ucon", L.f64p),
                ("lvar", L.f64p), ("uvar", L.f64p), ("x0", L.f64p), ("y0", L.f64p), ("minimize", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("status", C.c_int32), ("iter", C.c_int32), ("objective", C.c_double),
                ("dual_objective", C.c_double), ("inf_pr", C.c_double), ("inf_du", C.c_double),
                ("inf_compl", C.c_double), ("mu", C.c_double), ("total_time", C.c_double),
                ("linear_solver_time", C.c_double), ("init_time", C.c_double), ("exception", C.c_int32)]


# The exceptions solve!'s catch-all turns into INTERNAL_ERROR (src/solver.jl:398-403) and rethrows
# when rethrow_error = true (the reference benchmark sets it, scripts/benchmarks_cpu.jl:39).
class SolveException(Exception):
    """MadNLP.SolveException, thrown (as a type) by solve_system! (src/linear_solver.jl:40-41)."""


class UnfactorizedSolveException(Exception):
    """The linear solver refusing a solve after every trial of factorize_regularized_system!
    (src/linear_solver.jl:6-17) failed (LDLFactorizations' ldiv! on an unfactorized object [EXT])."""


EXC_NONE, EXC_SOLVE, EXC_UNFACTORIZED = 0, 1, 2
_EXCEPTIONS = {EXC_SOLVE: SolveException, EXC_UNFACTORIZED: UnfactorizedSolveException}


class IterTrace(C.Structure):
    _fields_ = [("k", C.c_int32), ("obj", C.c_double), ("inf_pr", C.c_double), ("inf_du", C.c_double),
                ("inf_compl", C.c_double), ("mu", C.c_double), ("alpha_p", C.c_double),
                ("alpha_d", C.c_double), ("del_w", C.c_double), ("dx_inf", C.c_double),
                ("residual", C.c_double)]


L._sig("madipm_default_options", None, [C.POINTER(Options)])
L._sig("madipm_solver_create", C.c_int, [C.POINTER(QPStruct), C.POINTER(Options), C.POINTER(L.vp)])
L._sig("madipm_solver_create_dist", C.c_int, [C.POINTER(QPStruct), C.POINTER(Options), L.vp, C.POINTER(L.vp)])
L._sig("madipm_solver_solve", C.c_int, [L.vp, C.POINTER(Stats)])
L._sig("madipm_solver_initialize", C.c_int, [L.vp])
L._sig("madipm_solver_set_max_iter", C.c_int, [L.vp, C.c_int32])
L._sig("madipm_solver_get_solution", C.c_int, [L.vp, L.f64p, L.f64p, L.f64p, L.f64p, L.f64p])
L._sig("madipm_solver_trace", C.c_int, [L.vp, C.POINTER(IterTrace), C.c_int32])
L._sig("madipm_solver_ldl_info", C.c_int, [L.vp, C.POINTER(L.LDLInfo)])
L._sig("madipm_solver_ldl_perm", C.c_int, [L.vp, L.i32p])
L._sig("madipm_solver_set_timing", C.c_int, [L.vp, C.c_uint32])
L._sig("madipm_solver_kernel_stats", C.c_int, [L.vp, C.POINTER(L.KStat)])
L._sig("madipm_solver_destroy", None, [L.vp])


class RCCLComm:
    """RCCL communicator of the sharded factorisation (one process per GPU; madipm_comm_*).

    `RCCLComm.from_torch(dist)` makes rank 0's 128-byte unique id, broadcasts it with the
    torch.distributed process group (any backend), and joins the communicator."""

    def __init__(self, rank: int, size: int, uid: bytes):
        assert len(uid) == 128
        self.rank, self.size = int(rank), int(size)
        h = L.vp()
        L.check(L.lib.madipm_comm_create(self.size, self.rank, uid, C.byref(h)), "madipm_comm_create")
        self.h = h

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        L.check(L.lib.madipm_comm_unique_id(buf), "madipm_comm_unique_id")
        return buf.raw

    @classmethod
    def from_torch(cls, dist) -> "RCCLComm":
        rank, size = dist.get_rank(), dist.get_world_size()
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return cls(rank, size, box[0])

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            L.lib.madipm_comm_destroy(h)
            self.h = None


class HostComm:
    """Host-staged communicator over a torch.distributed process group (e.g. gloo): every all-reduce
    goes device -> pinned host -> dist.all_reduce -> device.  For exercising the multi-process
    sharded path where RCCL cannot run (several ranks on one GPU); RCCLComm is the data path."""

    def __init__(self, dist):
        import torch
        self.rank, self.size = dist.get_rank(), dist.get_world_size()

        def _fn(p, n, _ctx):
            try:
                a = np.ctypeslib.as_array(p, shape=(int(n),))
                t = torch.from_numpy(a)
                dist.all_reduce(t)
                return 0
            except Exception:  # pragma: no cover - reported as a C error
                return -1
        self._cb = L.ALLREDUCE_FN(_fn)
        h = L.vp()
        L.check(L.lib.madipm_comm_create_host(self.size, self.rank, self._cb, None, C.byref(h)), "madipm_comm_create_host")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            L.lib.madipm_comm_destroy(h)
            self.h = None


@dataclass
class Counters:
    """MadNLP.MadNLPCounters subset reported by the reference benchmarks (scripts/benchmarks_cpu.jl:49-50)."""
    k: int = 0
    total_time: float = 0.0
    linear_solver_time: float = 0.0
    init_time: float = 0.0


@dataclass
class ExecutionStats:
    """MadNLP.MadNLPExecutionStats as filled by update_solution! (src/utils.jl:150-156)."""
    status: int
    iter: int
    objective: float
    dual_objective: float
    solution: np.ndarray
    constraints: np.ndarray
    multipliers: np.ndarray
    multipliers_L: np.ndarray
    multipliers_U: np.ndarray
    primal_feas: float
    dual_feas: float
    inf_compl: float
    counters: Counters
    trace: list = field(default_factory=list)

    @property
    def status_name(self) -> str:
        return STATUS_NAMES.get(self.status, str(self.status))


_KNOWN = {"tol", "max_iter", "max_wall_time", "divergence_tol", "scaling", "bound_push", "bound_fac",
          "bound_relax_factor", "regularization", "step_rule", "barrier_update", "max_ncorr", "mu_init",
          "mu_min", "tol_linear_solve", "check_residual", "kkt_system", "linear_solver", "print_level",
          "rethrow_error", "ordering", "relax", "pivot_tol", "small_front_max", "dense_alpha",
          "output_file", "file_print_level", "kappa_d", "s_max", "mu_superlinear_decrease_power", "tau_min",
          "fixed_variable_treatment", "equality_treatment", "nshards", "comm"}


def load_options(**kw) -> Options:
    """load_options (src/utils.jl:121-148): IPM options + linear-solver options."""
    unknown = set(kw) - _KNOWN
    if unknown:
        # MadNLP.print_ignored_options (src/utils.jl:140-142): unsupported options are reported, not fatal
        import sys
        print("The following options are ignored: " + ", ".join(f"{k} = {kw[k]!r}" for k in sorted(unknown)),
              file=sys.stderr)
    o = Options()
    L.lib.madipm_default_options(C.byref(o))
    for k in ("tol", "max_iter", "max_wall_time", "divergence_tol", "bound_push", "bound_fac",
              "bound_relax_factor", "max_ncorr", "mu_init", "mu_min", "tol_linear_solve"):
        if k in kw:
            setattr(o, k, kw[k])
    if "scaling" in kw:
        o.scaling = int(bool(kw["scaling"]))
    if "check_residual" in kw:
        o.check_residual = int(bool(kw["check_residual"]))
    reg = kw.get("regularization", FixedRegularization(1e-10, 1e-10))
    if isinstance(reg, NoRegularization):
        o.regularization = 0
    elif isinstance(reg, FixedRegularization):
        o.regularization, o.delta_p, o.delta_d = 1, reg.delta_p, reg.delta_d
    elif isinstance(reg, AdaptiveRegularization):
        o.regularization, o.delta_p, o.delta_d, o.delta_min = 2, reg.delta_p, reg.delta_d, reg.delta_min
    else:
        raise TypeError(f"unsupported regularization {reg!r}")
    rule = kw.get("step_rule", AdaptiveStep(0.99))
    if isinstance(rule, ConservativeStep):
        o.step_rule, o.step_tau = 0, rule.tau
    elif isinstance(rule, AdaptiveStep):
        o.step_rule, o.step_tau = 1, rule.tau_min
    elif isinstance(rule, MehrotraAdaptiveStep):
        o.step_rule, o.step_tau = 2, rule.gamma_f
    else:
        raise TypeError(f"unsupported step rule {rule!r}")
    kkt = kw.get("kkt_system", SparseKKTSystem)
    if kkt not in _KKT_CODES:
        raise TypeError(f"unsupported kkt_system {getattr(kkt, '__name__', kkt)!r}")
    o.kkt_system = _KKT_CODES[kkt]
    ls = kw.get("linear_solver", HIPLDLSolver)
    if ls is not HIPLDLSolver:
        raise NotImplementedError("linear_solver must be HIPLDLSolver (the GPU LDL^T)")
    o.print_level = int(kw.get("print_level", 0))
    for k in ("ordering", "relax", "small_front_max", "nshards"):
        if k in kw:
            setattr(o.ldl, k, int(kw[k]))
    for k in ("pivot_tol", "dense_alpha"):
        if k in kw:
            setattr(o.ldl, k, float(kw[k]))
    return o


class MPCSolver:
    """`MPCSolver(nlp; kwargs...)` (src/structure.jl:79-178) on the GPU."""

    def __init__(self, qp: QuadraticModel, **kwargs):
        self.qp = qp
        self.options = load_options(**kwargs)
        self.rethrow_error = bool(kwargs.get("rethrow_error", False))
        self._keep = []
        q = QPStruct()
        q.nvar, q.ncon = qp.nvar, qp.ncon
        q.nnzh, q.nnzj = qp.nnzh, qp.nnzj

        def f64(a):
            a = np.ascontiguousarray(a, np.float64)
            self._keep.append(a)
            return L.ptr(a, C.c_double)

        def i32(a):
            a = np.ascontiguousarray(a, np.int32)
            self._keep.append(a)
            return L.ptr(a, C.c_int32)

        q.c, q.c0 = f64(qp.c), float(qp.c0)
        q.Hrows, q.Hcols, q.Hvals = i32(qp.Hrows), i32(qp.Hcols), f64(qp.Hvals)
        q.Arows, q.Acols, q.Avals = i32(qp.Arows), i32(qp.Acols), f64(qp.Avals)
        q.lcon, q.ucon, q.lvar, q.uvar = f64(qp.lcon), f64(qp.ucon), f64(qp.lvar), f64(qp.uvar)
        q.x0, q.y0 = f64(qp.x0), f64(qp.y0)
        q.minimize = int(bool(qp.minimize))
        self._q = q
        h = L.vp()
        comm = kwargs.get("comm")
        if comm is not None and comm.size > 1:
            # subtree-sharded factorisation across the processes of `comm` (SURVEY §8 e)
            self._comm = comm
            L.check(L.lib.madipm_solver_create_dist(C.byref(q), C.byref(self.options), comm.h, C.byref(h)),
                    "MPCSolver")
        else:
            L.check(L.lib.madipm_solver_create(C.byref(q), C.byref(self.options), C.byref(h)), "MPCSolver")
        self.h = h

    def ldl_info(self) -> dict:
        inf = L.LDLInfo()
        L.check(L.lib.madipm_solver_ldl_info(self.h, C.byref(inf)), "ldl_info")
        return inf.as_dict()

    def kkt_perm(self) -> np.ndarray:
        """Pivot order of the K2 LDL^T (analysis output), over the K2 unknowns [x; s; y]."""
        n = self.ldl_info()["n"]
        p = np.empty(n, np.int32)
        L.check(L.lib.madipm_solver_ldl_perm(self.h, L.ptr(p, C.c_int32)), "kkt_perm")
        return p

    def set_kernel_timing(self, mask: int = (1 << L.NKERNELS) - 1):
        """Record HIP events around every launch of the LDL^T kernel kinds in `mask` (bit k = kind k,
        include/madipm_hip.h); clears the statistics.  mask=0 turns timing off."""
        L.check(L.lib.madipm_solver_set_timing(self.h, int(mask)), "set_timing")

    def kernel_stats(self) -> list:
        """Per kernel kind: launches, summed event time (ms), algorithmic bytes and flops."""
        arr = (L.KStat * L.NKERNELS)()
        L.check(L.lib.madipm_solver_kernel_stats(self.h, arr), "kernel_stats")
        return L.kstats_to_list(arr)

    def initialize(self):
        """initialize! alone (src/solver.jl:127-189); the next solve() runs only the MPC loop."""
        L.check(L.lib.madipm_solver_initialize(self.h), "initialize!")

    def set_max_iter(self, k: int):
        L.check(L.lib.madipm_solver_set_max_iter(self.h, int(k)), "set_max_iter")

    def solve(self, fetch_solution: bool = True) -> ExecutionStats:
        """solve!(solver) (src/solver.jl:362-418).  fetch_solution=False skips update_solution!'s
        device-to-host copies of x, y, z_L, z_U and the constraint values (the reference runs it after
        cnt.total_time is taken, solver.jl:406-413); the returned arrays are then None."""
        st = Stats()
        rc = L.lib.madipm_solver_solve(self.h, C.byref(st))
        if rc < 0:
            # solve!'s catch-all (src/solver.jl:398-403): INTERNAL_ERROR, rethrown only with rethrow_error
            if self.rethrow_error:
                L.check(rc, "solve!")
            st.status = INTERNAL_ERROR
            st.iter = len(self.trace()) - 1 if self.trace() else 0
        elif st.status == INTERNAL_ERROR and st.exception in _EXCEPTIONS and self.rethrow_error:
            raise _EXCEPTIONS[st.exception](
                "MPC loop: " + ("residual check of solve_system! (src/linear_solver.jl:40-41)"
                                if st.exception == EXC_SOLVE else "solve with an unfactorized KKT system"))
        if not fetch_solution:
            return ExecutionStats(status=st.status, iter=st.iter, objective=st.objective,
                                  dual_objective=st.dual_objective, solution=None, constraints=None,
                                  multipliers=None, multipliers_L=None, multipliers_U=None, primal_feas=st.inf_pr,
                                  dual_feas=st.inf_du, inf_compl=st.inf_compl,
                                  counters=Counters(k=st.iter, total_time=st.total_time,
                                                    linear_solver_time=st.linear_solver_time, init_time=st.init_time),
                                  trace=None)
        nx, m = self.qp.nvar, self.qp.ncon
        x, zl, zu = np.empty(nx), np.empty(nx), np.empty(nx)
        y, cons = np.empty(m), np.empty(m)
        rs = L.lib.madipm_solver_get_solution(self.h, L.ptr(x, C.c_double), L.ptr(y, C.c_double),
                                              L.ptr(zl, C.c_double), L.ptr(zu, C.c_double), L.ptr(cons, C.c_double))
        if rs < 0:
            if rc >= 0:
                L.check(rs, "get_solution")
            for a in (x, y, zl, zu, cons):
                a.fill(np.nan)
        return ExecutionStats(status=st.status, iter=st.iter, objective=st.objective,
                              dual_objective=st.dual_objective, solution=x, constraints=cons,
                              multipliers=y, multipliers_L=zl, multipliers_U=zu, primal_feas=st.inf_pr,
                              dual_feas=st.inf_du, inf_compl=st.inf_compl,
                              counters=Counters(k=st.iter, total_time=st.total_time,
                                                linear_solver_time=st.linear_solver_time, init_time=st.init_time),
                              trace=self.trace())

    def trace(self) -> list:
        n = L.check(L.lib.madipm_solver_trace(self.h, None, 0), "trace")
        buf = (IterTrace * max(n, 1))()
        L.lib.madipm_solver_trace(self.h, buf, n)
        return [{k: getattr(buf[i], k) for k, _ in IterTrace._fields_} for i in range(n)]

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            L.lib.madipm_solver_destroy(h)
            self.h = None


def solve(solver: MPCSolver) -> ExecutionStats:
    """`solve!(solver)` as a free function."""
    return solver.solve()


def madipm(qp: QuadraticModel, **kwargs) -> ExecutionStats:
    """`madipm(m; kwargs...)` (src/solver.jl:425-428)."""
    return MPCSolver(qp, **kwargs).solve()
