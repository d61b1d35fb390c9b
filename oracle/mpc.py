"""ORACLE (test infrastructure only) — CPU restatement of MadIPM's MPC solver, K2 formulation.

Each function cites the reference file:line it restates (paths relative to /root/reference).
Semantics of MadNLP 0.8 (callbacks, scaling, K2 layout, reduce_rhs!/finish_aug_solve!,
_kktmul!, adjust_boundary!) are restated from SURVEY.md Appendix B and tagged [EXT].

The linear algebra is deliberately independent from the product: the K2 system is assembled
with scipy.sparse and solved with SuperLU (`scipy.sparse.linalg.splu`, partial pivoting).
The product factorises the same matrix with its own supernodal LDL^T on the GPU.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

INF = math.inf

# MadNLP status codes (MadNLP.Status, [EXT]) — only the ones MadIPM sets.
REGULAR = 0
SOLVE_SUCCEEDED = 1
MAXIMUM_ITERATIONS_EXCEEDED = -1
MAXIMUM_WALLTIME_EXCEEDED = -2
DIVERGING_ITERATES = -3
INFEASIBLE_PROBLEM_DETECTED = 2
ERROR_IN_STEP_COMPUTATION = -4
INTERNAL_ERROR = -5


class SolveException(Exception):
    """MadNLP.SolveException: src/linear_solver.jl:41 throws the TYPE (`throw(MadNLP.SolveException)`),
    and a DataType is never `isa MadNLP.LinearSolverException`, so solve! (src/solver.jl:379-405) lands
    in its catch-all: INTERNAL_ERROR, rethrown when rethrow_error (the benchmark scripts set it,
    scripts/benchmarks_cpu.jl:39).  [EXT assumption: SolveException is a type, as in MadNLP 0.8.]"""


class UnfactorizedSolveException(Exception):
    """The linear solver refusing to solve with an unfactorized matrix (after every trial of
    factorize_regularized_system!, src/linear_solver.jl:6-17, failed): LDLFactorizations' ldiv!
    throws an exception that is no LinearSolverException [EXT] -> INTERNAL_ERROR as above."""


EXC_NONE, EXC_SOLVE, EXC_UNFACTORIZED = 0, 1, 2


@dataclass
class OracleOptions:
    """IPMOptions defaults, src/utils.jl:69-105."""
    tol: float = 1e-8
    max_iter: int = 3000
    max_wall_time: float = 1e6
    divergence_tol: float = 1e4
    scaling: bool = True
    bound_push: float = 1e-2
    bound_fac: float = 1e-2
    bound_relax_factor: float = 1e-12
    # regularization: ("fixed", delta_p, delta_d) | ("none",) | ("adaptive", dp, dd, dmin)
    regularization: tuple = ("fixed", 1e-10, 1e-10)
    # step_rule: ("adaptive", tau_min) | ("conservative", tau) | ("mehrotra", gamma_f)
    step_rule: tuple = ("adaptive", 0.99)
    max_ncorr: int = 0
    mu_init: float = 1e-1
    mu_min: float = 1e-12
    tol_linear_solve: float = 1e-8
    check_residual: bool = False
    rethrow_error: bool = False
    kkt_system: str = "K2"     # "K2" (SparseKKTSystem) | "K25" (ScaledSparseKKTSystem) | "normal"


@dataclass
class OracleStats:
    status: int = REGULAR
    iter: int = 0
    objective: float = 0.0
    solution: np.ndarray | None = None
    constraints: np.ndarray | None = None
    multipliers: np.ndarray | None = None
    multipliers_L: np.ndarray | None = None
    multipliers_U: np.ndarray | None = None
    total_time: float = 0.0
    linear_solver_time: float = 0.0
    trace: list = field(default_factory=list)
    exception: int = EXC_NONE


def get_index_constraints(lvar, uvar, lcon, ucon):
    """MadNLP.get_index_constraints with EnforceEquality + MakeParameter [EXT]
    (called at src/structure.jl:97-104; defaults src/utils.jl:83-84)."""
    ind_ineq = np.flatnonzero(lcon != ucon)
    xl = np.concatenate([lvar, lcon[ind_ineq]])
    xu = np.concatenate([uvar, ucon[ind_ineq]])
    ind_fixed = np.flatnonzero(xl == xu)
    ind_lb = np.flatnonzero((xl != -INF) & (xl != xu))
    ind_ub = np.flatnonzero((xu != INF) & (xl != xu))
    ind_llb = np.flatnonzero((lvar != -INF) & (uvar == INF))
    ind_uub = np.flatnonzero((lvar == -INF) & (uvar != INF))
    return dict(ind_ineq=ind_ineq, ind_fixed=ind_fixed, ind_lb=ind_lb, ind_ub=ind_ub,
                ind_llb=ind_llb, ind_uub=ind_uub)


class OracleMPC:
    """Restatement of `MPCSolver` (src/structure.jl:1-178) + `solve!` (src/solver.jl:362-418)."""

    def __init__(self, qp, opt: OracleOptions | None = None, record_trace: bool = True):
        self.opt = opt or OracleOptions()
        self.qp = qp
        self.record_trace = record_trace
        self.residuals = []          # residual ratio of every solve_system! call (diagnostics)
        nx = int(len(qp.c))
        m = int(len(qp.lcon))
        lvar = np.asarray(qp.lvar, float)
        uvar = np.asarray(qp.uvar, float)
        lcon = np.asarray(qp.lcon, float)
        ucon = np.asarray(qp.ucon, float)
        idx = get_index_constraints(lvar, uvar, lcon, ucon)
        self.ind_ineq = idx["ind_ineq"]
        self.ind_fixed = idx["ind_fixed"]
        self.ind_lb = idx["ind_lb"]
        self.ind_ub = idx["ind_ub"]
        # NOTE src/structure.jl:172-173 passes (ind_llb, ind_uub, ind_lb, ind_ub) into the fields
        # declared (ind_lb, ind_ub, ind_llb, ind_uub) (structure.jl:48-51).  The only reader of
        # the swapped fields is update_barrier! (kernels.jl:211), which therefore tests
        # length(ind_cons.ind_lb) + length(ind_cons.ind_ub) > 0.  Reproduced here.
        self.has_inequalities = (len(idx["ind_lb"]) + len(idx["ind_ub"])) > 0
        self.nx = nx
        self.ns = len(self.ind_ineq)
        self.n = nx + self.ns
        self.m = m
        self.nlb = len(self.ind_lb)
        self.nub = len(self.ind_ub)
        self._lvar, self._uvar, self._lcon, self._ucon = lvar, uvar, lcon, ucon
        # Problem data (0-based COO; H lower triangle)
        self.c_obj = np.asarray(qp.c, float)
        self.c0 = float(getattr(qp, "c0", 0.0))
        self.Hr = np.asarray(qp.Hrows, np.int64)
        self.Hc = np.asarray(qp.Hcols, np.int64)
        self.Hv = np.asarray(qp.Hvals, float)
        self.Ar = np.asarray(qp.Arows, np.int64)
        self.Ac = np.asarray(qp.Acols, np.int64)
        self.Av = np.asarray(qp.Avals, float)
        self.minimize = bool(getattr(qp, "minimize", True))
        # MadNLP callbacks minimise obj_sign * f (obj_sign = -1 for maximisation) [EXT];
        # update_solution! (src/utils.jl:150-156) flips the reported objective back.
        sgn = 1.0 if self.minimize else -1.0
        self.c_obj = sgn * self.c_obj
        self.c0 = sgn * self.c0
        self.Hv = sgn * self.Hv
        x0 = getattr(qp, "x0", None)
        y0 = getattr(qp, "y0", None)
        self._x0 = np.zeros(nx) if x0 is None else np.asarray(x0, float).copy()
        self._y0 = np.zeros(m) if y0 is None else np.asarray(y0, float).copy()
        # full symmetric H (unscaled) and A (unscaled) as CSR for model evaluation
        Hl = sp.coo_matrix((self.Hv, (self.Hr, self.Hc)), shape=(nx, nx)).tocsr()
        self._Hsym = (Hl + Hl.T - sp.diags(Hl.diagonal())).tocsr()
        self._A = sp.coo_matrix((self.Av, (self.Ar, self.Ac)), shape=(m, nx)).tocsr()
        # fixed-variable masks (MakeParameter [EXT])
        self._fixed_mask = np.zeros(self.n, bool)
        self._fixed_mask[self.ind_fixed] = True
        self.linear_solver_time = 0.0
        self.trace: list = []

    # ------------------------------------------------------------------ model callbacks [EXT]
    def _obj(self, x):
        xv = x[: self.nx]
        return self.c0 + self.c_obj @ xv + 0.5 * xv @ (self._Hsym @ xv)

    def eval_f(self, x):
        """MadNLP.eval_f_wrapper: obj_scale * obj(x) [EXT] (src/solver.jl:166,320)."""
        return self.obj_scale * self._obj(x)

    def eval_grad(self, x):
        """MadNLP.eval_grad_f_wrapper!: f = obj_scale*(Hx+c), slacks 0, fixed 0 [EXT]."""
        f = np.zeros(self.n)
        xv = x[: self.nx]
        f[: self.nx] = self.obj_scale * (self._Hsym @ xv + self.c_obj)
        f[self._fixed_mask] = 0.0
        return f

    def eval_cons(self, x):
        """MadNLP.eval_cons_wrapper!: c = con_scale.*(A x); c[ind_ineq] -= s; c -= rhs [EXT]."""
        cval = self.con_scale * (self._A @ x[: self.nx])
        cval[self.ind_ineq] -= x[self.nx:]
        cval -= self.rhs
        return cval

    def jtprod(self, y):
        """MadNLP.jtprod!(jacl, kkt, y) = jac_com' * y, including slack -1 entries [EXT]
        (src/solver.jl:37,187,324)."""
        out = np.zeros(self.n)
        out[: self.nx] = self.Jx.T @ y
        out[self.nx:] = -y[self.ind_ineq]
        return out

    # ------------------------------------------------------------------ initialize! (src/solver.jl:127-189)
    def initialize(self):
        opt = self.opt
        nx, n, m = self.nx, self.n, self.m
        # MadNLP.initialize!(cb, x, xl, xu, y, rhs, ind_ineq; tol, bound_push, bound_fac) [EXT]
        x = np.zeros(n)
        x[:nx] = self._x0
        xl = np.concatenate([self._lvar, self._lcon[self.ind_ineq]])
        xu = np.concatenate([self._uvar, self._ucon[self.ind_ineq]])
        x[self.ind_fixed] = xl[self.ind_fixed]              # MakeParameter
        y = self._y0.copy()
        rhs = np.where(self._lcon == self._ucon, self._lcon, 0.0)
        # bound relaxation (bound_relax_factor), not applied to fixed variables
        tol = opt.bound_relax_factor
        free = ~self._fixed_mask
        with np.errstate(invalid="ignore"):
            rl = xl - tol * np.maximum(1.0, np.abs(xl))
            ru = xu + tol * np.maximum(1.0, np.abs(xu))
        xl = np.where(free & np.isfinite(xl), rl, xl)
        xu = np.where(free & np.isfinite(xu), ru, xu)
        # initial slacks = constraint values, then push inside the bounds
        if self.ns:
            x[nx:] = (self._A @ x[:nx])[self.ind_ineq]
        x = _initialize_variables(x, xl, xu, opt.bound_push, opt.bound_fac, free)
        # set_scaling!(…, 100) (src/solver.jl:148-159) [EXT]
        self.obj_scale = 1.0
        self.con_scale = np.ones(m)
        if opt.scaling:
            g = self._Hsym @ x[:nx] + self.c_obj
            gmax = np.max(np.abs(g)) if nx else 0.0
            self.obj_scale = min(1.0, 100.0 / gmax) if gmax > 0 else 1.0
            rowmax = np.zeros(m)
            np.maximum.at(rowmax, self.Ar, np.abs(self.Av))
            with np.errstate(divide="ignore"):
                self.con_scale = np.minimum(1.0, 100.0 / rowmax)
            if self.ns:
                cs = self.con_scale[self.ind_ineq]
                xl[nx:] *= cs
                xu[nx:] *= cs
                x[nx:] *= cs
            rhs = rhs * self.con_scale
        self.rhs = rhs
        self.xl, self.xu = xl, xu
        self.x, self.y = x, y
        self.jacl = np.zeros(n)
        # scaled Jacobian values (compress_jacobian!, MakeParameter zeroes fixed columns) [EXT]
        jv = self.con_scale[self.Ar] * self.Av
        jv = np.where(self._fixed_mask[self.Ac], 0.0, jv)
        self.Jx = sp.coo_matrix((jv, (self.Ar, self.Ac)), shape=(m, nx)).tocsr()
        # scaled Hessian (lower), MakeParameter: rows/cols of fixed variables zeroed [EXT]
        hv = self.obj_scale * self.Hv
        fm = self._fixed_mask
        hv = np.where(fm[self.Hr] | fm[self.Hc], 0.0, hv)
        Hl = sp.coo_matrix((hv, (self.Hr, self.Hc)), shape=(n, n)).tocsr()
        self.Hlow = Hl
        self.Hfull = (Hl + Hl.T - sp.diags(Hl.diagonal())).tocsr()
        # MadNLP.initialize!(kkt) [EXT]: reg=1, pr_diag=1, du_diag=0, l/u_lower=0, l/u_diag=1
        self._k25_init = True
        self.reg = np.ones(n)
        self.pr_diag = np.ones(n)
        self.du_diag = np.zeros(m)
        self.l_diag = np.ones(self.nlb)
        self.u_diag = np.ones(self.nub)
        self.l_lower = np.zeros(self.nlb)
        self.u_lower = np.zeros(self.nub)
        # init_regularization! (src/kernels.jl:364-392)
        kind = opt.regularization[0]
        if kind == "none":
            self.del_w, self.del_c = 1.0, 0.0
        elif kind == "fixed":
            self.del_w, self.del_c = 1.0, opt.regularization[2]
        elif kind == "adaptive":
            self._adapt = [opt.regularization[1], opt.regularization[2], opt.regularization[3]]
            self.del_w, self.del_c = 1.0, opt.regularization[2]
        else:
            raise ValueError(kind)
        # callbacks (src/solver.jl:166-170)
        self.obj_val = self.eval_f(x)
        self.f = self.eval_grad(x)
        self.c = self.eval_cons(x)
        # normalization factors (src/solver.jl:173-174)
        self.norm_b = np.max(np.abs(self.rhs)) if m else 0.0
        self.norm_c = np.max(np.abs(self.f)) if n else 0.0
        self.zl = np.zeros(n)
        self.zu = np.zeros(n)
        self.k = 0
        self.alpha_p = 0.0
        self.alpha_d = 0.0
        self.init_starting_point()
        self.mu = opt.mu_init
        self.best_complementarity = INF
        self.status = REGULAR
        self.jacl = self.jtprod(self.y)

    # ------------------------------------------------------------------ KKT (K2, SparseKKTSystem [EXT])
    def kkt_matrix(self):
        """Lower COO of K2 in MadNLP order: pr_diag, hess, jac, slack(-1), du_diag [EXT],
        symmetrised for the SuperLU solve."""
        n, m, nx = self.n, self.m, self.nx
        rows = [np.arange(n), self.Hlow.tocoo().row, self.Jx.tocoo().row + n,
                n + self.ind_ineq, n + np.arange(m)]
        cols = [np.arange(n), self.Hlow.tocoo().col, self.Jx.tocoo().col,
                nx + np.arange(self.ns), n + np.arange(m)]
        vals = [self.pr_diag, self.Hlow.tocoo().data, self.Jx.tocoo().data,
                -np.ones(self.ns), self.du_diag]
        L = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                          shape=(n + m, n + m)).tocsr()
        return L

    def _aug_A(self):
        """A with slack columns (m x n): the Jacobian block of K2 / NormalKKTSystem.A
        (normalkkt.jl:70-80: slack -1 at (ind_ineq[k], nx + k))."""
        m, n, nx = self.m, self.n, self.nx
        J = self.Jx.tocoo()
        rows = np.concatenate([J.row, self.ind_ineq])
        cols = np.concatenate([J.col, nx + np.arange(self.ns)])
        vals = np.concatenate([J.data, -np.ones(self.ns)])
        return sp.coo_matrix((vals, (rows, cols)), shape=(m, n)).tocsr()

    def _k25_scaling(self):
        """K2.5 (MadNLP.ScaledSparseKKTSystem [EXT], set_aug_diagonal_reg! kernels.jl:139-149):
        s_i = sqrt((x - xl)(xu - x)) over the bounds present (a missing bound contributes 1)."""
        s2 = np.ones(self.n)
        s2[self.ind_lb] *= -self.l_diag          # x - xl  (l_diag = xl - x in the K2 convention)
        s2[self.ind_ub] *= -self.u_diag          # xu - x
        return np.sqrt(s2)

    def factorize_wrapper(self):
        """MadNLP.factorize_wrapper!: build_kkt! + factorize! timed into linear_solver_time [EXT]."""
        t0 = time.perf_counter()
        kind = self.opt.kkt_system
        if kind == "normal":
            # NormalKKTSystem.build_kkt! (normalkkt.jl:180-194): C = A Sigma^{-1} A^T, Sigma = pr_diag
            A = self._aug_A()
            K = (A @ sp.diags(1.0 / self.pr_diag) @ A.T).tocsc()
        else:
            L = self.kkt_matrix()
            K = (L + L.T - sp.diags(L.diagonal())).tocsc()
            if kind == "K25" and getattr(self, "_k25_init", False):
                # init_starting_point! sets pr_diag directly (solver.jl:14-16); the scaling factor
                # is still the one of MadNLP.initialize!(kkt) (= 1): K2.5 == K2 for this factorization
                self._k25_s = np.ones(self.n)
            elif kind == "K25":
                # S K2 S on the primal block; diagonal s^2 (reg + H_ii) + zl (xu - x) + zu (x - xl)
                s = self._k25_scaling()
                self._k25_s = s
                S = sp.diags(np.concatenate([s, np.ones(self.m)]))
                K = (S @ K @ S).tolil()
                dg = s * s * (self.reg + self.Hlow.diagonal())
                zl = np.zeros(self.n)
                zu = np.zeros(self.n)
                zl[self.ind_lb] = self.l_lower
                zu[self.ind_ub] = self.u_lower
                dist_l = np.ones(self.n)
                dist_u = np.ones(self.n)
                dist_l[self.ind_lb] = -self.l_diag
                dist_u[self.ind_ub] = -self.u_diag
                dg = dg + zl * dist_u + zu * dist_l
                K.setdiag(np.concatenate([dg, self.du_diag]))
                K = K.tocsc()
        ls = getattr(self, "linear_solver", "superlu")
        if not isinstance(ls, str):
            # a linear-solver PLUGIN (the reference's `linear_solver = LS` seam, src/structure.jl:79-123):
            # LS(aug_com) once per pattern (normalkkt.jl:113-115; the lower triangle in CSC), then
            # MadNLP.factorize!(ls) with the values (linear_solver.jl:10 via factorize_wrapper!),
            # MadIPM.is_factorized(ls) (utils.jl:54-62, linear_solver.jl:11) and, in kkt_solve,
            # MadNLP.solve!(ls, x) (linear_solver.jl:26).  Tests plug the HIP library in here to run the
            # reference-shaped loop around it (test/test_gpu.jl:9-19).
            Lw = sp.tril(K).tocsc()
            Lw.sort_indices()
            pat = getattr(self, "_plugin_pattern", None)
            if pat is None or not (np.array_equal(pat[0], Lw.indptr) and np.array_equal(pat[1], Lw.indices)):
                self._plugin = ls(Lw)
                self._plugin_pattern = (Lw.indptr.copy(), Lw.indices.copy())
            self._plugin.factorize(Lw.data)
            self._factorized = bool(self._plugin.is_factorized())
            self._lu = self._plugin
        elif ls == "pardiso":
            # CPU baseline (oracle/pardiso.py): MKL PARDISO, pattern analysed once per solver
            from .pardiso import PardisoLDL
            F = getattr(self, "_pardiso", None)
            if F is None or not F.same_pattern(K):
                F = self._pardiso = PardisoLDL(K, getattr(self, "ldl_perm", None))
            self._factorized = F.factorize(K)
            self._lu = F
        elif ls == "ldl":
            # oracle/ldl_ref.c: LDLFactorizations' up-looking LDL^T (static pivots) in the order
            # `ldl_perm` (default: SuperLU's minimum degree on A+A^T)
            from .ldl import OracleLDL
            if getattr(self, "ldl_perm", None) is None:
                self.ldl_perm = np.argsort(spla.splu(K, permc_spec="MMD_AT_PLUS_A").perm_c)
            F = OracleLDL(K, self.ldl_perm)
            self._factorized = F.factorize() == K.shape[0]
            # the HIP library's `pivot_tol` option (madipm_ldl_opts): a pivot with |d| <= tol (or a
            # non-finite one) also reports is_factorized == false; LDLFactorizations' own test is d == 0
            tol = getattr(self, "pivot_tol", 0.0)
            if self._factorized and tol > 0.0:
                dg = F.diag()
                self._factorized = bool(np.all(np.abs(dg) > tol) and np.all(np.isfinite(dg)))
            self._lu = F
        else:
            try:
                self._lu = spla.splu(K)
                self._factorized = True
            except RuntimeError:
                self._factorized = False
        self.linear_solver_time += time.perf_counter() - t0

    def kkt_solve(self, w):
        """MadNLP.solve!(kkt, w) [EXT]: reduce_rhs! → solve → finish_aug_solve!.
        K2 (SparseKKTSystem), K2.5 (scaled: solve S K S z = S r, d = S z) or the normal equations
        (normalkkt.jl:196-219)."""
        n, m, nlb = self.n, self.m, self.nlb
        xp = w[:n]
        wl = w[n + m: n + m + nlb]
        wu = w[n + m + nlb:]
        xp[self.ind_lb] -= wl / self.l_diag
        xp[self.ind_ub] -= wu / self.u_diag
        kind = self.opt.kkt_system
        if kind == "normal":
            A = self._aug_A()
            Sig = self.pr_diag
            wx, wy = w[:n], w[n:n + m]
            r1 = wx / Sig                       # Sigma^{-1} r1
            r2 = A @ r1 - wy                    # A Sigma^{-1} r1 - r2
            dy = self._lu.solve(r2)
            wy[:] = dy
            wx[:] = (wx - A.T @ dy) / Sig       # Sigma^{-1} (r1 - A^T dy)
        elif kind == "K25":
            s = self._k25_s
            w[:n] *= s
            w[: n + m] = self._lu.solve(w[: n + m])
            w[:n] *= s
        else:
            w[: n + m] = self._lu.solve(w[: n + m])
        xp = w[:n]
        wl[:] = (-wl + self.l_lower * xp[self.ind_lb]) / self.l_diag
        wu[:] = (wu - self.u_lower * xp[self.ind_ub]) / self.u_diag
        return w

    def kkt_mul(self, x, alpha=1.0, beta=0.0, w=None):
        """mul!(w, kkt::SparseKKTSystem, x, alpha, beta) + _kktmul! [EXT]."""
        n, m, nlb = self.n, self.m, self.nlb
        if w is None:
            w = np.zeros_like(x)
        xp, xy = x[:n], x[n:n + m]
        xl_, xu_ = x[n + m:n + m + nlb], x[n + m + nlb:]
        wp = beta * w[:n] + alpha * (self.Hfull @ xp)
        wp[: self.nx] += alpha * (self.Jx.T @ xy)
        wp[self.nx:] += alpha * (-xy[self.ind_ineq])
        wy = beta * w[n:n + m] + alpha * (self.Jx @ xp[: self.nx])
        wy[self.ind_ineq] -= alpha * xp[self.nx:]
        wp += alpha * self.reg * xp
        wy += alpha * self.du_diag * xy
        wp[self.ind_lb] -= alpha * xl_
        wp[self.ind_ub] += alpha * xu_
        wl = beta * w[n + m:n + m + nlb] + alpha * (xp[self.ind_lb] * self.l_lower - xl_ * self.l_diag)
        wu = beta * w[n + m + nlb:] + alpha * (xp[self.ind_ub] * self.u_lower + xu_ * self.u_diag)
        return np.concatenate([wp, wy, wl, wu])

    def solve_system(self, p):
        """solve_system! src/linear_solver.jl:19-44 (copy, solve, residual check)."""
        if not getattr(self, "_factorized", True):
            # every trial of factorize_regularized_system! failed: LDLFactorizations' ldiv! refuses an
            # unfactorized object [EXT]
            raise UnfactorizedSolveException("solve with an unfactorized KKT system")
        d = self.kkt_solve(p.copy())
        w = self.kkt_mul(d, -1.0, 1.0, p.copy())
        norm_w = np.max(np.abs(w)) if len(w) else 0.0
        norm_p = np.max(np.abs(p)) if len(p) else 0.0
        ratio = norm_w / max(1.0, norm_p)
        self.last_residual = ratio
        self.residuals.append(ratio)
        if math.isnan(ratio) or (self.opt.check_residual and ratio > self.opt.tol_linear_solve):
            raise SolveException("residual check of solve_system!")
        return d

    # ---------------------------------------------------------------- views
    def _split(self, v):
        n, m, nlb = self.n, self.m, self.nlb
        return v[:n], v[n:n + m], v[n + m:n + m + nlb], v[n + m + nlb:]

    # ------------------------------------------------------------------ init_starting_point! (src/solver.jl:6-125)
    def init_starting_point(self):
        n, m = self.n, self.m
        ind_lb, ind_ub = self.ind_lb, self.ind_ub
        L = len(self.x) + m + self.nlb + self.nub
        # lines 16-18
        self.reg[:] = self.del_w
        self.pr_diag[:] = self.del_w
        self.du_diag[:] = self.del_c
        self.factorize_wrapper()                                     # line 21
        # Step 1 (lines 25-28): set_initial_primal_rhs! kernels.jl:1-9
        p = np.zeros(L)
        p[n:n + m] = -self.c
        d = self.solve_system(p)
        self.x += d[:n]
        # Step 2 (lines 31-33): set_initial_dual_rhs! kernels.jl:11-19
        p = np.zeros(L)
        p[:n] = -self.f
        d = self.solve_system(p)
        self.y = d[n:n + m].copy()
        # Step 3 (lines 37-66)
        res = self.jtprod(self.y) + self.f
        l, u = self.xl, self.xu
        fl, fu = np.isfinite(l), np.isfinite(u)
        self.zl = np.where(fl & fu, 0.5 * res, np.where(fl, res, self.zl))
        self.zu = np.where(fl & fu, -0.5 * res, np.where(fu, -res, self.zu))
        x = self.x
        xl_v, lb = x[ind_lb], self.xl[ind_lb]
        xu_v, ub = x[ind_ub], self.xu[ind_ub]
        zl, zu = self.zl[ind_lb], self.zu[ind_ub]
        # lines 68-78
        delta_x = max(0.0, -1.5 * min(np.min(xl_v - lb, initial=0.0), 0.0),
                      -1.5 * min(np.min(ub - xu_v, initial=0.0), 0.0))
        delta_s = max(0.0, -1.5 * min(np.min(zl, initial=0.0), 0.0),
                      -1.5 * min(np.min(zu, initial=0.0), 0.0))
        # lines 80-83 (x_lr / x_ur are views of the same x: doubly bounded entries net zero)
        x[ind_lb] = x[ind_lb] + delta_x
        x[ind_ub] = x[ind_ub] - delta_x
        zl = zl + 1.0 + delta_s
        zu = zu + 1.0 + delta_s
        xl_v, xu_v = x[ind_lb], x[ind_ub]
        # lines 85-99
        mu = 0.0
        if len(zl):
            mu += xl_v @ zl - lb @ zl
        if len(zu):
            mu += ub @ zu - xu_v @ zu
        delta_x2 = mu / (2 * (np.sum(zl) + np.sum(zu)))
        delta_s2 = mu / (2 * (np.sum(xl_v - lb) + np.sum(ub - xu_v)))
        x[ind_lb] = x[ind_lb] + delta_x2
        x[ind_ub] = x[ind_ub] - delta_x2
        zl = zl + delta_s2
        zu = zu + delta_s2
        self.zl[ind_lb] = zl
        self.zu[ind_ub] = zu
        # lines 102-118: Ipopt projection
        kappa = self.opt.bound_fac
        with np.errstate(invalid="ignore"):
            pl = np.minimum(kappa * np.maximum(1.0, l), kappa * (u - l))
            pu = np.minimum(kappa * np.maximum(1.0, u), kappa * (u - l))
        with np.errstate(invalid="ignore"):
            x[:] = np.where(x < l, l + pl, np.where(u < x, u - pu, x))
        # lines 120-123
        if not (np.all(self.zl[ind_lb] > 0) and np.all(self.zu[ind_ub] > 0)
                and np.all(x[ind_lb] > self.xl[ind_lb]) and np.all(x[ind_ub] < self.xu[ind_ub])):
            raise AssertionError("init_starting_point!: interior assertion failed")

    # ------------------------------------------------------------------ kernels.jl
    def set_aug_diagonal_reg(self):
        """kernels.jl:124-136 (K2); the K2.5 diagonal (kernels.jl:139-149) is formed from these in
        factorize_wrapper."""
        self._k25_init = False
        x = self.x
        self.reg[:] = self.del_w
        self.du_diag[:] = self.del_c
        self.l_diag = self.xl[self.ind_lb] - x[self.ind_lb]
        self.u_diag = x[self.ind_ub] - self.xu[self.ind_ub]
        self.l_lower = self.zl[self.ind_lb].copy()
        self.u_lower = self.zu[self.ind_ub].copy()
        pr = self.reg.copy()
        pr[self.ind_lb] -= self.l_lower / self.l_diag
        pr[self.ind_ub] -= self.u_lower / self.u_diag
        self.pr_diag = pr

    def _rhs_common(self):
        n, m = self.n, self.m
        p = np.zeros(n + m + self.nlb + self.nub)
        p[:n] = -self.f + self.zl - self.zu - self.jacl
        p[n:n + m] = -self.c
        return p

    def set_predictive_rhs(self):
        """kernels.jl:21-41."""
        n, m, nlb = self.n, self.m, self.nlb
        p = self._rhs_common()
        x = self.x
        p[n + m:n + m + nlb] = (self.xl[self.ind_lb] - x[self.ind_lb]) * self.zl[self.ind_lb]
        p[n + m + nlb:] = (self.xu[self.ind_ub] - x[self.ind_ub]) * self.zu[self.ind_ub]
        return p

    def set_correction_rhs(self, mu, corr_lb, corr_ub):
        """kernels.jl:43-58."""
        n, m, nlb = self.n, self.m, self.nlb
        p = self._rhs_common()
        x = self.x
        p[n + m:n + m + nlb] = (self.xl[self.ind_lb] - x[self.ind_lb]) * self.zl[self.ind_lb] + mu - corr_lb
        p[n + m + nlb:] = (self.xu[self.ind_ub] - x[self.ind_ub]) * self.zu[self.ind_ub] - mu - corr_ub
        return p

    def get_correction(self, d):
        """kernels.jl:60-71."""
        dx, _, dzl, dzu = self._split(d)
        return dx[self.ind_lb] * dzl, dx[self.ind_ub] * dzu

    def set_extra_correction(self, d, corr_lb, corr_ub, alpha_p, alpha_d, bmin, bmax, mu):
        """kernels.jl:74-122 (Gondzio)."""
        dx, _, dzl, dzu = self._split(d)
        tmin, tmax = bmin * mu, bmax * mu
        x = self.x
        xx = x[self.ind_lb] + alpha_p * dx[self.ind_lb] - self.xl[self.ind_lb]
        zz = self.zl[self.ind_lb] + alpha_d * dzl
        v = xx * zz
        delta = np.where(v < tmin, tmin - v, np.where(v > tmax, tmax - v, 0.0))
        corr_lb = corr_lb - delta
        xx = self.xu[self.ind_ub] - alpha_p * dx[self.ind_ub] - x[self.ind_ub]
        zz = self.zu[self.ind_ub] + alpha_d * dzu
        v = xx * zz
        delta = np.where(v < tmin, tmin - v, np.where(v > tmax, tmax - v, 0.0))
        corr_ub = corr_ub + delta
        return corr_lb, corr_ub

    def complementarity_measure(self):
        """kernels.jl:155-174."""
        m1, m2 = self.nlb, self.nub
        if m1 + m2 == 0:
            return 0.0
        x = self.x
        cl = np.sum((x[self.ind_lb] - self.xl[self.ind_lb]) * self.zl[self.ind_lb])
        cu = np.sum((self.xu[self.ind_ub] - x[self.ind_ub]) * self.zu[self.ind_ub])
        return (cl + cu) / (m1 + m2)

    def affine_complementarity_measure(self, d, alpha_p, alpha_d):
        """kernels.jl:176-208."""
        m1, m2 = self.nlb, self.nub
        if m1 + m2 == 0:
            return 0.0
        dx, _, dzl, dzu = self._split(d)
        x = self.x
        cl = np.sum(((x[self.ind_lb] + alpha_p * dx[self.ind_lb]) - self.xl[self.ind_lb])
                    * (self.zl[self.ind_lb] + alpha_d * dzl))
        cu = np.sum((self.xu[self.ind_ub] - (x[self.ind_ub] + alpha_p * dx[self.ind_ub]))
                    * (self.zu[self.ind_ub] + alpha_d * dzu))
        return (cl + cu) / (m1 + m2)

    def update_barrier(self, mu_affine):
        """kernels.jl:210-220 (Mehrotra)."""
        mu_curr = self.complementarity_measure()
        if self.has_inequalities:
            sigma = min(max((mu_affine / mu_curr) ** 3, 1e-6), 10.0)
        else:
            sigma = 1.0
        self.mu = max(self.opt.mu_min, sigma * mu_curr)
        return mu_curr

    @staticmethod
    def _argmin_ratio(num, den, mask):
        """mapreduce((val, i), (e1, e2) -> e1[1] < e2[1] ? e1 : e2; init=(1.0, 0)) of kernels.jl:226-272,
        a LEFT fold: a later element replaces the accumulator unless the accumulator is strictly
        smaller, so among equal ratios the last index wins, and an element whose ratio is exactly
        1.0 replaces the init element.  Returns (alpha, index or -1 for the init element)."""
        if not np.any(mask):
            return 1.0, -1
        with np.errstate(divide="ignore", invalid="ignore"):
            vals = np.where(mask, num / den, INF)
        i = len(vals) - 1 - int(np.argmin(vals[::-1]))   # last occurrence of the minimum
        if vals[i] <= 1.0:
            return float(vals[i]), i
        return 1.0, -1

    def alpha_max_primal(self, d, tau):
        """get_alpha_max_primal kernels.jl:226-248."""
        dx = d[: self.n]
        x = self.x
        dxl, dxu = dx[self.ind_lb], dx[self.ind_ub]
        a_l, i_l = self._argmin_ratio((-x[self.ind_lb] + self.xl[self.ind_lb]) * tau, dxl, dxl < 0)
        a_u, i_u = self._argmin_ratio((-x[self.ind_ub] + self.xu[self.ind_ub]) * tau, dxu, dxu > 0)
        return a_l, a_u, i_l, i_u

    def alpha_max_dual(self, d, tau):
        """get_alpha_max_dual kernels.jl:250-272 (note the extra zu+dzu<0 test, l.263)."""
        _, _, dzl, dzu = self._split(d)
        zl, zu = self.zl[self.ind_lb], self.zu[self.ind_ub]
        a_l, i_l = self._argmin_ratio(-zl * tau, dzl, dzl < 0)
        a_u, i_u = self._argmin_ratio(-zu * tau, dzu, (dzu < 0) & (zu + dzu < 0))
        return a_l, a_u, i_l, i_u

    def fraction_to_boundary(self, d, tau):
        """get_fraction_to_boundary_step kernels.jl:274-289."""
        a_xl, a_xu, _, _ = self.alpha_max_primal(d, tau)
        a_zl, a_zu, _, _ = self.alpha_max_dual(d, tau)
        return min(a_xl, a_xu), min(a_zl, a_zu)

    def update_step(self, d):
        """update_step! kernels.jl:291-358 (on the bounded-coordinate views, step_on_vectors)."""
        dx, _, dzl, dzu = self._split(d)
        x = self.x
        r = step_on_vectors(self.opt.step_rule, self.mu, x[self.ind_lb], self.xl[self.ind_lb], self.zl[self.ind_lb],
                            dx[self.ind_lb], dzl, x[self.ind_ub], self.xu[self.ind_ub], self.zu[self.ind_ub],
                            dx[self.ind_ub], dzu)
        self.alpha_p, self.alpha_d = r["alpha_p"], r["alpha_d"]

    def update_regularization(self):
        """kernels.jl:370-401."""
        kind = self.opt.regularization[0]
        if kind == "none":
            self.del_w, self.del_c = 0.0, 0.0
        elif kind == "fixed":
            self.del_w, self.del_c = self.opt.regularization[1], self.opt.regularization[2]
        else:
            dp, dd, dmin = self._adapt
            dp = max(dp / 10.0, dmin)
            dd = min(dd / 10.0, -dmin)
            self._adapt = [dp, dd, dmin]
            self.del_w, self.del_c = dp, dd

    def factorize_regularized_system(self):
        """linear_solver.jl:6-17."""
        for _ in range(3):
            self.set_aug_diagonal_reg()
            self.factorize_wrapper()
            if self._factorized:
                break
            self.del_w *= 100.0
            self.del_c *= 100.0

    def dual_objective(self):
        """kernels.jl:408-417."""
        dobj = -(self.y @ self.rhs)
        if self.nlb:
            dobj += self.zl[self.ind_lb] @ self.xl[self.ind_lb]
        if self.nub:
            dobj -= self.zu[self.ind_ub] @ self.xu[self.ind_ub]
        return dobj

    def optimality_gap(self):
        """kernels.jl:419-430 → MadNLP.get_inf_compl(…, 0., 1.0) [EXT]."""
        x = self.x
        g = 0.0
        if self.nlb:
            g = max(g, np.max(np.abs((x[self.ind_lb] - self.xl[self.ind_lb]) * self.zl[self.ind_lb])))
        if self.nub:
            g = max(g, np.max(np.abs((self.xu[self.ind_ub] - x[self.ind_ub]) * self.zu[self.ind_ub])))
        return g

    def update_termination_criteria(self):
        """src/solver.jl:194-222."""
        dobj = self.dual_objective()
        self.inf_pr = (np.max(np.abs(self.c)) if self.m else 0.0) / max(1.0, self.norm_b)
        r = self.f - self.zl + self.zu + self.jacl
        self.inf_du = (np.max(np.abs(r)) if self.n else 0.0) / max(1.0, self.norm_c)
        self.inf_compl = self.optimality_gap() / max(1.0, self.norm_c)
        self.best_complementarity = min(self.best_complementarity, self.inf_compl)
        opt = self.opt
        if max(self.inf_pr, self.inf_du, self.inf_compl) <= opt.tol:
            self.status = SOLVE_SUCCEEDED
        elif (self.inf_compl > opt.divergence_tol * self.best_complementarity) and \
                (dobj > max(10.0 * abs(self.obj_val), 1.0)):
            self.status = INFEASIBLE_PROBLEM_DETECTED
        elif self.obj_val < -opt.divergence_tol * max(10.0, abs(dobj), 1.0):
            self.status = DIVERGING_ITERATES
        elif self.k >= opt.max_iter:
            self.status = MAXIMUM_ITERATIONS_EXCEEDED
        elif time.perf_counter() - self._start >= opt.max_wall_time:
            self.status = MAXIMUM_WALLTIME_EXCEEDED

    def adjust_boundary(self):
        """MadNLP.adjust_boundary! [EXT] (called at src/solver.jl:313)."""
        c1 = np.finfo(float).eps * self.mu
        c2 = np.finfo(float).eps ** 0.75
        x = self.x
        xl_r = self.xl[self.ind_lb]
        xlr = x[self.ind_lb]
        self.xl[self.ind_lb] = np.where(xlr - xl_r < c1, xl_r - c2 * np.maximum(1.0, np.abs(xlr)), xl_r)
        xu_r = self.xu[self.ind_ub]
        xur = x[self.ind_ub]
        self.xu[self.ind_ub] = np.where(xu_r - xur < c1, xu_r + c2 * np.maximum(1.0, np.abs(xur)), xu_r)

    def apply_step(self, d):
        """src/solver.jl:308-317."""
        dx, dy, dzl, dzu = self._split(d)
        self.x = self.x + self.alpha_p * dx
        self.y = self.y + self.alpha_d * dy
        self.zl[self.ind_lb] += self.alpha_d * dzl
        self.zu[self.ind_ub] += self.alpha_d * dzu
        self.adjust_boundary()
        self.k += 1

    def evaluate_model(self):
        """src/solver.jl:319-326."""
        self.obj_val = self.eval_f(self.x)
        self.c = self.eval_cons(self.x)
        self.f = self.eval_grad(self.x)
        self.jacl = self.jtprod(self.y)

    def gondzio(self, d):
        """src/solver.jl:245-298."""
        if self.opt.max_ncorr <= 0:
            return d
        delta, bmin, bmax, tau = 0.1, 0.1, 10.0, 0.995
        alpha_p, alpha_d = self.fraction_to_boundary(d, tau)
        for _ in range(self.opt.max_ncorr):
            tap = min(alpha_p + delta, 1.0)
            tad = min(alpha_d + delta, 1.0)
            ga = self.affine_complementarity_measure(d, tap, tad)
            g = self.mu_curr
            mu = (ga / g) ** 2 * ga
            self.corr_lb, self.corr_ub = self.set_extra_correction(
                d, self.corr_lb, self.corr_ub, tap, tad, bmin, bmax, mu)
            p = self.set_correction_rhs(mu, self.corr_lb, self.corr_ub)
            dprev = d
            d = self.solve_system(p)
            hap, had = self.fraction_to_boundary(d, tau)
            if hap < 1.005 * alpha_p or had < 1.005 * alpha_d:
                d = dprev
                break
            alpha_p, alpha_d = hap, had
        return d

    def _record(self):
        if self.record_trace:
            self.trace.append(dict(k=self.k, obj=self.obj_val / self.obj_scale, inf_pr=self.inf_pr,
                                   inf_du=self.inf_du, inf_compl=self.inf_compl, mu=self.mu,
                                   alpha_p=self.alpha_p, alpha_d=self.alpha_d, del_w=self.del_w))

    def mpc(self):
        """mpc! src/solver.jl:332-360."""
        while True:
            self.update_termination_criteria()
            self._record()
            if self.status != REGULAR:
                return
            self.update_regularization()                 # factorize_system! solver.jl:299-303
            self.factorize_regularized_system()
            # prediction_step! solver.jl:230-237
            d = self.solve_system(self.set_predictive_rhs())
            ap, ad = self.fraction_to_boundary(d, 1.0)
            mu_aff = self.affine_complementarity_measure(d, ap, ad)
            self.corr_lb, self.corr_ub = self.get_correction(d)
            self.mu_curr = self.update_barrier(mu_aff)
            # mehrotra_correction_direction! solver.jl:239-243
            d = self.solve_system(self.set_correction_rhs(self.mu, self.corr_lb, self.corr_ub))
            d = self.gondzio(d)
            self.update_step(d)
            self.apply_step(d)
            self.evaluate_model()

    def solve(self) -> OracleStats:
        """solve! src/solver.jl:362-418 (exceptions → status)."""
        t0 = time.perf_counter()
        self._start = t0
        self.exception = EXC_NONE
        try:
            self.initialize()
            self._start = time.perf_counter()      # src/solver.jl:181
            self.mpc()
        except (SolveException, UnfactorizedSolveException) as e:
            # neither is a MadNLP.LinearSolverException: the catch-all (src/solver.jl:398-403)
            self.status = INTERNAL_ERROR
            self.exception = EXC_SOLVE if isinstance(e, SolveException) else EXC_UNFACTORIZED
            if self.opt.rethrow_error:
                raise
        total = time.perf_counter() - self._start
        return self.stats(total)

    def stats(self, total_time=0.0) -> OracleStats:
        """update_solution! src/utils.jl:150-156 + MadNLP.update! [EXT]."""
        obj = self.obj_val / self.obj_scale
        if not self.minimize:
            obj = -obj
        xv = self.x[: self.nx].copy()
        cons = self._A @ xv
        return OracleStats(status=self.status, iter=self.k, objective=obj, solution=xv,
                           constraints=cons,
                           multipliers=self.y * self.con_scale / self.obj_scale,
                           multipliers_L=self.zl[: self.nx] / self.obj_scale,
                           multipliers_U=self.zu[: self.nx] / self.obj_scale,
                           total_time=total_time, linear_solver_time=self.linear_solver_time,
                           trace=list(self.trace), exception=getattr(self, "exception", EXC_NONE))


def step_on_vectors(rule, mu, x_lr, xl_r, zl_r, dx_lr, dzl, x_ur, xu_r, zu_r, dx_ur, dzu) -> dict:
    """update_step!(rule, solver) (kernels.jl:291-358) with get_alpha_max_primal / _dual
    (kernels.jl:226-272) on the bounded-coordinate views.  rule: ("conservative", tau) |
    ("adaptive", tau_min) | ("mehrotra", gamma_f).  Indices 0-based, -1 = the init element."""
    am = OracleMPC._argmin_ratio

    def primal(tau):
        a_l, i_l = am((-x_lr + xl_r) * tau, dx_lr, dx_lr < 0)
        a_u, i_u = am((-x_ur + xu_r) * tau, dx_ur, dx_ur > 0)
        return a_l, a_u, i_l, i_u

    def dual(tau):
        a_l, i_l = am(-zl_r * tau, dzl, dzl < 0)
        a_u, i_u = am(-zu_r * tau, dzu, (dzu < 0) & (zu_r + dzu < 0))   # kernels.jl:263
        return a_l, a_u, i_l, i_u

    kind, par = rule[0], rule[1]
    if kind in ("conservative", "adaptive"):
        tau = par if kind == "conservative" else max(1 - mu, par)
        a_xl, a_xu, i_xl, i_xu = primal(tau)
        a_zl, a_zu, i_zl, i_zu = dual(tau)
        ap, ad = min(a_xl, a_xu), min(a_zl, a_zu)
    elif kind == "mehrotra":
        gamma_f = par
        gamma_a = 1.0 / (1.0 - gamma_f)
        a_xl, a_xu, i_xl, i_xu = primal(1.0)
        a_zl, a_zu, i_zl, i_zu = dual(1.0)
        max_p, max_d = min(a_xl, a_xu), min(a_zl, a_zu)
        cnt = len(x_lr) + len(x_ur)
        mu_full = 0.0
        if cnt:   # get_affine_complementarity_measure (kernels.jl:176-208)
            mu_full = (np.sum(((x_lr + max_p * dx_lr) - xl_r) * (zl_r + max_d * dzl))
                       + np.sum((xu_r - (x_ur + max_p * dx_ur)) * (zu_r + max_d * dzu))) / cnt
        mu_full /= gamma_a
        ap, ad = 1.0, 1.0
        if max_p < 1.0:
            if a_xl <= a_xu:
                i = i_xl
                tmp = mu_full / (zl_r[i] + max_d * dzl[i])
                ap = (x_lr[i] - xl_r[i] - tmp) / (-dx_lr[i])
            else:
                i = i_xu
                tmp = mu_full / (zu_r[i] + max_d * dzu[i])
                ap = (xu_r[i] - x_ur[i] - tmp) / dx_ur[i]
        if max_d < 1.0:
            if a_zl <= a_zu:
                i = i_zl
                tmp = mu_full / (x_lr[i] + max_p * dx_lr[i] - xl_r[i])
                ad = -(zl_r[i] - tmp) / dzl[i]
            else:
                i = i_zu
                tmp = mu_full / (xu_r[i] - x_ur[i] - max_p * dx_ur[i])
                ad = -(zu_r[i] - tmp) / dzu[i]
        ap, ad = max(ap, gamma_f * max_p), max(ad, gamma_f * max_d)
    else:
        raise ValueError(rule)
    return dict(alpha_p=float(ap), alpha_d=float(ad), alpha_xl=a_xl, alpha_xu=a_xu, alpha_zl=a_zl, alpha_zu=a_zu,
                i_xl=i_xl, i_xu=i_xu, i_zl=i_zl, i_zu=i_zu)


def _initialize_variables(x, xl, xu, bound_push, bound_fac, free):
    """MadNLP.initialize_variables! (Ipopt bound push) [EXT]."""
    x = x.copy()
    with np.errstate(invalid="ignore"):
        span = xu - xl
        pl = np.where(np.isfinite(xu), np.minimum(bound_push * np.maximum(1.0, np.abs(xl)), bound_fac * span),
                      bound_push * np.maximum(1.0, np.abs(xl)))
        pu = np.where(np.isfinite(xl), np.minimum(bound_push * np.maximum(1.0, np.abs(xu)), bound_fac * span),
                      bound_push * np.maximum(1.0, np.abs(xu)))
        lo = np.where(np.isfinite(xl), xl + pl, -INF)
        hi = np.where(np.isfinite(xu), xu - pu, INF)
    xn = np.minimum(np.maximum(x, lo), hi)
    return np.where(free, xn, x)


def madipm(qp, **kw) -> OracleStats:
    """madipm(m; kwargs...) src/solver.jl:425-428."""
    opt = OracleOptions(**kw)
    return OracleMPC(qp, opt).solve()
