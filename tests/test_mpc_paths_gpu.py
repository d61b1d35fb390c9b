"""GPU tests of the MPC loop's exceptional paths, each against the oracle on the same problem.

* regularization retry: factorize_regularized_system! (src/linear_solver.jl:6-17) multiplies
  (del_w, del_c) by 100 after each failed trial, up to 3 trials.  Forced here with a free LP column
  (Sigma_j = 0, H = 0): its pivot is exactly del_w when it is eliminated before its row, and the
  library's `pivot_tol` option (mirrored by the oracle) rejects del_w = 1e-12 and 1e-10, accepts 1e-8.
  With max_ncorr = 0 this also runs the recomputation of the speculatively enqueued directions.
* every trial failing (del_w = 0): the solve would use an unfactorized LDL^T, which the linear solver
  refuses with an exception that is no MadNLP.LinearSolverException -> solve!'s catch-all:
  INTERNAL_ERROR (solver.jl:398-403), the iterate untouched and the iteration not counted
  (cnt.k += 1 is in apply_step!, solver.jl:316); rethrown with rethrow_error = true.
* check_residual with an impossible tol_linear_solve -> `throw(MadNLP.SolveException)`
  (linear_solver.jl:40-41) throws the TYPE, which is not `isa LinearSolverException` -> INTERNAL_ERROR
  (solver.jl:398-403), rethrown with rethrow_error = true (scripts/benchmarks_cpu.jl:39 sets it).
* INFEASIBLE_PROBLEM_DETECTED / DIVERGING_ITERATES (solver.jl:209-213).
* maximization: the objective sign flip of update_solution! (src/utils.jl:150-156).
Tolerances as tests/test_mpc_gpu.py: status and iteration count equal, objective 1e-6 relative.
"""
import numpy as np
import pytest

from oracle.mpc import OracleMPC, OracleOptions

pytestmark = pytest.mark.gpu

INF = np.inf


def _qp(**kw):
    from madipm_amd.qp import QuadraticModel
    base = dict(Hrows=[], Hcols=[], Hvals=[])
    base.update(kw)
    return QuadraticModel(**base)


def _free_column_lp():
    # min x0 + x1  s.t.  x0 + x1 = 1,  x0 - x1 + x2 = 0,  x0, x1 >= 0, x2 free
    return _qp(c=np.array([1.0, 1.0, 0.0]), Arows=[0, 0, 1, 1, 1], Acols=[0, 1, 0, 1, 2],
               Avals=[1.0, 1.0, 1.0, -1.0, 1.0], lcon=[1.0, 0.0], ucon=[1.0, 0.0],
               lvar=[0.0, 0.0, -INF], uvar=[INF, INF, INF], name="free_column")


def _run_pair(qp, reg, pivot_tol=0.0, max_ncorr=0, **extra):
    """GPU solve (AMD order) and the oracle with the oracle LDL^T in the GPU's pivot order."""
    from madipm_amd import MPCSolver, FixedRegularization
    s = MPCSolver(qp, regularization=FixedRegularization(*reg), ordering=1, pivot_tol=pivot_tol,
                  max_ncorr=max_ncorr, max_iter=100, **extra)
    gpu = s.solve()
    o = OracleMPC(qp, OracleOptions(regularization=("fixed",) + tuple(reg), max_ncorr=max_ncorr, max_iter=100,
                                    **{k: v for k, v in extra.items() if k in ("check_residual", "tol_linear_solve")}))
    o.linear_solver = "ldl"
    o.ldl_perm = s.kkt_perm()
    o.pivot_tol = pivot_tol
    ref = o.solve()
    return gpu, ref


@pytest.mark.parametrize("max_ncorr", [0, 2])
def test_regularization_retry_matches_oracle(max_ncorr):
    from madipm_amd import SOLVE_SUCCEEDED
    gpu, ref = _run_pair(_free_column_lp(), (1e-12, -1e-8), pivot_tol=1e-9, max_ncorr=max_ncorr)
    assert gpu.status == ref.status == SOLVE_SUCCEEDED, (gpu.status_name, ref.status)
    assert gpu.iter == ref.iter
    assert abs(gpu.objective - 1.0) <= 1e-6 and abs(ref.objective - 1.0) <= 1e-6
    # the printed regularization of iteration k >= 1 is the accepted trial of iteration k-1: 1e-12 * 100^2
    dw_g = [t["del_w"] for t in gpu.trace]
    dw_r = [t["del_w"] for t in ref.trace]
    assert dw_g == dw_r, (dw_g, dw_r)
    assert all(abs(d - 1e-8) <= 1e-20 for d in dw_g[1:]) and len(dw_g) > 1
    for tg, tr in zip(gpu.trace[:3], ref.trace[:3]):
        for key in ("obj", "inf_pr", "inf_du", "mu"):
            assert abs(tg[key] - tr[key]) <= 1e-6 * abs(tr[key]) + 1e-12, (tg["k"], key, tg[key], tr[key])


def test_all_trials_fail_is_internal_error():
    from madipm_amd import INTERNAL_ERROR
    from madipm_amd.solver import EXC_UNFACTORIZED
    qp = _free_column_lp()
    gpu, ref = _run_pair(qp, (0.0, -1e-8))
    assert gpu.status == ref.status == INTERNAL_ERROR, (gpu.status_name, ref.status)
    assert ref.exception == EXC_UNFACTORIZED
    assert gpu.iter == ref.iter == 0
    assert len(gpu.trace) == len(ref.trace) == 1
    # the iterate is the one after initialize!: no step was applied
    assert np.allclose(gpu.solution, ref.solution, rtol=1e-9, atol=1e-12), (gpu.solution, ref.solution)
    # rethrow_error = true: solve! rethrows (src/solver.jl:402)
    from madipm_amd import MPCSolver, FixedRegularization, UnfactorizedSolveException
    import oracle.mpc as om
    with pytest.raises(UnfactorizedSolveException):
        MPCSolver(qp, regularization=FixedRegularization(0.0, -1e-8), ordering=1, max_iter=100,
                  rethrow_error=True).solve()
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 0.0, -1e-8), max_iter=100, rethrow_error=True))
    o.linear_solver = "ldl"
    o.ldl_perm = MPCSolver(qp, ordering=1).kkt_perm()
    with pytest.raises(om.UnfactorizedSolveException):
        o.solve()


def test_check_residual_impossible_tol():
    from madipm_amd import INTERNAL_ERROR, MPCSolver, FixedRegularization, SolveException
    from madipm_amd import read_mps, standard_form_qp
    from madipm_amd.solver import EXC_SOLVE
    import os
    qp = standard_form_qp(read_mps(os.path.join(os.path.dirname(__file__), "golden", "afiro.mps")))
    gpu = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), check_residual=True,
                    tol_linear_solve=1e-300).solve()
    ref = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), check_residual=True,
                                      tol_linear_solve=1e-300)).solve()
    assert gpu.status == ref.status == INTERNAL_ERROR
    assert ref.exception == EXC_SOLVE
    assert gpu.iter == ref.iter == 0
    with pytest.raises(SolveException):
        MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), check_residual=True,
                  tol_linear_solve=1e-300, rethrow_error=True).solve()
    # a loose tolerance never triggers: same answer as without the check
    ok = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), check_residual=True,
                   tol_linear_solve=1e-6).solve()
    assert ok.status_name == "SOLVE_SUCCEEDED" and abs(ok.objective + 464.75314286) <= 1e-6 * 464.75


def _random_infeasible(seed, m=40, n=60):
    """Random feasible LP plus one row that contradicts a nonnegative combination of two others."""
    rng = np.random.default_rng(seed)
    A = (rng.random((m, n)) < 0.15) * rng.uniform(0.5, 2.0, (m, n))
    A[:, rng.integers(0, n, m)] += 1.0
    x0 = rng.uniform(0.5, 1.5, n)
    b = A @ x0
    # row m: a_0 + a_1, rhs far below what x >= 0 allows for the sum of rows 0 and 1
    A = np.vstack([A, A[0] + A[1]])
    b = np.concatenate([b, [-(b[0] + b[1]) - 5.0]])
    r, c = np.nonzero(A)
    return _qp(c=rng.uniform(0.1, 1.0, n), Arows=r, Acols=c, Avals=A[r, c], lcon=b, ucon=b,
               lvar=np.zeros(n), uvar=np.full(n, INF), name=f"infeasible{seed}")


@pytest.mark.parametrize("which", ["tiny", "random0", "random1"])
def test_infeasible_detected(which):
    from madipm_amd import INFEASIBLE_PROBLEM_DETECTED, MPCSolver, FixedRegularization
    if which == "tiny":  # x1 + x2 <= -1, x >= 0
        qp = _qp(c=np.ones(2), Arows=[0, 0], Acols=[0, 1], Avals=[1.0, 1.0], lcon=[-INF], ucon=[-1.0],
                 lvar=[0.0, 0.0], uvar=[INF, INF], name="infeasible_tiny")
    else:
        qp = _random_infeasible(int(which[-1]))
    gpu = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8), max_iter=200).solve()
    ref = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=200)).solve()
    assert ref.status == INFEASIBLE_PROBLEM_DETECTED
    assert gpu.status == ref.status, (gpu.status_name, ref.status)
    assert abs(gpu.iter - ref.iter) <= 1, (gpu.iter, ref.iter)


def test_unbounded_diverges():
    from madipm_amd import DIVERGING_ITERATES, MPCSolver, FixedRegularization
    # min -x0  s.t.  x0 - x1 = 0, x >= 0
    qp = _qp(c=np.array([-1.0, 0.0]), Arows=[0, 0], Acols=[0, 1], Avals=[1.0, -1.0], lcon=[0.0], ucon=[0.0],
             lvar=[0.0, 0.0], uvar=[INF, INF], name="unbounded")
    gpu = MPCSolver(qp, regularization=FixedRegularization(1e-8, -1e-8)).solve()
    ref = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8))).solve()
    assert gpu.status == ref.status == DIVERGING_ITERATES, (gpu.status_name, ref.status)
    assert gpu.iter == ref.iter


def test_maximize_sign_flip():
    from madipm_amd import MPCSolver, FixedRegularization, SOLVE_SUCCEEDED
    # max x0 + x1  s.t.  x0 + 2 x1 <= 1, x >= 0  -> optimum 1 at (1, 0)
    kw = dict(c=np.ones(2), Arows=[0, 0], Acols=[0, 1], Avals=[1.0, 2.0], lcon=[-INF], ucon=[1.0],
              lvar=[0.0, 0.0], uvar=[INF, INF])
    qmax = _qp(minimize=False, name="max", **kw)
    gpu = MPCSolver(qmax, regularization=FixedRegularization(1e-8, -1e-8)).solve()
    ref = OracleMPC(qmax, OracleOptions(regularization=("fixed", 1e-8, -1e-8))).solve()
    assert gpu.status == ref.status == SOLVE_SUCCEEDED
    assert gpu.iter == ref.iter
    assert abs(gpu.objective - 1.0) <= 1e-7 and abs(gpu.objective - ref.objective) <= 1e-9
    assert np.allclose(gpu.solution, [1.0, 0.0], atol=1e-6)
    # the same problem stated as a minimisation of -c: objective -1, same solution
    kw["c"] = -kw["c"]
    gmin = MPCSolver(_qp(name="min", **kw), regularization=FixedRegularization(1e-8, -1e-8)).solve()
    assert abs(gmin.objective + gpu.objective) <= 1e-7
    assert np.allclose(gmin.solution, gpu.solution, atol=1e-6)


def test_max_wall_time_stop():
    """MAXIMUM_WALLTIME_EXCEEDED (src/solver.jl:216-217: `elapsed_time(solver) >= max_wall_time`, tested
    after the optimality / infeasibility / divergence / max_iter rules): with max_wall_time = 0 the
    first termination test stops at the starting point — the oracle's starting point, objective to
    1e-9; with a budget below the full solve's loop time the solve stops early, after at least that
    budget, with the status and an iterate that is not optimal yet."""
    from madipm_amd import MPCSolver, FixedRegularization, MAXIMUM_WALLTIME_EXCEEDED, SOLVE_SUCCEEDED
    from madipm_amd.instances import random_lp
    qp = random_lp(300, 700, 0.02, 5)
    reg = FixedRegularization(1e-8, -1e-8)
    gpu = MPCSolver(qp, regularization=reg, max_iter=300, max_wall_time=0.0).solve()
    ref = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=300, max_wall_time=0.0)).solve()
    assert gpu.status == MAXIMUM_WALLTIME_EXCEEDED == ref.status
    assert gpu.iter == ref.iter == 0
    assert abs(gpu.objective - ref.objective) <= 1e-9 * max(1.0, abs(ref.objective))
    s = MPCSolver(qp, regularization=reg, max_iter=300)
    full = s.solve()
    assert full.status == SOLVE_SUCCEEDED and full.iter >= 6
    budget = 0.4 * full.counters.total_time
    part = MPCSolver(qp, regularization=reg, max_iter=300, max_wall_time=budget).solve()
    assert part.status == MAXIMUM_WALLTIME_EXCEEDED
    assert 0 < part.iter < full.iter
    assert part.counters.total_time >= budget
