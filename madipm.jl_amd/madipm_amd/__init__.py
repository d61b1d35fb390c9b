"""madipm_amd — MI355X-native (gfx950) hot path of MadIPM's Mehrotra predictor-corrector.

Host-side mirror of the reference's interface (klamike/MadIPM.jl: `MPCSolver`, `solve!`, `madipm`,
`IPMOptions` types, `standard_form_qp`, `presolve_qp`-style helpers) over the C-ABI library
libmadipm_hip.so (include/madipm_hip.h).  Importing the solver requires the built library.
"""
from .qp import QuadraticModel, simple_lp, standard_form_qp, scale_qp  # noqa: F401
from .mps import read_mps, parse_mps  # noqa: F401
from .presolve import presolve_qp, postsolve  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # the GPU pieces load libmadipm_hip lazily so that the pure-host helpers import without it
    if name in ("MPCSolver", "madipm", "solve", "AdaptiveStep", "ConservativeStep", "MehrotraAdaptiveStep",
                "NoRegularization", "FixedRegularization", "AdaptiveRegularization", "Mehrotra",
                "SparseKKTSystem", "ScaledSparseKKTSystem", "NormalKKTSystem", "ExecutionStats",
                "SOLVE_SUCCEEDED", "INFEASIBLE_PROBLEM_DETECTED", "MAXIMUM_ITERATIONS_EXCEEDED",
                "MAXIMUM_WALLTIME_EXCEEDED", "DIVERGING_ITERATES", "ERROR_IN_STEP_COMPUTATION", "INTERNAL_ERROR",
                "STATUS_NAMES", "RCCLComm", "HostComm", "SolveException", "UnfactorizedSolveException"):
        from . import solver
        return getattr(solver, name)
    if name == "HIPLDLSolver":
        from .linear_solver import HIPLDLSolver
        return HIPLDLSolver
    raise AttributeError(name)
