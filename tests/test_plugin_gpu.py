"""The `linear_solver=` seam in a loop (SURVEY §8 b; BASELINE north star: "an AbstractLinearSolver ...
that drops into the existing MPCSolver / solve! / linear_solver= plugin surface").

The reference's GPU test (/root/reference/test/test_gpu.jl:9-19) runs MadIPM's OWN `MPCSolver`
loop with a plugged-in GPU linear solver for (K2.5, LDL), (K2, LDL) and (NormalKKT, CHOLESKY) and
checks SOLVE_SUCCEEDED.  Julia is absent here, so the reference-shaped loop is the oracle's
restatement of `mpc!` (oracle/mpc.py, src/solver.jl:332-360): it builds each KKT matrix itself and
drives the HIP library only through the plugin methods, in the reference's order —
`LS(aug_com)` once per pattern (normalkkt.jl:113-115), then per factorisation `factorize!`
(linear_solver.jl:10) -> `is_factorized` (linear_solver.jl:11, utils.jl:54-62; the x100
regularisation retry reads it) and per solve `solve!(ls, x)` on a DEVICE vector
(linear_solver.jl:26).  Checked: status SOLVE_SUCCEEDED (the reference's assertion) and status +
objective equal to the native GPU driver (madipm_solver_*) within 1e-6 max(1, |obj|).
"""
import os

import numpy as np
import pytest

from oracle.mpc import OracleMPC, OracleOptions

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


class HIPPlugin:
    """MadNLP.AbstractLinearSolver calls of the loop -> madipm_amd.linear_solver.HIPLDLSolver.  The
    loop lives on the host (numpy): values and right-hand sides are uploaded, the factor and the
    solve run on the GPU through the C-ABI (madipm_ldl_analyze / _factorize / _is_factorized /
    _solve)."""

    calls = []

    def __init__(self, Lw, cholesky=False):
        from madipm_amd.linear_solver import HIPLDLSolver
        self.ls = HIPLDLSolver(Lw.shape[0], Lw.indptr, Lw.indices, cholesky=cholesky)
        HIPPlugin.calls.append("LS")

    def factorize(self, vals):                       # MadNLP.factorize!(ls)
        HIPPlugin.calls.append("factorize!")
        self.ls.factorize(torch.from_numpy(np.ascontiguousarray(vals, np.float64)).cuda())

    def is_factorized(self):                         # MadIPM.is_factorized(ls)
        return self.ls.is_factorized()

    def solve(self, b):                              # MadNLP.solve!(ls, x): in place on a device vector
        HIPPlugin.calls.append("solve!")
        x = torch.from_numpy(np.array(b, np.float64)).cuda()
        self.ls.solve(x)
        return x.cpu().numpy()


def _problems():
    from madipm_amd import read_mps, simple_lp
    gold = os.path.join(os.path.dirname(__file__), "golden", "afiro.mps")
    return {"simple_lp": simple_lp, "afiro": lambda: read_mps(gold)}


@pytest.mark.parametrize("kkt,algo", [("K25", "LDL"), ("K2", "LDL"), ("normal", "CHOLESKY")])
@pytest.mark.parametrize("case", ["simple_lp", "afiro"])
def test_linear_solver_plugin_in_mpc_loop(case, kkt, algo):
    from madipm_amd import MPCSolver, FixedRegularization, SOLVE_SUCCEEDED
    from madipm_amd import solver as S
    qp = _problems()[case]()
    chol = algo == "CHOLESKY"
    HIPPlugin.calls.clear()
    o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), max_iter=300, kkt_system=kkt))
    o.linear_solver = lambda Lw: HIPPlugin(Lw, cholesky=chol)
    res = o.solve()
    assert res.status == SOLVE_SUCCEEDED, res.status       # test/test_gpu.jl:20
    # the seam was used the reference's way: one analysis, a factorisation per iteration (+ init),
    # two solves per factorisation at least (predictor + corrector; init: primal + dual)
    assert HIPPlugin.calls.count("LS") == 1
    nf = HIPPlugin.calls.count("factorize!")
    assert nf >= res.iter and HIPPlugin.calls.count("solve!") >= 2 * nf
    kcls = {"K2": S.SparseKKTSystem, "K25": S.ScaledSparseKKTSystem, "normal": S.NormalKKTSystem}[kkt]
    nat = MPCSolver(qp, kkt_system=kcls, regularization=FixedRegularization(1e-8, -1e-8), max_iter=300).solve()
    assert nat.status == res.status
    assert abs(nat.objective - res.objective) <= 1e-6 * max(1.0, abs(res.objective)), (nat.objective, res.objective)
    if case == "simple_lp":
        assert abs(res.objective - 1.0) <= 1e-6              # test/runtests.jl:29-60


def test_plugin_cholesky_rejects_indefinite():
    """Cholesky semantics at the plugin: a quasi-definite K2 (negative pivots) is not factorised
    (is_factorized == false: the loop's regularisation retry sees it); the LDL^T setting accepts it."""
    import scipy.sparse as sp
    from madipm_amd.linear_solver import HIPLDLSolver
    K = sp.csc_matrix(np.array([[2.0, 1.0], [1.0, -1.0]]))
    Lw = sp.tril(K).tocsc()
    Lw.sort_indices()
    vals = torch.from_numpy(Lw.data.copy()).cuda()
    chol = HIPLDLSolver(2, Lw.indptr, Lw.indices, cholesky=True)
    assert chol.factorize(vals) > 0 and not chol.is_factorized()
    ldl = HIPLDLSolver(2, Lw.indptr, Lw.indices)
    assert ldl.factorize(vals) == 0 and ldl.is_factorized() and ldl.inertia() == (1, 0, 1)
