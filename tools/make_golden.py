"""Generate tests/golden/oracle_traces.json: per-iteration traces of the oracle restatement on the
reference-pinned problems (simple_lp, AFIRO) and seeded random LPs, with HiGHS objectives.

Run from the repo root:  python tools/make_golden.py
The fixture is DATA (inputs are regenerated from seeds / the committed MPS; outputs are numbers).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "madipm.jl_amd")]

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.optimize import linprog  # noqa: E402

from madipm_amd import read_mps, simple_lp, standard_form_qp  # noqa: E402
from madipm_amd.instances import random_lp  # noqa: E402
from oracle.mpc import OracleMPC, OracleOptions  # noqa: E402


def highs(qp):
    A = sp.coo_matrix((qp.Avals, (qp.Arows, qp.Acols)), shape=(qp.ncon, qp.nvar)).tocsr()
    eq = qp.lcon == qp.ucon
    up = ~eq & np.isfinite(qp.ucon)
    lo = ~eq & np.isfinite(qp.lcon)
    Aub = sp.vstack([A[up], -A[lo]])
    bub = np.concatenate([qp.ucon[up], -qp.lcon[lo]])
    bounds = list(zip(np.where(np.isfinite(qp.lvar), qp.lvar, None), np.where(np.isfinite(qp.uvar), qp.uvar, None)))
    sgn = 1.0 if qp.minimize else -1.0
    r = linprog(sgn * qp.c, A_ub=Aub if Aub.shape[0] else None, b_ub=bub if Aub.shape[0] else None,
                A_eq=A[eq] if eq.any() else None, b_eq=qp.lcon[eq] if eq.any() else None, bounds=bounds,
                method="highs")
    return sgn * r.fun + qp.c0


CASES = {
    "simple_lp_noreg": (lambda: simple_lp(), dict(regularization=("none",))),
    "simple_lp_std": (lambda: standard_form_qp(simple_lp()), dict()),
    "afiro_fixed": (lambda: read_mps(os.path.join(ROOT, "tests", "golden", "afiro.mps")),
                    dict(regularization=("fixed", 1e-8, -1e-8), max_iter=300)),
    "afiro_std_fixed": (lambda: standard_form_qp(read_mps(os.path.join(ROOT, "tests", "golden", "afiro.mps"))),
                        dict(regularization=("fixed", 1e-8, -1e-8), max_iter=300)),
    "random_lp_60x120_s0": (lambda: random_lp(60, 120, 0.05, 0, ineq_frac=0.3, free_frac=0.05),
                            dict(regularization=("fixed", 1e-8, -1e-8))),
    "random_lp_100x200_s1": (lambda: random_lp(100, 200, 0.03, 1, ineq_frac=0.2),
                             dict(regularization=("fixed", 1e-8, -1e-8))),
}


def main():
    out = {}
    for name, (mk, kw) in CASES.items():
        qp = mk()
        st = OracleMPC(qp, OracleOptions(**kw)).solve()
        out[name] = {"options": {k: list(v) if isinstance(v, tuple) else v for k, v in kw.items()},
                     "status": st.status, "iter": st.iter, "objective": st.objective,
                     "highs_objective": highs(qp), "trace": st.trace}
        print(name, st.status, st.iter, st.objective, out[name]["highs_objective"])
    with open(os.path.join(ROOT, "tests", "golden", "oracle_traces.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
