"""Diagnostics: one MPC solve of a stand-in on cuda:0 (status, iterations, objective, LDL info);
python tools/diag_mpc.py CASE [SCALE]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "madipm.jl_amd"))
from madipm_amd import MPCSolver, FixedRegularization, standard_form_qp  # noqa: E402
from madipm_amd import instances as I  # noqa: E402

case = sys.argv[1]
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
mk = {"ex10": I.ex10_standin, "sc10": I.supportcase10_standin, "neos": I.neos5052403_standin}[case]
qp = standard_form_qp(mk(scale=scale))
kw = dict(regularization=FixedRegularization(1e-8, -1e-8), max_iter=300)
for k in ("nshards",):
    if os.environ.get("DIAG_" + k.upper()):
        kw[k] = int(os.environ["DIAG_" + k.upper()])
t = time.perf_counter()
s = MPCSolver(qp, rethrow_error=True, **kw)
inf = s.ldl_info()
try:
    r = s.solve()
except Exception as e:  # noqa: BLE001  (diagnostics: the rethrown solver exception)
    print(f"{case} exception {type(e).__name__}: {e}", flush=True)
    raise SystemExit(0)
print(f"{case} scale={scale} status={r.status} iter={r.iter} obj={r.objective:.12e} t={time.perf_counter() - t:.2f}s "
      f"tree_fronts={inf['tree_fronts']} fold_fronts={inf['fold_fronts']} max_front={inf['max_front']} nbig={inf['nbig']}",
      flush=True)
