"""Which configurations run the factorisation's root tail on the side stream (MADIPM_ROOT_ASYNC=2
prints the launch list and the last launch's fronts with their solve kind): python tools/root_tail_probe.py"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "madipm.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
os.environ.setdefault("MADIPM_ROOT_ASYNC", "2")
import torch  # noqa: F401,E402
from helpers import lp_k2  # noqa: E402
from madipm_amd import standard_form_qp  # noqa: E402
from madipm_amd import instances as I  # noqa: E402
from madipm_amd.linear_solver import HIPLDLSolver  # noqa: E402
for name, qp in [("supportcase10 0.15", lambda: I.supportcase10_standin(scale=0.15)),
                 ("supportcase10 0.3", lambda: I.supportcase10_standin(scale=0.3)),
                 ("supportcase10 1.0", lambda: I.supportcase10_standin())]:
    K, Lw = lp_k2(standard_form_qp(qp()), 0, well=True)
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices)
    print(name, "root_tail_async", ls.info()["root_tail_async"], flush=True)
    del ls
