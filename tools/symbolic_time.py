"""Host symbolic analysis time of a bench config, CPU only (no GPU needed): MADIPM_SYMBOLIC_TIMING=1
python tools/symbolic_time.py neos|ex10|supportcase10 prints the phase clocks and the total."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "madipm.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from helpers import lp_k2  # noqa: E402
from madipm_amd import _lib as L  # noqa: E402
from madipm_amd import instances as I  # noqa: E402
from madipm_amd import standard_form_qp  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "neos"
make = {"ex10": I.ex10_standin, "supportcase10": I.supportcase10_standin, "neos": I.neos5052403_standin}[name]
K, Lw = lp_k2(standard_form_qp(make()), 0, well=True)
cp = np.ascontiguousarray(Lw.indptr, np.int64)
rv = np.ascontiguousarray(Lw.indices, np.int32)
o = L.LDLOpts()
L.madipm_ldl_default_opts(C.byref(o))
for rep in range(int(os.environ.get("REPS", "2"))):
    h = L.vp()
    t = time.time()
    rc = L.lib.madipm_symbolic_analyze(Lw.shape[0], L.ptr(cp, C.c_int64), L.ptr(rv, C.c_int32), C.byref(o), None,
                                       C.byref(h))
    dt = time.time() - t
    inf = L.LDLInfo()
    L.lib.madipm_symbolic_info(h, C.byref(inf))
    print(f"{name} symbolic rc {rc} {dt:.3f} s flops {inf.flops:.4g} nnzL {inf.nnzL}", flush=True)
    L.lib.madipm_symbolic_destroy(h)
