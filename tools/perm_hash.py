"""Ordering hash + analysis wall time of bench configs, CPU only: checks that a host-analysis speed-up
keeps the permutation bit-identical (python tools/perm_hash.py ex10 supportcase10 neos)."""
import ctypes as C, os, sys, time, hashlib
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "madipm.jl_amd")); sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from helpers import lp_k2
from madipm_amd import _lib as L, instances as I, standard_form_qp
for name in sys.argv[1:]:
    make = {"ex10": I.ex10_standin, "supportcase10": I.supportcase10_standin, "neos": I.neos5052403_standin}[name]
    K, Lw = lp_k2(standard_form_qp(make()), 0, well=True)
    cp = np.ascontiguousarray(Lw.indptr, np.int64); rv = np.ascontiguousarray(Lw.indices, np.int32)
    o = L.LDLOpts(); L.madipm_ldl_default_opts(C.byref(o))
    h = L.vp(); t = time.time()
    rc = L.lib.madipm_symbolic_analyze(Lw.shape[0], L.ptr(cp, C.c_int64), L.ptr(rv, C.c_int32), C.byref(o), None, C.byref(h))
    dt = time.time() - t
    p = np.zeros(Lw.shape[0], np.int32)
    L.lib.madipm_symbolic_perm(h, L.ptr(p, C.c_int32))
    print(name, rc, f"{dt:.3f} s", hashlib.sha1(p.tobytes()).hexdigest()[:12], flush=True)
    L.lib.madipm_symbolic_destroy(h)
