"""ORACLE (test infrastructure only): ctypes wrapper of oracle/ldl_ref.c, the up-looking sparse
LDL^T of LDLFactorizations.jl (see the C file header).  Built by oracle/Makefile into
oracle/_build/libldl_oracle.so.  Only tests/ and bench.py's cpu_baseline leg may use it."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np
import scipy.sparse as sp

_DIR = Path(__file__).resolve().parent
_SO = _DIR / "_build" / "libldl_oracle.so"


def build():
    subprocess.run(["make", "-s", "-C", str(_DIR)], check=True)


def _load():
    if not _SO.exists():
        build()
    lib = C.CDLL(str(_SO))
    vp = C.c_void_p
    lib.ldl_ref_symbolic.restype = vp
    lib.ldl_ref_symbolic.argtypes = [C.c_int64, vp, vp, vp]
    lib.ldl_ref_numeric.restype = C.c_int64
    lib.ldl_ref_numeric.argtypes = [vp, vp, vp, vp]
    lib.ldl_ref_solve.restype = None
    lib.ldl_ref_solve.argtypes = [vp, vp]
    lib.ldl_ref_nnz.restype = C.c_int64
    lib.ldl_ref_nnz.argtypes = [vp]
    lib.ldl_ref_get_d.restype = None
    lib.ldl_ref_get_d.argtypes = [vp, vp]
    lib.ldl_ref_free.restype = None
    lib.ldl_ref_free.argtypes = [vp]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


class OracleLDL:
    """LDL^T of a symmetric matrix (scipy sparse, any format) in the given pivot order."""

    def __init__(self, K, perm=None):
        K = sp.csc_matrix(K)
        K.sort_indices()
        self.n = K.shape[0]
        self.Ap = np.ascontiguousarray(K.indptr, np.int64)
        self.Ai = np.ascontiguousarray(K.indices, np.int32)
        self.Ax = np.ascontiguousarray(K.data, np.float64)
        self.perm = None if perm is None else np.ascontiguousarray(perm, np.int32)
        L = lib()
        self.h = L.ldl_ref_symbolic(self.n, self.Ap.ctypes.data, self.Ai.ctypes.data,
                                    self.perm.ctypes.data if self.perm is not None else None)

    def factorize(self, values=None) -> int:
        if values is not None:
            self.Ax = np.ascontiguousarray(values, np.float64)
        r = lib().ldl_ref_numeric(self.h, self.Ap.ctypes.data, self.Ai.ctypes.data, self.Ax.ctypes.data)
        self.ok = (r == self.n)
        return r

    def solve(self, b):
        if not getattr(self, "ok", False):
            raise FloatingPointError("OracleLDL.solve: the factorization stopped at a zero pivot")
        x = np.ascontiguousarray(b, np.float64).copy()
        lib().ldl_ref_solve(self.h, x.ctypes.data)
        return x

    def nnzL(self) -> int:
        return int(lib().ldl_ref_nnz(self.h)) + self.n

    def diag(self):
        d = np.empty(self.n)
        lib().ldl_ref_get_d(self.h, d.ctypes.data)
        return d

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.ldl_ref_free(h)
            self.h = None
