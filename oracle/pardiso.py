"""MKL PARDISO (symmetric indefinite, mtype -2) as the oracle MPC's linear solver — CPU BASELINE ONLY.

Test/benchmark infrastructure: used by bench.py's `cpu_baseline` leg and by tests, never by the
product.  The reference's CPU benchmark (scripts/benchmarks_cpu.jl:26-50) drives MadIPM with a
supernodal multithreaded direct solver (HSL MA57); neither MA57 nor LDLFactorizations can run here
(no Julia, no HSL), so the strongest supernodal symmetric-indefinite CPU solver in this image —
Intel MKL PARDISO (`/opt/conda/lib/libmkl_rt.so`) — stands in, driven by the oracle's MPC loop
(oracle/mpc.py, `linear_solver = "pardiso"`).

Usage per pattern: analysis (phase 11, METIS nested dissection or a given order) once; per
iteration numeric factorisation (phase 22) and solves (phase 33).  Static pivoting with PARDISO's
pivot perturbation (quasi-definite K2 needs no 2x2 pivots); maximum weighted matching and scaling
off (not needed for quasi-definite matrices, and they cost time).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np
import scipy.sparse as sp

_MKL = None
MKL_PATH = "/opt/conda/lib/libmkl_rt.so"


def available() -> bool:
    return os.path.exists(MKL_PATH)


def mkl():
    global _MKL
    if _MKL is None:
        # GNU OpenMP threading layer: the process may already hold torch's libgomp, and MKL's default
        # Intel OpenMP runtime beside it crashes multithreaded PARDISO (measured: SIGSEGV at 8 threads).
        # Selected through the environment before the library loads (MKL_Set_Threading_Layer after
        # loading leaves MKL single-threaded).
        os.environ.setdefault("MKL_THREADING_LAYER", "GNU")
        _MKL = C.CDLL(MKL_PATH)
        _MKL.pardiso.restype = None
        _MKL.MKL_Set_Num_Threads.argtypes = [C.c_int]
        _MKL.MKL_Get_Max_Threads.restype = C.c_int
    return _MKL


def set_threads(n: int) -> int:
    m = mkl()
    m.MKL_Set_Num_Threads(int(n))
    return int(m.MKL_Get_Max_Threads())


class PardisoLDL:
    """LDL^T of a symmetric (quasi-definite) matrix with MKL PARDISO; the pattern is analysed once.

    `K` may be any scipy sparse symmetric matrix; its upper triangle (CSR, 0-based) is handed over.
    `perm` (optional): pivot order (perm[k] = original index of the k-th pivot), else METIS."""

    def __init__(self, K, perm=None, perturb_exp: int = 13, iparm: dict | None = None):
        U = sp.triu(sp.csr_matrix(K)).tocsr()
        U.sort_indices()
        self.n = U.shape[0]
        self.ia = np.ascontiguousarray(U.indptr, np.int32)
        self.ja = np.ascontiguousarray(U.indices, np.int32)
        self.a = np.ascontiguousarray(U.data, np.float64)
        self.pt = (C.c_int64 * 64)()
        self.iparm = (C.c_int32 * 64)()
        ip = self.iparm
        ip[0] = 1            # non-default iparm
        ip[1] = 3            # parallel nested dissection (METIS), unless a user order is given
        ip[7] = 0            # iterative refinement: default (up to 2 steps after perturbed pivots)
        ip[9] = perturb_exp  # pivot perturbation 10^-perturb_exp
        ip[10] = 0           # no scaling
        ip[12] = 0           # no weighted matching
        ip[17] = -1          # report nnz(L)
        ip[20] = 0           # 1x1 diagonal pivoting only (quasi-definite)
        ip[23] = 1           # two-level parallel factorisation
        ip[34] = 1           # zero-based indexing
        for k, v in (iparm or {}).items():
            ip[k] = v
        self.perm = np.zeros(self.n, np.int32)
        if perm is not None:
            # user fill-in reducing order, perm[k] = original index of pivot k (checked: this convention
            # reproduces the analysis' nnz(L); its inverse multiplies the fill by ~45 on ex10)
            ip[4] = 1
            self.perm[:] = np.asarray(perm, np.int32)
        self.mtype = -2
        self.t_analysis = self.t_factor = self.t_solve = 0.0
        self.nfactor = self.nsolve = 0
        t0 = time.perf_counter()
        self._call(11, self.a)
        self.t_analysis = time.perf_counter() - t0
        self.nnzL = int(ip[17])
        self.ok = False

    def _call(self, phase, a, b=None, x=None, nrhs=1):
        err = C.c_int32(0)
        maxfct, mnum, msg = C.c_int32(1), C.c_int32(1), C.c_int32(0)
        dummy = np.zeros(1)
        bb = b if b is not None else dummy
        xx = x if x is not None else dummy
        mkl().pardiso(self.pt, C.byref(maxfct), C.byref(mnum), C.byref(C.c_int32(self.mtype)),
                      C.byref(C.c_int32(phase)), C.byref(C.c_int32(self.n)), a.ctypes.data_as(C.c_void_p),
                      self.ia.ctypes.data_as(C.c_void_p), self.ja.ctypes.data_as(C.c_void_p),
                      self.perm.ctypes.data_as(C.c_void_p), C.byref(C.c_int32(nrhs)), self.iparm,
                      C.byref(msg), bb.ctypes.data_as(C.c_void_p), xx.ctypes.data_as(C.c_void_p), C.byref(err))
        return err.value

    def same_pattern(self, K) -> bool:
        U = sp.triu(sp.csr_matrix(K)).tocsr()
        U.sort_indices()
        return (U.nnz == len(self.ja) and np.array_equal(U.indptr, self.ia) and np.array_equal(U.indices, self.ja))

    def factorize(self, K) -> bool:
        U = sp.triu(sp.csr_matrix(K)).tocsr()
        U.sort_indices()
        if not (np.array_equal(U.indptr, self.ia) and np.array_equal(U.indices, self.ja)):
            raise ValueError("PardisoLDL.factorize: pattern changed since the analysis")
        self.a[:] = U.data  # in place: PARDISO keeps referring to the array of the analysis
        t0 = time.perf_counter()
        err = self._call(22, self.a)
        self.t_factor += time.perf_counter() - t0
        self.nfactor += 1
        # iparm[13]: number of perturbed pivots; an exact zero pivot is an error (-4)
        self.ok = err == 0
        self.nperturbed = int(self.iparm[13])
        self.inertia = (int(self.iparm[21]), int(self.iparm[22]))
        return self.ok

    def solve(self, b):
        b = np.ascontiguousarray(b, np.float64)
        x = np.empty_like(b)
        bc = b.copy()
        t0 = time.perf_counter()
        err = self._call(33, self.a, bc, x)
        self.t_solve += time.perf_counter() - t0
        self.nsolve += 1
        if err != 0:
            raise FloatingPointError(f"PARDISO solve error {err}")
        return x

    def free(self):
        if getattr(self, "pt", None) is not None:
            self._call(-1, self.a)
            self.pt = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
