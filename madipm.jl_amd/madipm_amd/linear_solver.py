"""`HIPLDLSolver`: the MadNLP.AbstractLinearSolver the reference plugs in via `linear_solver=`.

Mirrors the methods MadNLP calls on a linear solver: construction from the lower
CSC `aug_com` (`LS(aug_com; opt)`, src/KKT/normalkkt.jl:113-115), `factorize!`, `solve!`,
`is_inertia` / `inertia`, `improve!`, `introduce`, and MadIPM's `is_factorized`
(src/utils.jl:54-62).  Device vectors are torch tensors on `cuda:*` (HIP); values never leave HBM.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class HIPLDLSolver:
    """Multifrontal supernodal LDL^T on the GPU (libmadipm_hip)."""

    def __init__(self, n, colptr, rowval, *, ordering=4, relax=1, pivot_tol=0.0, perm=None,
                 small_front_max=128, nshards=1, shard=None, cholesky=False):
        """nshards > 1 and shard None: all shards of a subtree-sharded factorisation on this device
        (SURVEY §8 e, local all-reduce).  shard = r: only shard r (one process per GPU); drive it with
        factorize_phase / solve_phase and your own collective (or use MPCSolver(comm=...)).
        cholesky=True: Cholesky semantics (SPD; a pivot that is not > 0 fails — cuDSS CHOLESKY, the
        reference's NormalKKTSystem pairing, test/test_gpu.jl:11)."""
        self.n = int(n)
        self._colptr = np.ascontiguousarray(colptr, np.int64)
        self._rowval = np.ascontiguousarray(rowval, np.int32)
        opts = L.default_ldl_opts(ordering=2 if perm is not None else ordering, relax=relax,
                                  pivot_tol=pivot_tol, small_front_max=small_front_max,
                                  nshards=nshards if shard is None else 1, cholesky=int(bool(cholesky)))
        up = None if perm is None else np.ascontiguousarray(perm, np.int32)
        upp = L.ptr(up, C.c_int32) if up is not None else None
        h = L.vp()
        cp, rv = L.ptr(self._colptr, C.c_int64), L.ptr(self._rowval, C.c_int32)
        if shard is None:
            L.check(L.lib.madipm_ldl_analyze(self.n, cp, rv, C.byref(opts), upp, C.byref(h)), "madipm_ldl_analyze")
        else:
            L.check(L.lib.madipm_ldl_analyze_shard(self.n, cp, rv, C.byref(opts), int(nshards), int(shard), upp,
                                                   C.byref(h)), "madipm_ldl_analyze_shard")
        self.h = h
        self.nshards, self.shard = int(nshards), shard

    # ---- MadNLP interface names
    def introduce(self) -> str:
        return "madipm-hip supernodal LDL^T (gfx950)"

    @staticmethod
    def is_supported(dtype=np.float64) -> bool:
        return dtype == np.float64

    def info(self) -> dict:
        inf = L.LDLInfo()
        L.check(L.lib.madipm_ldl_get_info(self.h, C.byref(inf)), "madipm_ldl_get_info")
        return inf.as_dict()

    def factorize(self, nzval, stream=None) -> int:
        """factorize!: nzval is a device tensor (float64, CSC order of construction)."""
        assert nzval.dtype.itemsize == 8 and nzval.numel() == self._colptr[-1]
        rc = L.lib.madipm_ldl_factorize(self.h, C.c_void_p(nzval.data_ptr()), C.c_void_p(_stream(stream)))
        return L.check(rc, "madipm_ldl_factorize")

    def is_factorized(self) -> bool:
        return bool(L.check(L.lib.madipm_ldl_is_factorized(self.h), "madipm_ldl_is_factorized"))

    def solve(self, x, stream=None):
        """solve!(ls, x): in place on a device tensor of length n (or n x nrhs column blocks)."""
        assert x.dtype.itemsize == 8 and x.is_contiguous()
        nrhs = x.numel() // max(self.n, 1)
        L.check(L.lib.madipm_ldl_solve(self.h, C.c_void_p(x.data_ptr()), nrhs, C.c_void_p(_stream(stream))),
                "madipm_ldl_solve")
        return x

    def is_inertia(self) -> bool:
        return True

    def inertia(self):
        p, z, n = C.c_int32(), C.c_int32(), C.c_int32()
        L.check(L.lib.madipm_ldl_inertia(self.h, C.byref(p), C.byref(z), C.byref(n)), "madipm_ldl_inertia")
        return p.value, z.value, n.value

    def improve(self) -> bool:
        return False

    def diag(self) -> np.ndarray:
        d = np.empty(self.n)
        L.check(L.lib.madipm_ldl_get_d(self.h, L.ptr(d, C.c_double)), "madipm_ldl_get_d")
        return d

    def perm(self) -> np.ndarray:
        p = np.empty(self.n, np.int32)
        L.check(L.lib.madipm_ldl_perm(self.h, L.ptr(p, C.c_int32)), "madipm_ldl_perm")
        return p

    # ---- subtree sharding (one shard per process; the caller runs the all-reduces)
    def factorize_phase(self, phase, nzval=None, stream=None):
        """phase 1 returns (ptr, len) of the device buffer to all-reduce before phase 2."""
        xb, xl = L.vp(), C.c_int64()
        L.check(L.lib.madipm_ldl_factorize_phase(self.h, int(phase), C.c_void_p(nzval.data_ptr() if nzval is not None else 0),
                                                 C.c_void_p(_stream(stream)), C.byref(xb), C.byref(xl)),
                "madipm_ldl_factorize_phase")
        return xb.value, xl.value

    def solve_phase(self, phase, x, stream=None):
        """phase 1 -> (ptr, len) to all-reduce; phase 2 -> (ptr, len) of the gather buffer (nshards
        slices, this shard's filled, the others zero): all-gather it in place (or sum all-reduce it);
        phase 3 scatters the gathered slices into x -> (0, 0)."""
        xb, xl = L.vp(), C.c_int64()
        L.check(L.lib.madipm_ldl_solve_phase(self.h, int(phase), C.c_void_p(x.data_ptr()), C.c_void_p(_stream(stream)),
                                             C.byref(xb), C.byref(xl)), "madipm_ldl_solve_phase")
        return xb.value, xl.value

    def shard_info(self) -> dict:
        ns = self.info()["nsuper"]
        owner = np.empty(ns, np.int32)
        tc, mx, sm = C.c_double(), C.c_double(), C.c_double()
        L.check(L.lib.madipm_ldl_shard_info(self.h, L.ptr(owner, C.c_int32), C.byref(tc), C.byref(mx), C.byref(sm)),
                "madipm_ldl_shard_info")
        return {"owner": owner, "top_cost": tc.value, "shard_cost_max": mx.value, "shard_cost_sum": sm.value}

    def set_kernel_timing(self, mask: int = (1 << L.NKERNELS) - 1):
        """HIP events around every launch of the kernel kinds in `mask`; clears the statistics."""
        L.check(L.lib.madipm_ldl_set_timing(self.h, int(mask)), "madipm_ldl_set_timing")

    def kernel_stats(self) -> list:
        arr = (L.KStat * L.NKERNELS)()
        L.check(L.lib.madipm_ldl_kernel_stats(self.h, arr), "madipm_ldl_kernel_stats")
        return L.kstats_to_list(arr)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            L.lib.madipm_ldl_destroy(h)
            self.h = None


def local_allreduce(ptrs, n, stream=None):
    """Sum of device buffers (raw pointers) written back to all of them (single-process shards)."""
    arr = (L.vp * len(ptrs))(*[L.vp(p) for p in ptrs])
    L.check(L.lib.madipm_local_allreduce(arr, len(ptrs), int(n), C.c_void_p(_stream(stream))), "local_allreduce")


def _stream(stream) -> int:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return int(stream)
