"""ctypes binding of libmadipm_hip.so (declarations: include/madipm_hip.h).

The product path has no CPU fallback: if the library is missing this module raises on import.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# MADIPM_LIB (A/B measurements of build variants) points at another build of the same library
LIB_PATH = Path(os.environ["MADIPM_LIB"]) if os.environ.get("MADIPM_LIB") else _HERE / "lib" / "libmadipm_hip.so"

if not LIB_PATH.exists():
    raise ImportError(
        f"libmadipm_hip.so not found at {LIB_PATH}; build it with `python -c \"import __graft_entry__ as g; g.build()\"` "
        "(the HIP extension is required: there is no CPU fallback)")

lib = C.CDLL(str(LIB_PATH))

i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
f64p = C.POINTER(C.c_double)
vp = C.c_void_p


class LDLOpts(C.Structure):
    _fields_ = [("ordering", C.c_int32), ("dense_alpha", C.c_double), ("relax", C.c_int32),
                ("small_front_max", C.c_int32), ("pivot_tol", C.c_double), ("nshards", C.c_int32),
                ("cholesky", C.c_int32)]


class LDLInfo(C.Structure):
    _fields_ = [("n", C.c_int64), ("nnzK", C.c_int64), ("nnzL", C.c_int64), ("nnzL_stored", C.c_int64),
                ("flops", C.c_double), ("nsuper", C.c_int32), ("nlevels", C.c_int32),
                ("max_front", C.c_int32), ("nbig", C.c_int32), ("arena_bytes", C.c_int64),
                ("lb_groups", C.c_int32), ("lb_members", C.c_int32),
                ("fold_fronts", C.c_int32), ("fold_leaves", C.c_int32),
                ("xch_fact", C.c_int64), ("xch_solve", C.c_int64), ("xch_gather", C.c_int64),
                ("tree_fronts", C.c_int32), ("tree_medium", C.c_int32),
                ("root_tail_async", C.c_int32), ("pad_", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


NKERNELS = 24  # MADIPM_NKERNELS


class KStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("time_ms", C.c_double),
                ("bytes", C.c_double), ("flops", C.c_double), ("alg_bytes", C.c_double)]


def kstats_to_list(arr) -> list:
    return [{"name": k.name.decode(), "launches": int(k.launches), "time_ms": float(k.time_ms),
             "bytes": float(k.bytes), "flops": float(k.flops), "alg_bytes": float(k.alg_bytes)} for k in arr]


def _sig(name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


madipm_version = _sig("madipm_version", C.c_int, [])
madipm_last_error = _sig("madipm_last_error", C.c_char_p, [])
madipm_device_count = _sig("madipm_device_count", C.c_int, [])
madipm_set_device = _sig("madipm_set_device", C.c_int, [C.c_int32])
madipm_ldl_default_opts = _sig("madipm_ldl_default_opts", None, [C.POINTER(LDLOpts)])
madipm_symbolic_analyze = _sig("madipm_symbolic_analyze", C.c_int,
                               [C.c_int32, i64p, i32p, C.POINTER(LDLOpts), i32p, C.POINTER(vp)])
madipm_symbolic_info = _sig("madipm_symbolic_info", C.c_int, [vp, C.POINTER(LDLInfo)])
madipm_symbolic_perm = _sig("madipm_symbolic_perm", C.c_int, [vp, i32p])
madipm_symbolic_supernodes = _sig("madipm_symbolic_supernodes", C.c_int, [vp, i32p, i32p, i32p])
madipm_symbolic_destroy = _sig("madipm_symbolic_destroy", None, [vp])
_sig("madipm_symbolic_analyze_shard", C.c_int, [C.c_int32, i64p, i32p, C.POINTER(LDLOpts), C.c_int32, C.c_int32, i32p,
                                                C.POINTER(vp)])
_sig("madipm_symbolic_shard_info", C.c_int, [vp, i32p, f64p, f64p, f64p])
_sig("madipm_ldl_analyze", C.c_int, [C.c_int32, i64p, i32p, C.POINTER(LDLOpts), i32p, C.POINTER(vp)])
_sig("madipm_ldl_get_info", C.c_int, [vp, C.POINTER(LDLInfo)])
_sig("madipm_ldl_factorize", C.c_int, [vp, vp, vp])
_sig("madipm_ldl_factorize_async", C.c_int, [vp, vp, vp])
_sig("madipm_ldl_is_factorized", C.c_int, [vp])
_sig("madipm_ldl_solve", C.c_int, [vp, vp, C.c_int32, vp])
_sig("madipm_ldl_inertia", C.c_int, [vp, i32p, i32p, i32p])
_sig("madipm_ldl_get_d", C.c_int, [vp, f64p])
_sig("madipm_ldl_perm", C.c_int, [vp, i32p])
_sig("madipm_ldl_destroy", None, [vp])
_sig("madipm_ldl_set_timing", C.c_int, [vp, C.c_uint32])
_sig("madipm_ldl_kernel_stats", C.c_int, [vp, C.POINTER(KStat)])
_sig("madipm_ldl_analyze_shard", C.c_int, [C.c_int32, i64p, i32p, C.POINTER(LDLOpts), C.c_int32, C.c_int32, i32p,
                                           C.POINTER(vp)])
_sig("madipm_ldl_factorize_phase", C.c_int, [vp, C.c_int32, vp, vp, C.POINTER(vp), i64p])
_sig("madipm_ldl_solve_phase", C.c_int, [vp, C.c_int32, vp, vp, C.POINTER(vp), i64p])
_sig("madipm_ldl_shard_info", C.c_int, [vp, i32p, f64p, f64p, f64p])
_sig("madipm_local_allreduce", C.c_int, [C.POINTER(vp), C.c_int32, C.c_int64, vp])
_sig("madipm_comm_unique_id", C.c_int, [C.c_char_p])
_sig("madipm_comm_create", C.c_int, [C.c_int32, C.c_int32, C.c_char_p, C.POINTER(vp)])
_sig("madipm_comm_destroy", None, [vp])
_sig("madipm_comm_allreduce", C.c_int, [vp, vp, C.c_int64, vp])
_sig("madipm_comm_allgather", C.c_int, [vp, vp, C.c_int64, vp])
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, f64p, C.c_int64, vp)
_sig("madipm_comm_create_host", C.c_int, [C.c_int32, C.c_int32, ALLREDUCE_FN, vp, C.POINTER(vp)])


class MadIPMError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        raise MadIPMError(f"{what}: {madipm_last_error().decode(errors='replace')} (code {rc})")
    return rc


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None


def default_ldl_opts(**kw) -> LDLOpts:
    o = LDLOpts()
    madipm_ldl_default_opts(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


class Symbolic:
    """Host-side symbolic analysis (ordering, etree, supernodes) of a lower CSC pattern."""

    def __init__(self, n, colptr, rowval, opts: LDLOpts | None = None, perm=None, nshards=1, shard=0):
        self.n = int(n)
        self._colptr = np.ascontiguousarray(colptr, np.int64)
        self._rowval = np.ascontiguousarray(rowval, np.int32)
        up = None if perm is None else np.ascontiguousarray(perm, np.int32)
        if opts is None:
            opts = default_ldl_opts(ordering=2 if perm is not None else 4)
        h = vp()
        upp = ptr(up, C.c_int32) if up is not None else None
        if nshards > 1:
            check(lib.madipm_symbolic_analyze_shard(self.n, ptr(self._colptr, C.c_int64), ptr(self._rowval, C.c_int32),
                                                    C.byref(opts), int(nshards), int(shard), upp, C.byref(h)),
                  "madipm_symbolic_analyze_shard")
        else:
            check(madipm_symbolic_analyze(self.n, ptr(self._colptr, C.c_int64), ptr(self._rowval, C.c_int32),
                                          C.byref(opts), upp, C.byref(h)), "madipm_symbolic_analyze")
        self.h = h

    def shard_info(self) -> dict:
        ns = self.info()["nsuper"]
        owner = np.empty(ns, np.int32)
        tc, mx, sm = C.c_double(), C.c_double(), C.c_double()
        check(lib.madipm_symbolic_shard_info(self.h, ptr(owner, C.c_int32), C.byref(tc), C.byref(mx), C.byref(sm)),
              "madipm_symbolic_shard_info")
        return {"owner": owner, "top_cost": tc.value, "shard_cost_max": mx.value, "shard_cost_sum": sm.value}

    def info(self) -> dict:
        inf = LDLInfo()
        check(madipm_symbolic_info(self.h, C.byref(inf)), "madipm_symbolic_info")
        return inf.as_dict()

    def perm(self) -> np.ndarray:
        p = np.empty(self.n, np.int32)
        check(madipm_symbolic_perm(self.h, ptr(p, C.c_int32)), "madipm_symbolic_perm")
        return p

    def supernodes(self):
        ns = self.info()["nsuper"]
        first = np.empty(ns + 1, np.int32)
        parent = np.empty(ns, np.int32)
        nrows = np.empty(ns, np.int32)
        check(madipm_symbolic_supernodes(self.h, ptr(first, C.c_int32), ptr(parent, C.c_int32),
                                         ptr(nrows, C.c_int32)), "madipm_symbolic_supernodes")
        return first, parent, nrows

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            madipm_symbolic_destroy(h)
            self.h = None
