"""The array-type overrides of MadIPM's GPU extension over the C-ABI (csrc/kkt.hip).

Python mirror of `ext/MadIPMCUDAExt/cuda_wrapper.jl` + `MadIPMCUDAExt.jl` (what the Julia extension
`madipm.jl_amd/ext/MadIPMHIPExt` binds with `ccall`): device arrays are torch tensors on `cuda:*`
(HIP), indices 0-based int32 (int64 maps), values float64.

    transfer!(dest, src, map)                      cuda_wrapper.jl:4-24   -> Transfer(map, ndest)(dest, src)
    compress_jacobian!(kkt::NormalKKTSystem)       cuda_wrapper.jl:32-41  -> compress_jacobian
    MadIPMOperator(A; transa, symmetric), mul!     cuda_wrapper.jl:43-94  -> MadIPMOperator
    coo_to_csr(n_rows, n_cols, Ai, Aj, Ax)         cuda_wrapper.jl:96-106 -> coo_to_csr
    assemble_normal_system!(...)                   cuda_wrapper.jl:108-156 -> assemble_normal_system
    build_normal_system(n_rows, n_cols, Jtp, Jtj)  cuda_wrapper.jl:214-234 -> build_normal_system (host)
    fill_structure!(A, rows, cols)                 MadIPMCUDAExt.jl:15-32 -> fill_structure
    NLPModels.obj / grad!                          MadIPMCUDAExt.jl:34-45 -> qp_obj / qp_grad
    update_step!(rule, solver) + get_alpha_max_*   kernels.jl:226-358     -> update_step
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

vp, i32p, i64p, f64p = L.vp, L.i32p, L.i64p, L.f64p

L._sig("madipm_transfer_create", C.c_int, [C.c_int64, vp, C.c_int32, C.c_int64, C.POINTER(vp)])
L._sig("madipm_transfer", C.c_int, [vp, vp, vp, vp])
L._sig("madipm_transfer_destroy", None, [vp])
L._sig("madipm_compress_jacobian", C.c_int, [vp, C.c_int64, C.c_int32, vp, vp, vp])
L._sig("madipm_spmv_create", C.c_int, [C.c_int32, C.c_int32, C.c_int64, vp, vp, vp, C.c_char, C.c_int32,
                                       C.POINTER(vp)])
L._sig("madipm_spmv_apply", C.c_int, [vp, vp, vp, C.c_double, C.c_double, vp])
L._sig("madipm_spmv_size", C.c_int, [vp, i32p, i32p, i64p])
L._sig("madipm_spmv_destroy", None, [vp])
L._sig("madipm_coo_to_csr", C.c_int, [C.c_int32, C.c_int32, C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int32, vp])
L._sig("madipm_build_normal_system", C.c_int, [C.c_int32, C.c_int32, i32p, i32p, i32p, i32p, C.c_int64, i64p])
L._sig("madipm_assemble_normal_system", C.c_int, [C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, vp, vp])
L._sig("madipm_csr_fill_structure", C.c_int, [C.c_int32, vp, vp, vp, vp, vp])
L._sig("madipm_qp_obj", C.c_int, [vp, vp, C.c_double, vp, vp, C.c_int32, vp, f64p, vp])
L._sig("madipm_qp_grad", C.c_int, [vp, vp, vp, vp, C.c_int32, vp])


class StepResult(C.Structure):
    _fields_ = [("alpha_p", C.c_double), ("alpha_d", C.c_double), ("alpha_xl", C.c_double),
                ("alpha_xu", C.c_double), ("alpha_zl", C.c_double), ("alpha_zu", C.c_double),
                ("i_xl", C.c_int32), ("i_xu", C.c_int32), ("i_zl", C.c_int32), ("i_zu", C.c_int32)]


L._sig("madipm_update_step", C.c_int, [C.c_int32, C.c_double, C.c_double, C.c_int32, C.c_int32] + [vp] * 10
       + [C.POINTER(StepResult), vp])


def _stream(stream) -> int:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return int(stream)


def _dptr(t, dtype=None) -> int:
    """Device address of a contiguous torch cuda tensor (None -> NULL)."""
    if t is None:
        return None
    import torch
    assert t.is_cuda and t.is_contiguous(), "expected a contiguous device tensor"
    if dtype is not None:
        assert t.dtype == dtype, (t.dtype, dtype)
    return t.data_ptr() if t.numel() else None


def _torch():
    import torch
    return torch


class Transfer:
    """`MadNLP.transfer!(dest, src, map)`: dest .= 0; dest[map[k]] += src[k] (ascending k per entry)."""

    def __init__(self, map, ndest: int):
        torch = _torch()
        self.h = vp()
        if isinstance(map, torch.Tensor) and map.is_cuda:
            m = map.to(torch.int64).contiguous()
            L.check(L.lib.madipm_transfer_create(m.numel(), _dptr(m), 1, int(ndest), C.byref(self.h)),
                    "madipm_transfer_create")
        else:
            m = np.ascontiguousarray(map, np.int64)
            L.check(L.lib.madipm_transfer_create(m.size, m.ctypes.data, 0, int(ndest), C.byref(self.h)),
                    "madipm_transfer_create")
        self.nsrc, self.ndest = int(m.numel() if hasattr(m, "numel") else m.size), int(ndest)

    def __call__(self, dest, src, stream=None):
        torch = _torch()
        assert dest.numel() == self.ndest and src.numel() == self.nsrc
        L.check(L.lib.madipm_transfer(self.h, _dptr(dest, torch.float64), _dptr(src, torch.float64), _stream(stream)),
                "madipm_transfer")
        return dest

    def __del__(self):
        if getattr(self, "h", None):
            L.lib.madipm_transfer_destroy(self.h)
            self.h = None


def compress_jacobian(AV, n_slack: int, csr_map, ATnz, stream=None):
    """`compress_jacobian!(kkt::NormalKKTSystem)`: AV[end-n_slack+1:end] .= -1 (in place);
    ATnz .= AV[csr_map]."""
    torch = _torch()
    assert csr_map.dtype == torch.int64 and ATnz.numel() == csr_map.numel() == AV.numel()
    L.check(L.lib.madipm_compress_jacobian(_dptr(AV, torch.float64), AV.numel(), int(n_slack), _dptr(csr_map),
                                           _dptr(ATnz, torch.float64), _stream(stream)), "madipm_compress_jacobian")
    return ATnz


class MadIPMOperator:
    """`MadIPMOperator(A::CSR; transa='N', symmetric=false)` and `mul!(y, op, x[, alpha, beta])`.

    A is given as device CSR arrays (rowptr int32 m+1, colval int32, nzval float64).  symmetric:
    the operator is tril(A,-1) + A' (copied at construction, as the reference's `mat`)."""

    def __init__(self, m: int, n: int, rowptr, colval, nzval, transa: str = "N", symmetric: bool = False):
        torch = _torch()
        self._keep = (rowptr, colval, nzval)  # the 'N'/'T' operators read these live
        self.h = vp()
        L.check(L.lib.madipm_spmv_create(int(m), int(n), int(nzval.numel()), _dptr(rowptr, torch.int32),
                                         _dptr(colval, torch.int32), _dptr(nzval, torch.float64),
                                         transa.encode(), int(bool(symmetric)), C.byref(self.h)),
                "madipm_spmv_create")
        self.transa, self.symmetric = transa, bool(symmetric)

    @property
    def shape(self):
        m, n, z = C.c_int32(), C.c_int32(), C.c_int64()
        L.check(L.lib.madipm_spmv_size(self.h, C.byref(m), C.byref(n), C.byref(z)), "madipm_spmv_size")
        return (m.value, n.value)

    def nnz(self) -> int:
        z = C.c_int64()
        L.check(L.lib.madipm_spmv_size(self.h, None, None, C.byref(z)), "madipm_spmv_size")
        return z.value

    def mul(self, y, x, alpha: float = 1.0, beta: float = 0.0, stream=None):
        torch = _torch()
        L.check(L.lib.madipm_spmv_apply(self.h, _dptr(x, torch.float64), _dptr(y, torch.float64), float(alpha),
                                        float(beta), _stream(stream)), "madipm_spmv_apply")
        return y

    def __del__(self):
        if getattr(self, "h", None):
            L.lib.madipm_spmv_destroy(self.h)
            self.h = None


def coo_to_csr(n_rows: int, n_cols: int, Ai, Aj, Ax, sort_cols: bool = False, stream=None):
    """`MadIPM.coo_to_csr`: (Bp, Bj, Bx) device tensors, rows in input order (sort_cols: columns
    ascending within a row, cuSPARSE's layout)."""
    torch = _torch()
    nnz = Ai.numel()
    dev = Ai.device
    Bp = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    Bj = torch.empty(nnz, dtype=torch.int32, device=dev)
    Bx = torch.empty(nnz, dtype=torch.float64, device=dev)
    L.check(L.lib.madipm_coo_to_csr(int(n_rows), int(n_cols), nnz, _dptr(Ai, torch.int32), _dptr(Aj, torch.int32),
                                    _dptr(Ax, torch.float64), _dptr(Bp), _dptr(Bj), _dptr(Bx), int(bool(sort_cols)),
                                    _stream(stream)), "madipm_coo_to_csr")
    return Bp, Bj, Bx


def build_normal_system(n_rows: int, n_cols: int, Jtp, Jtj):
    """`MadIPM.build_normal_system` (host): (Cp, Cj) of tril(J J') as a lower CSC, 0-based int32."""
    Jtp = np.ascontiguousarray(Jtp, np.int32)
    Jtj = np.ascontiguousarray(Jtj, np.int32)
    Cp = np.zeros(n_rows + 1, np.int32)
    nnz = C.c_int64()
    L.check(L.lib.madipm_build_normal_system(int(n_rows), int(n_cols), L.ptr(Jtp, C.c_int32), L.ptr(Jtj, C.c_int32),
                                             L.ptr(Cp, C.c_int32), None, 0, C.byref(nnz)), "madipm_build_normal_system")
    Cj = np.zeros(max(1, nnz.value), np.int32)
    L.check(L.lib.madipm_build_normal_system(int(n_rows), int(n_cols), L.ptr(Jtp, C.c_int32), L.ptr(Jtj, C.c_int32),
                                             L.ptr(Cp, C.c_int32), L.ptr(Cj, C.c_int32), Cj.size, C.byref(nnz)),
            "madipm_build_normal_system")
    return Cp, Cj[:nnz.value]


def assemble_normal_system(n_rows: int, n_cols: int, Jtp, Jtj, Jtx, Cp, Cj, Cx, Dx, stream=None):
    """`MadIPM.assemble_normal_system!`: Cx of A diag(Dx) A' on the pattern (Cp, Cj), device arrays."""
    torch = _torch()
    L.check(L.lib.madipm_assemble_normal_system(int(n_rows), int(n_cols), _dptr(Jtp, torch.int32),
                                                _dptr(Jtj, torch.int32), _dptr(Jtx, torch.float64),
                                                _dptr(Cp, torch.int32), _dptr(Cj, torch.int32),
                                                _dptr(Cx, torch.float64), _dptr(Dx, torch.float64), _stream(stream)),
            "madipm_assemble_normal_system")
    return Cx


def fill_structure(n_rows: int, Ap, Aj, rows, cols, stream=None):
    """`fill_structure!(A::CSR, rows, cols)`: COO structure of a CSR matrix."""
    torch = _torch()
    L.check(L.lib.madipm_csr_fill_structure(int(n_rows), _dptr(Ap, torch.int32), _dptr(Aj, torch.int32),
                                            _dptr(rows, torch.int32), _dptr(cols, torch.int32), _stream(stream)),
            "madipm_csr_fill_structure")
    return rows, cols


def qp_obj(H: MadIPMOperator, c, c0: float, x, v, stream=None) -> float:
    """`NLPModels.obj(qp, x)` = c0 + c'x + (Hx)'x/2 (v receives Hx)."""
    torch = _torch()
    work = torch.empty(513, dtype=torch.float64, device=x.device)
    out = C.c_double()
    L.check(L.lib.madipm_qp_obj(H.h, _dptr(c, torch.float64), float(c0), _dptr(x, torch.float64),
                                _dptr(v, torch.float64), x.numel(), _dptr(work), C.byref(out), _stream(stream)),
            "madipm_qp_obj")
    return out.value


def qp_grad(H: MadIPMOperator, c, x, g, stream=None):
    """`NLPModels.grad!(qp, x, g)`: g = Hx + c."""
    torch = _torch()
    L.check(L.lib.madipm_qp_grad(H.h, _dptr(c, torch.float64), _dptr(x, torch.float64), _dptr(g, torch.float64),
                                 x.numel(), _stream(stream)), "madipm_qp_grad")
    return g


_RULES = {"conservative": 0, "adaptive": 1, "mehrotra": 2}


def update_step(rule: str, tau: float, mu: float, x_lr, xl_r, zl_r, dx_lr, dzl, x_ur, xu_r, zu_r, dx_ur, dzu,
                stream=None) -> dict:
    """update_step!(rule, solver) (kernels.jl:291-358) on device vectors over the bounded coordinates:
    rule "conservative" (tau), "adaptive" (tau_min = tau, with mu), "mehrotra" (gamma_f = tau).
    Returns alpha_p, alpha_d, the four max ratios and their 0-based argmin indices (-1 = init)."""
    f64 = _torch().float64
    nlb, nub = int(x_lr.numel()), int(x_ur.numel())
    r = StepResult()
    ptrs = [_dptr(t, f64) for t in (x_lr, xl_r, zl_r, dx_lr, dzl, x_ur, xu_r, zu_r, dx_ur, dzu)]
    L.check(L.lib.madipm_update_step(_RULES[rule], float(tau), float(mu), nlb, nub, *ptrs, C.byref(r),
                                     _stream(stream)), "update_step!")
    return {k: getattr(r, k) for k, _ in StepResult._fields_}
