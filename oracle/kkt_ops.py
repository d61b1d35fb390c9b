"""CPU restatement of the reference's array-type methods — TEST INFRASTRUCTURE ONLY (the checker of
csrc/kkt.hip; never imported by the product).

Each function restates the reference's CPU method (0-based here; the reference is 1-based) with
the same loop order and floating-point association, so the HIP kernels that follow the same order
can be compared bit for bit:

    transfer            MadNLP.transfer! [EXT; CPU loop dest[map[k]] += src[k]], GPU cuda_wrapper.jl:4-24
    compress_jacobian   src/KKT/normalkkt.jl:163-172
    coo_to_csr          src/utils.jl:158-201
    build_normal_system src/utils.jl:209-274
    assemble_normal_system  src/utils.jl:276-308
    operator_matrix     cuda_wrapper.jl:62-68 (mat = symmetric ? tril(A,-1) + A' : A)
    fill_structure      ext/MadIPMCUDAExt/MadIPMCUDAExt.jl:15-21
    qp_obj / qp_grad    ext/MadIPMCUDAExt/MadIPMCUDAExt.jl:34-45
Pure-Python loops: for the small cases of the tests only.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def transfer(ndest, src, map_):
    """fill!(dest, 0); for k: dest[map[k]] += src[k]."""
    dest = [0.0] * ndest
    for k in range(len(map_)):
        dest[map_[k]] += float(src[k])
    return np.array(dest)


def compress_jacobian(AV, n_slack, csr_map):
    """normalkkt.jl:163-172: A.V[end-n_slack+1:end] .= -1; AT.nzval[i] = A.V[A_csr_map[i]]."""
    AV = np.array(AV, np.float64)
    if n_slack:
        AV[len(AV) - n_slack:] = -1.0
    return AV, AV[np.asarray(csr_map)].copy()


def coo_to_csr(n_rows, n_cols, Ai, Aj, Ax):
    """utils.jl:158-201: counting sort by row, entries of a row in input order, no duplicate merge."""
    nnz = len(Ai)
    Bp = [0] * (n_rows + 1)
    Bj = [0] * nnz
    Bx = [0.0] * nnz
    for k in range(nnz):
        Bp[Ai[k]] += 1
    cumsum = 0
    for i in range(n_rows):
        tmp = Bp[i]
        Bp[i] = cumsum
        cumsum += tmp
    Bp[n_rows] = nnz
    for k in range(nnz):
        i = Ai[k]
        dest = Bp[i]
        Bj[dest] = int(Aj[k])
        Bx[dest] = float(Ax[k])
        Bp[i] += 1
    last = 0
    for i in range(n_rows + 1):
        tmp = Bp[i]
        Bp[i] = last
        last = tmp
    return np.array(Bp, np.int32), np.array(Bj, np.int32), np.array(Bx)


def build_normal_system(n_rows, n_cols, Jtp, Jtj):
    """utils.jl:209-274: for row i, the rows j >= i (ascending) sharing a column with row i."""
    Cp = [0] * (n_rows + 1)
    Cj = []
    xb = bytearray(n_cols)
    for i in range(n_rows):
        for c in range(Jtp[i], Jtp[i + 1]):
            xb[Jtj[c]] = 1
        for j in range(i, n_rows):
            for c in range(Jtp[j], Jtp[j + 1]):
                if xb[Jtj[c]] == 1:
                    Cj.append(j)
                    break
        for c in range(Jtp[i], Jtp[i + 1]):
            xb[Jtj[c]] = 0
        Cp[i + 1] = len(Cj)
    return np.array(Cp, np.int32), np.array(Cj, np.int32)


def assemble_normal_system(n_rows, n_cols, Jtp, Jtj, Jtx, Cp, Cj, Dx):
    """utils.jl:276-308: buffer[k] = Jtx[i,k] * Dx[k]; Cx[c] = sum over row j's entries (storage
    order) of buffer[k] * Jtx[j,k]."""
    buffer = [0.0] * n_cols
    Cx = [0.0] * len(Cj)
    for i in range(n_rows):
        for c in range(Jtp[i], Jtp[i + 1]):
            j = Jtj[c]
            buffer[j] = float(Jtx[c]) * float(Dx[j])
        for c in range(Cp[i], Cp[i + 1]):
            j = Cj[c]
            acc = 0.0
            for d in range(Jtp[j], Jtp[j + 1]):
                acc += buffer[Jtj[d]] * float(Jtx[d])
            Cx[c] = acc
        for c in range(Jtp[i], Jtp[i + 1]):
            buffer[Jtj[c]] = 0.0
    return np.array(Cx)


def operator_matrix(m, n, Ap, Aj, Ax, transa="N", symmetric=False):
    """The matrix MadIPMOperator applies (cuda_wrapper.jl:62-68), as scipy CSR."""
    A = sp.csr_matrix((np.asarray(Ax, np.float64), np.asarray(Aj), np.asarray(Ap)), shape=(m, n))
    if symmetric and A.nnz > 0:
        return (sp.tril(A, -1) + A.T).tocsr()
    return (A.T if transa == "T" else A).tocsr()


def fill_structure(n_rows, Ap, Aj):
    rows = np.zeros(Ap[n_rows], np.int32)
    for i in range(n_rows):
        rows[Ap[i]:Ap[i + 1]] = i
    return rows, np.asarray(Aj, np.int32).copy()


def qp_obj(Hmat, c, c0, x):
    v = Hmat @ x
    return c0 + float(np.dot(c, x)) + float(np.dot(v, x)) / 2


def qp_grad(Hmat, c, x):
    return Hmat @ x + c
