"""QuadraticModel container and QP reformulations (host side).

Mirrors the data the reference hands to `MPCSolver` (QuadraticModels.QuadraticModel: `data.c`,
`data.c0`, lower-triangular COO `data.H`, COO `data.A`, `meta.lvar/uvar/lcon/ucon/x0/y0/minimize`)
with 0-based indices.  `standard_form_qp` restates src/utils.jl:373-505.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

INF = math.inf


@dataclass
class QuadraticModel:
    """min c0 + c'x + 1/2 x'Hx  s.t. lcon <= Ax <= ucon, lvar <= x <= uvar.

    H is given by its lower triangle (row >= col) in COO form, as NLPModels' hess_coord."""
    c: np.ndarray
    Hrows: np.ndarray
    Hcols: np.ndarray
    Hvals: np.ndarray
    Arows: np.ndarray
    Acols: np.ndarray
    Avals: np.ndarray
    lcon: np.ndarray
    ucon: np.ndarray
    lvar: np.ndarray
    uvar: np.ndarray
    c0: float = 0.0
    x0: np.ndarray | None = None
    y0: np.ndarray | None = None
    minimize: bool = True
    name: str = ""
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        self.c = np.ascontiguousarray(self.c, dtype=np.float64)
        for k in ("Hrows", "Hcols", "Arows", "Acols"):
            setattr(self, k, np.ascontiguousarray(getattr(self, k), dtype=np.int64))
        for k in ("Hvals", "Avals", "lcon", "ucon", "lvar", "uvar"):
            setattr(self, k, np.ascontiguousarray(getattr(self, k), dtype=np.float64))
        n, m = len(self.c), len(self.lcon)
        if self.x0 is None:
            self.x0 = np.zeros(n)
        if self.y0 is None:
            self.y0 = np.zeros(m)
        self.x0 = np.ascontiguousarray(self.x0, dtype=np.float64)
        self.y0 = np.ascontiguousarray(self.y0, dtype=np.float64)
        if not (len(self.lvar) == len(self.uvar) == n and len(self.ucon) == m):
            raise ValueError("inconsistent QuadraticModel dimensions")
        if len(self.Hrows) and np.any(self.Hrows < self.Hcols):
            raise ValueError("H must be given by its lower triangle (row >= col)")
        if len(self.Arows) and (self.Arows.max() >= m or self.Acols.max() >= n or
                                self.Arows.min() < 0 or self.Acols.min() < 0):
            raise ValueError("A index out of range")

    @property
    def nvar(self) -> int:
        return len(self.c)

    @property
    def ncon(self) -> int:
        return len(self.lcon)

    @property
    def nnzj(self) -> int:
        return len(self.Avals)

    @property
    def nnzh(self) -> int:
        return len(self.Hvals)


def simple_lp() -> QuadraticModel:
    """The reference test problem `simple_lp` (test/runtests.jl:29-60): min x1+x2, x1+x2 = 1, x >= 0."""
    return QuadraticModel(
        c=np.ones(2), Hrows=[], Hcols=[], Hvals=[],
        Arows=[0, 0], Acols=[0, 1], Avals=[1.0, 1.0],
        lcon=[1.0], ucon=[1.0], lvar=[0.0, 0.0], uvar=[INF, INF],
        c0=0.0, x0=np.ones(2), name="simpleLP")


def standard_form_qp(qp: QuadraticModel) -> QuadraticModel:
    """Restates `standard_form_qp` (src/utils.jl:373-505), 0-based.

    Introduces slacks s = Ax for inequality rows (l.381-385, 430-436) and moves finite upper
    bounds of range-bounded x / s into equality rows x + w = xu (l.388-416, 437-447)."""
    n, m = qp.nvar, qp.ncon
    lvar, uvar, lcon, ucon = qp.lvar, qp.uvar, qp.lcon, qp.ucon
    ind_ineq = [i for i in range(m) if lcon[i] < ucon[i]]                      # l.381-384
    ns = len(ind_ineq)
    ind_rng, ind_only_ub, ind_fixed, xu = [], [], [], []
    for i in range(n):                                                          # l.392-404
        if lvar[i] == uvar[i]:
            ind_fixed.append(i)
        elif -INF < lvar[i] < uvar[i] < INF:
            ind_rng.append(i)
            xu.append(uvar[i])
        elif uvar[i] < INF:
            ind_only_ub.append(i)
    for k, i in enumerate(ind_ineq):                                            # l.407-416
        if -INF < lcon[i] < ucon[i] < INF:
            ind_rng.append(k + n)
            xu.append(ucon[i])
        elif ucon[i] < INF:
            ind_only_ub.append(k + n)
    nw = len(ind_rng)
    nvar, ncon = n + ns + nw, m + nw                                            # l.420-421
    Bi, Bj, Bx = [], [], []
    for k, i in enumerate(ind_ineq):                                            # l.431-436
        Bi.append(i); Bj.append(n + k); Bx.append(-1.0)
    for k, i in enumerate(ind_rng):                                             # l.438-447
        Bi.append(m + k); Bj.append(i); Bx.append(1.0)
        Bi.append(m + k); Bj.append(k + n + ns); Bx.append(1.0)
    Arows = np.concatenate([qp.Arows, np.asarray(Bi, np.int64)])
    Acols = np.concatenate([qp.Acols, np.asarray(Bj, np.int64)])
    Avals = np.concatenate([qp.Avals, np.asarray(Bx, np.float64)])
    lcon_ = np.zeros(ncon)
    ucon_ = np.zeros(ncon)
    for i in range(m):                                                          # l.455-465
        if lcon[i] < ucon[i]:
            lcon_[i] = 0.0
            ucon_[i] = 0.0
        else:
            lcon_[i] = lcon[i]
            ucon_[i] = ucon[i]
    for k in range(nw):                                                         # l.466-469
        lcon_[m + k] = xu[k]
        ucon_[m + k] = xu[k]
    ineq = np.asarray(ind_ineq, np.int64)
    lvar_ = np.concatenate([lvar, lcon[ineq], np.zeros(nw)])                   # l.471-476
    uvar_ = np.concatenate([uvar, ucon[ineq], np.full(nw, INF)])
    uvar_[np.asarray(ind_rng, np.int64)] = INF
    uvar_[np.asarray(ind_fixed, np.int64)] = uvar[np.asarray(ind_fixed, np.int64)]
    return QuadraticModel(
        c=np.concatenate([qp.c, np.zeros(ns + nw)]),
        Hrows=qp.Hrows.copy(), Hcols=qp.Hcols.copy(), Hvals=qp.Hvals.copy(),
        Arows=Arows, Acols=Acols, Avals=Avals,
        lcon=lcon_, ucon=ucon_, lvar=lvar_, uvar=uvar_, c0=qp.c0,
        x0=np.concatenate([qp.x0, np.zeros(ns + nw)]),
        y0=np.concatenate([qp.y0, np.zeros(nw)]),
        minimize=qp.minimize, name=qp.name)


def scale_qp(qp: QuadraticModel, iters: int = 20, tol: float = 1e-8) -> QuadraticModel:
    """Ruiz equilibration of A (scripts/common.jl:38-100 uses HSL mc77, absent here; this is
    the published Ruiz iteration: Dr_i <- sqrt(max_j |A_ij|), Dc_j <- sqrt(max_i |A_ij|)).

    As scale_qp, returns As = Dr^-1 A Dc^-1 with the reference's bound/cost transforms."""
    m, n = qp.ncon, qp.nvar
    if qp.nnzj == 0:
        return qp
    Dr = np.ones(m)
    Dc = np.ones(n)
    r, c, v = qp.Arows, qp.Acols, np.abs(qp.Avals)
    for _ in range(iters):
        a = v / (Dr[r] * Dc[c])
        rmax = np.zeros(m); np.maximum.at(rmax, r, a)
        cmax = np.zeros(n); np.maximum.at(cmax, c, a)
        rmax[rmax == 0] = 1.0
        cmax[cmax == 0] = 1.0
        Dr *= np.sqrt(rmax)
        Dc *= np.sqrt(cmax)
        if max(np.max(np.abs(1 - rmax)), np.max(np.abs(1 - cmax))) < tol:
            break
    # _scale_coo!(H, Dc, Dc), _scale_coo!(A, Dr, Dc) (scripts/common.jl:38-44,70-72)
    Hv = qp.Hvals / (Dc[qp.Hrows] * Dc[qp.Hcols])
    Av = qp.Avals / (Dr[qp.Arows] * Dc[qp.Acols])
    return QuadraticModel(
        c=qp.c / Dc, Hrows=qp.Hrows, Hcols=qp.Hcols, Hvals=Hv,
        Arows=qp.Arows, Acols=qp.Acols, Avals=Av,
        lcon=qp.lcon / Dr, ucon=qp.ucon / Dr, lvar=qp.lvar * Dc, uvar=qp.uvar * Dc,
        c0=qp.c0, x0=qp.x0 * Dc, y0=qp.y0 / Dr, minimize=qp.minimize, name=qp.name,
        meta=dict(qp.meta, Dr=Dr, Dc=Dc))
