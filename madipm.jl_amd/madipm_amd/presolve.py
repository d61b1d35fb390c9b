"""`presolve_qp` (src/utils.jl:319-343) — host preprocessing before the GPU solve.

The reference delegates to `QuadraticModels.presolve` (QuadraticModels.jl 0.9.14, un-vendored [EXT])
and returns `(presolved_qp, flag)`, `flag = false` (and the original qp) when the presolve finds the
problem infeasible / unbounded or removes every variable.  This restates the published basic
presolve operations of that package, applied to a fixed point:

* fixed variables (lvar == uvar): substituted out — their column moves into the row bounds, their
  objective and Hessian terms into c0 / c;
* empty rows: dropped (infeasible if 0 is outside [lcon, ucon]);
* singleton rows a x_j in [l, u]: turned into bounds on x_j and dropped (infeasible when the
  bounds cross);
* empty columns of an LP-like variable (no A entries, no H entries): fixed at the bound the cost
  points to (unbounded when that bound is infinite);
* free rows (lcon = -Inf, ucon = +Inf): dropped (multiplier 0);
* unconstrained variables with a diagonal Hessian entry only (no A entries, H_jj > 0): fixed at the
  minimiser clip(-c_j / H_jj, l_j, u_j);
* free linear column singletons in an equality row (x_j free, no H entries, one A entry a_ij, row i
  an equality with right-hand side b_i): x_j = (b_i - sum_k a_ik x_k) / a_ij is substituted into the
  objective (c0 += c_j b_i / a_ij, c_k -= c_j a_ik / a_ij), row i and column j are dropped, and the
  row's multiplier is recovered exactly as y_i = -c_j / a_ij (MadNLP's sign convention
  c + H x + A' y - zl + zu = 0).

Which reductions QuadraticModels.presolve 0.9.14 applies, and in which order, is [EXT, unverified]:
the package is not vendored and cannot be run here.  The list above restates the operations its
published presolve module is built from (remove_ifix!, empty_rows!, singleton_rows!, free_rows!,
unconstrained_variables!, free_linear_singleton_columns!), to a fixed point; parity is pinned on
optimal objectives (the presolved problem's optimum plus c0 equals the original's:
tests/test_host_cpu.py presolve tests, AFIRO's netlib optimum).

`postsolve(pre, x, y, zl, zu)` maps a solution of the presolved problem back to the original
variables and constraints (removed rows get multiplier 0, removed singleton rows the multiplier
of the bound they became).  The multipliers of the presolved problem are kept for the surviving
rows.  Host-side numpy: this runs once per problem, before the per-iteration hot path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .qp import QuadraticModel

INF = math.inf


@dataclass
class PresolveInfo:
    """What postsolve needs (QuadraticModels' PresolvedQuadraticModel state, restated)."""
    n: int
    m: int
    keep_var: np.ndarray              # original indices of the surviving variables
    keep_con: np.ndarray              # original indices of the surviving rows
    xfix: np.ndarray                  # value of every original variable removed (NaN if kept)
    singleton_rows: list = field(default_factory=list)  # (row, var, a) turned into bounds
    free_singletons: list = field(default_factory=list)  # (row, var, a_ij, b_i, cols, vals, c_j), removal order
    status: str = "ok"                # "ok" | "infeasible" | "unbounded" | "empty"


def presolve_qp(qp: QuadraticModel):
    """Returns (new_qp, flag) like the reference: flag False -> the original qp is returned."""
    new, info = presolve(qp)
    if info.status != "ok":
        return qp, False
    new.meta = dict(new.meta, presolve=info)
    return new, True


def presolve(qp: QuadraticModel):
    n, m = qp.nvar, qp.ncon
    lvar, uvar = qp.lvar.copy(), qp.uvar.copy()
    lcon, ucon = qp.lcon.copy(), qp.ucon.copy()
    # every reduction below is stated for a minimisation (the minimiser of an unconstrained variable,
    # the bound an empty column's cost points to, y_i = -c_j / a_ij): a MAX model is reduced as
    # min -f and the objective is negated back at the end; recovered multipliers are those of min -f,
    # MadNLP's internal convention (the solver's multipliers of a MAX model are too)
    sg = 1.0 if qp.minimize else -1.0
    c = sg * qp.c
    c0 = sg * float(qp.c0)
    Ar, Ac, Av = qp.Arows.copy(), qp.Acols.copy(), qp.Avals.copy()
    Hr, Hc, Hv = qp.Hrows.copy(), qp.Hcols.copy(), sg * qp.Hvals
    var_alive = np.ones(n, bool)
    con_alive = np.ones(m, bool)
    xfix = np.full(n, np.nan)
    singles = []
    fsing = []
    status = "ok"
    tol = 1e-12

    def fix_vars(js, vals):
        """substitute x_j = v: A columns -> row bounds, H -> c / c0, c_j v -> c0"""
        nonlocal c0, Av, Hv
        if len(js) == 0:
            return
        v = np.zeros(n)
        v[js] = vals
        mask = np.zeros(n, bool)
        mask[js] = True
        xfix[js] = vals
        # constraints: A x with x_j = v_j moves to the bounds
        ea = mask[Ac] & con_alive[Ar]
        shift = np.zeros(m)
        np.add.at(shift, Ar[ea], Av[ea] * v[Ac[ea]])
        lcon[:] -= shift
        ucon[:] -= shift
        Av = np.where(mask[Ac], 0.0, Av)
        # objective: c_j v_j + 1/2 v' H v + (H v) for the free variables
        c0 += float(np.dot(c[js], vals))
        hm = mask[Hr] | mask[Hc]
        for k in np.flatnonzero(hm):
            i, j, h = Hr[k], Hc[k], Hv[k]
            if mask[i] and mask[j]:
                c0 += (0.5 if i == j else 1.0) * h * v[i] * v[j]
            elif mask[j]:
                c[i] += h * v[j]
            else:
                c[j] += h * v[i]
        Hv = np.where(hm, 0.0, Hv)
        var_alive[js] = False

    changed = True
    while changed and status == "ok":
        changed = False
        # fixed variables
        fx = np.flatnonzero(var_alive & (lvar == uvar))
        if len(fx):
            fix_vars(fx, lvar[fx])
            changed = True
        live_e = (Av != 0.0) & var_alive[Ac] & con_alive[Ar]
        rcount = np.bincount(Ar[live_e], minlength=m)
        # empty rows
        er = np.flatnonzero(con_alive & (rcount == 0))
        if len(er):
            if np.any((lcon[er] > tol) | (ucon[er] < -tol)):
                status = "infeasible"
                break
            con_alive[er] = False
            changed = True
        # singleton rows -> bounds
        sr = np.flatnonzero(con_alive & (rcount == 1))
        if len(sr):
            srmask = np.zeros(m, bool)
            srmask[sr] = True
            for k in np.flatnonzero(live_e & srmask[Ar]):
                i, j, a = Ar[k], Ac[k], Av[k]
                lo, hi = (lcon[i] / a, ucon[i] / a) if a > 0 else (ucon[i] / a, lcon[i] / a)
                lvar[j] = max(lvar[j], lo)
                uvar[j] = min(uvar[j], hi)
                if lvar[j] > uvar[j] + tol * max(1.0, abs(lvar[j])):
                    status = "infeasible"
                    break
                if abs(uvar[j] - lvar[j]) <= tol * max(1.0, abs(lvar[j])):
                    uvar[j] = lvar[j]
                singles.append((int(i), int(j), float(a)))
                con_alive[i] = False
            changed = True
        # free rows: no bound on either side
        fr = np.flatnonzero(con_alive & np.isneginf(lcon) & np.isposinf(ucon))
        if len(fr):
            con_alive[fr] = False
            changed = True
        # empty columns (no A, no H): fix at the bound the cost points to
        live_e = (Av != 0.0) & var_alive[Ac] & con_alive[Ar]
        ccount = np.bincount(Ac[live_e], minlength=n)
        hlive = (Hv != 0.0) & var_alive[Hr] & var_alive[Hc]
        hcount = np.bincount(np.concatenate([Hr[hlive], Hc[hlive]]), minlength=n)
        ec = np.flatnonzero(var_alive & (ccount == 0) & (hcount == 0) & (lvar < uvar))
        if len(ec):
            vals = np.where(c[ec] > 0, lvar[ec], np.where(c[ec] < 0, uvar[ec],
                            np.where(np.isfinite(lvar[ec]), lvar[ec], np.where(np.isfinite(uvar[ec]), uvar[ec], 0.0))))
            if not np.all(np.isfinite(vals)):
                status = "unbounded"
                break
            fix_vars(ec, vals)
            changed = True
            continue
        # unconstrained variables with only a diagonal Hessian entry: fixed at their minimiser
        hdiag = np.zeros(n)
        offd = np.zeros(n, bool)
        dmask = hlive & (Hr == Hc)
        np.add.at(hdiag, Hr[dmask], Hv[dmask])
        omask = hlive & (Hr != Hc)
        offd[Hr[omask]] = True
        offd[Hc[omask]] = True
        uc = np.flatnonzero(var_alive & (ccount == 0) & ~offd & (hdiag > 0) & (lvar < uvar))
        if len(uc):
            fix_vars(uc, np.clip(-c[uc] / hdiag[uc], lvar[uc], uvar[uc]))
            changed = True
            continue
        # free linear column singletons in equality rows
        cand = np.flatnonzero(var_alive & (ccount == 1) & (hcount == 0) & np.isneginf(lvar) & np.isposinf(uvar))
        if len(cand):
            ecol = {}
            for k in np.flatnonzero(live_e & (ccount[Ac] == 1)):
                ecol[int(Ac[k])] = k
            le = np.flatnonzero(live_e)
            le = le[np.argsort(Ar[le], kind="stable")]
            rptr = np.searchsorted(Ar[le], np.arange(m + 1))
            used_rows = set()
            for j in cand:
                k = ecol.get(int(j))
                if k is None:
                    continue
                i, a = int(Ar[k]), float(Av[k])
                if i in used_rows or not con_alive[i] or lcon[i] != ucon[i] or not np.isfinite(lcon[i]) or abs(a) <= tol:
                    continue
                row = le[rptr[i]:rptr[i + 1]]
                row = row[(Ac[row] != j) & var_alive[Ac[row]]]
                cols, vals = Ac[row].copy(), Av[row].copy()
                cj, bi = float(c[j]), float(lcon[i])
                c0 += cj * bi / a
                np.add.at(c, cols, -cj * vals / a)
                fsing.append((i, int(j), a, bi, cols, vals, cj))
                con_alive[i] = False
                var_alive[j] = False
                xfix[j] = np.nan
                used_rows.add(i)
                changed = True
    if status == "ok" and not var_alive.any():
        status = "empty"
    keep_var = np.flatnonzero(var_alive)
    keep_con = np.flatnonzero(con_alive)
    info = PresolveInfo(n=n, m=m, keep_var=keep_var, keep_con=keep_con, xfix=xfix, singleton_rows=singles,
                        free_singletons=fsing, status=status)
    if status != "ok":
        return qp, info
    vmap = np.full(n, -1, np.int64)
    vmap[keep_var] = np.arange(len(keep_var))
    cmap = np.full(m, -1, np.int64)
    cmap[keep_con] = np.arange(len(keep_con))
    ea = (Av != 0.0) & var_alive[Ac] & con_alive[Ar]
    eh = (Hv != 0.0) & var_alive[Hr] & var_alive[Hc]
    new = QuadraticModel(
        c=sg * c[keep_var], c0=sg * c0, Hrows=vmap[Hr[eh]], Hcols=vmap[Hc[eh]], Hvals=sg * Hv[eh],
        Arows=cmap[Ar[ea]], Acols=vmap[Ac[ea]], Avals=Av[ea],
        lcon=lcon[keep_con], ucon=ucon[keep_con], lvar=lvar[keep_var], uvar=uvar[keep_var],
        x0=np.clip(qp.x0[keep_var], lvar[keep_var], uvar[keep_var]), y0=qp.y0[keep_con],
        minimize=qp.minimize, name=qp.name + "_presolved")
    return new, info


def postsolve(info: PresolveInfo, x, y=None):
    """Original-space primal x (and row multipliers y, 0 for dropped rows)."""
    xo = info.xfix.copy()
    xo[info.keep_var] = x
    yo = np.zeros(info.m)
    if y is not None:
        yo[info.keep_con] = y
    for i, j, a, b, cols, vals, cj in reversed(info.free_singletons):  # later removals are known first
        xo[j] = (b - float(np.dot(vals, xo[cols]))) / a
        yo[i] = -cj / a
    return xo, yo
