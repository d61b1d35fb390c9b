"""MPS / QPS reader (host side) producing a QuadraticModel.

Stands in for QPSReader.jl (`readqps`, used by scripts/common.jl:21-36 → `QuadraticModel(qpdat)`),
which is an un-vendored dependency.  Supports the sections the reference's benchmark instances
use: NAME, OBJSENSE, ROWS, COLUMNS (integer MARKERs are read as continuous: LP relaxation),
RHS (objective RHS = -c0), RANGES, BOUNDS (UP LO FX FR MI PL BV LI UI), QUADOBJ/QMATRIX, ENDATA.
Reads plain text, `.gz` and `.bz2`.
"""
from __future__ import annotations

import bz2
import gzip
import math

import numpy as np

from .qp import QuadraticModel

INF = math.inf


def _open(path):
    if str(path).endswith(".gz"):
        return gzip.open(path, "rt")
    if str(path).endswith(".bz2"):
        return bz2.open(path, "rt")
    return open(path, "r")


def read_mps(path) -> QuadraticModel:
    with _open(path) as fh:
        return parse_mps(fh.read())


def parse_mps(text: str) -> QuadraticModel:
    name = ""
    section = None
    obj_row = None
    minimize = True
    row_index: dict[str, int] = {}
    row_type: list[str] = []
    col_index: dict[str, int] = {}
    col_int: list[bool] = []
    A_r, A_c, A_v = [], [], []
    cost: dict[int, float] = {}
    rhs: dict[int, float] = {}
    rng: dict[int, float] = {}
    c0 = 0.0
    lb: dict[int, float] = {}
    ub: dict[int, float] = {}
    Q: dict[tuple, float] = {}
    integer = False

    def col(nm):
        j = col_index.get(nm)
        if j is None:
            j = len(col_index)
            col_index[nm] = j
            col_int.append(integer)
        return j

    for raw in text.splitlines():
        if not raw.strip() or raw.startswith("*"):
            continue
        if not raw[0].isspace():
            tok = raw.split()
            head = tok[0].upper()
            if head == "NAME":
                name = tok[1] if len(tok) > 1 else ""
                section = None
            elif head == "OBJSENSE":
                section = "OBJSENSE"
                if len(tok) > 1:
                    minimize = tok[1].upper() not in ("MAX", "MAXIMIZE")
            elif head in ("ROWS", "COLUMNS", "RHS", "RANGES", "BOUNDS", "QUADOBJ", "QMATRIX",
                          "QSECTION", "ENDATA"):
                section = head
                if head == "ENDATA":
                    break
            else:
                raise ValueError(f"unknown MPS section {head!r}")
            continue
        tok = raw.split()
        if section == "OBJSENSE":
            minimize = tok[0].upper() not in ("MAX", "MAXIMIZE")
        elif section == "ROWS":
            t, nm = tok[0].upper(), tok[1]
            if t == "N":
                if obj_row is None:
                    obj_row = nm
                continue
            row_index[nm] = len(row_type)
            row_type.append(t)
        elif section == "COLUMNS":
            if len(tok) >= 3 and tok[1].strip("'").upper() == "MARKER":
                integer = tok[2].strip("'").upper() == "INTORG"
                continue
            j = col(tok[0])
            for k in range(1, len(tok) - 1, 2):
                rn, val = tok[k], float(tok[k + 1])
                if rn == obj_row:
                    cost[j] = cost.get(j, 0.0) + val
                elif rn in row_index:
                    A_r.append(row_index[rn]); A_c.append(j); A_v.append(val)
        elif section in ("RHS", "RANGES"):
            start = 1 if len(tok) % 2 == 1 else 0
            for k in range(start, len(tok) - 1, 2):
                rn, val = tok[k], float(tok[k + 1])
                if section == "RHS":
                    if rn == obj_row:
                        c0 = -val
                    else:
                        rhs[row_index[rn]] = val
                else:
                    rng[row_index[rn]] = val
        elif section == "BOUNDS":
            bt = tok[0].upper()
            cn = tok[2] if len(tok) >= 3 else tok[1]
            j = col(cn)
            val = float(tok[3]) if len(tok) >= 4 else (float(tok[2]) if bt not in ("FR", "MI", "PL", "BV") and len(tok) == 3 else 0.0)
            if bt == "UP":
                ub[j] = val
                if val < 0 and lb.get(j, 0.0) == 0.0:
                    lb[j] = -INF
            elif bt == "LO":
                lb[j] = val
            elif bt == "FX":
                lb[j] = val; ub[j] = val
            elif bt == "FR":
                lb[j] = -INF; ub[j] = INF
            elif bt == "MI":
                lb[j] = -INF
            elif bt == "PL":
                ub[j] = INF
            elif bt == "BV":
                lb[j] = 0.0; ub[j] = 1.0
            elif bt == "LI":
                lb[j] = val
            elif bt == "UI":
                ub[j] = val
            else:
                raise ValueError(f"unknown bound type {bt}")
        elif section in ("QUADOBJ", "QMATRIX", "QSECTION"):
            i, j, val = col(tok[0]), col(tok[1]), float(tok[2])
            a, b = max(i, j), min(i, j)
            if section == "QMATRIX" and i < j:
                continue          # QMATRIX lists both triangles
            Q[(a, b)] = Q.get((a, b), 0.0) + val

    n, m = len(col_index), len(row_type)
    c = np.zeros(n)
    for j, v in cost.items():
        c[j] = v
    lvar = np.zeros(n)
    uvar = np.full(n, INF)
    for j, v in lb.items():
        lvar[j] = v
    for j, v in ub.items():
        uvar[j] = v
    lcon = np.empty(m)
    ucon = np.empty(m)
    for i, t in enumerate(row_type):
        b = rhs.get(i, 0.0)
        if t == "E":
            lcon[i] = ucon[i] = b
            if i in rng:
                r = rng[i]
                if r > 0:
                    ucon[i] = b + abs(r)
                elif r < 0:
                    lcon[i] = b - abs(r)
        elif t == "L":
            lcon[i], ucon[i] = -INF, b
            if i in rng:
                lcon[i] = b - abs(rng[i])
        elif t == "G":
            lcon[i], ucon[i] = b, INF
            if i in rng:
                ucon[i] = b + abs(rng[i])
        else:
            raise ValueError(f"unknown row type {t}")
    if Q:
        keys = list(Q.keys())
        Hr = np.array([k[0] for k in keys], np.int64)
        Hc = np.array([k[1] for k in keys], np.int64)
        Hv = np.array([Q[k] for k in keys])
    else:
        Hr = Hc = np.zeros(0, np.int64)
        Hv = np.zeros(0)
    qp = QuadraticModel(c=c, Hrows=Hr, Hcols=Hc, Hvals=Hv,
                        Arows=np.asarray(A_r, np.int64), Acols=np.asarray(A_c, np.int64),
                        Avals=np.asarray(A_v, float), lcon=lcon, ucon=ucon, lvar=lvar, uvar=uvar,
                        c0=c0, minimize=minimize, name=name)
    qp.meta["integer"] = np.asarray(col_int, bool)
    qp.meta["col_names"] = list(col_index.keys())
    qp.meta["row_names"] = list(row_index.keys())
    return qp
