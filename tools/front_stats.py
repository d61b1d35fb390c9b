"""Front-size statistics of the K2 symbolic analysis for a benchmark config (host only)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "madipm.jl_amd"))
import numpy as np, scipy.sparse as sp
from madipm_amd import standard_form_qp
from madipm_amd.instances import ex10_standin
from madipm_amd._lib import Symbolic, default_ldl_opts

def k2_pattern(qp):
    n, m = qp.nvar, qp.ncon
    A = sp.coo_matrix((np.ones(qp.nnzj), (qp.Arows, qp.Acols)), shape=(m, n))
    K = sp.bmat([[sp.eye(n), None], [A, sp.eye(m)]]).tocsc()
    K = sp.tril(K).tocsc(); K.sort_indices(); K.sum_duplicates()
    return K

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
qp = standard_form_qp(ex10_standin(scale=scale))
K = k2_pattern(qp)
S = Symbolic(K.shape[0], K.indptr, K.indices)
info = S.info(); print(info)
first, parent, nrows = S.supernodes()
w = np.diff(first)
r = nrows
# level = height
ns = len(w); lev = np.zeros(ns, int)
for s in range(ns):
    if parent[s] >= 0: lev[parent[s]] = max(lev[parent[s]], lev[s] + 1)
for L in range(lev.max() + 1):
    sel = lev == L
    print(f"level {L:3d}: fronts {sel.sum():6d}  r max {r[sel].max():6d} mean {r[sel].mean():8.1f}  w max {w[sel].max():6d}  "
          f"big {np.sum(r[sel] > 128):5d}  L-bytes {8*np.sum(r[sel]*w[sel])/1e6:8.1f} MB  flops {np.sum([( (r[s]-np.arange(w[s]))**2 ).sum() for s in np.flatnonzero(sel)])/1e9:.2f} G")
