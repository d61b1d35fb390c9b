// Approximate minimum degree ordering on a quotient graph.
//
// Replaces the AMD ordering that the reference's linear solvers run inside their constructors
// (LDLFactorizations.jl's `ldl_analyze` uses AMD; cuDSS/MA57 use their own orderings) — SURVEY
// §8 a12.  Algorithm: Amestoy, Davis & Duff, "An approximate minimum degree ordering algorithm",
// SIAM J. Matrix Anal. Appl. 17(4), 1996: quotient graph with element absorption, mass
// elimination, approximate external degrees |Le \ Lk|, supervariable detection by hashing,
// aggressive absorption, dense-node deferral, and a final postorder of the assembly tree.
// Written for this project (host code, runs once per symbolic analysis).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "symbolic.hpp"

namespace madipm {

namespace {

inline int64_t flip(int64_t i) { return -i - 2; }

int64_t reset_marks(int64_t mark, int64_t lemax, std::vector<int64_t>& w, int n) {
  if (mark < 2 || mark + lemax < 0) {
    for (int k = 0; k < n; ++k)
      if (w[k] != 0) w[k] = 1;
    mark = 2;
  }
  return mark;
}

// Non-recursive depth-first postorder of the tree rooted at j (children lists head/next).
int64_t tree_dfs(int j, int64_t k, std::vector<int32_t>& head, const std::vector<int32_t>& next,
                 std::vector<int32_t>& post, std::vector<int32_t>& stack) {
  int64_t top = 0;
  stack[0] = j;
  while (top >= 0) {
    int p = stack[top];
    int i = head[p];
    if (i == -1) {
      --top;
      post[k++] = p;
    } else {
      head[p] = next[i];
      stack[++top] = i;
    }
  }
  return k;
}

}  // namespace

bool amd_order(int n, const std::vector<int64_t>& Ap, const std::vector<int32_t>& Ai,
               std::vector<int32_t>& perm, double dense_alpha, const std::atomic<double>* cap) {
  perm.assign(n, 0);
  if (n == 0) return true;
  const int64_t nz = Ap[n];
  int64_t dense = (int64_t)std::max(16.0, dense_alpha * std::sqrt((double)n));
  dense = std::min<int64_t>(n - 2, dense);
  if (dense_alpha < 0) dense = n;  // no dense-node deferral
  const int64_t nzmax = nz + nz / 5 + 2 * (int64_t)n + 64;
  std::vector<int32_t> iw(nzmax);
  std::vector<int64_t> pe(n + 1);
  std::vector<int32_t> len(n + 1), nv(n + 1), next(n + 1), head(n + 1), elen(n + 1), last(n + 1),
      hhead(n + 1);
  std::vector<int64_t> degree(n + 1), w(n + 1);

  for (int i = 0; i < n; ++i) {
    len[i] = (int32_t)(Ap[i + 1] - Ap[i]);
    pe[i] = Ap[i];
  }
  std::copy(Ai.begin(), Ai.begin() + nz, iw.begin());
  len[n] = 0;
  int64_t cnz = nz;
  for (int i = 0; i <= n; ++i) {
    head[i] = -1;
    last[i] = -1;
    next[i] = -1;
    hhead[i] = -1;
    nv[i] = 1;
    w[i] = 1;
    elen[i] = 0;
    degree[i] = len[i];
  }
  int64_t mark = reset_marks(0, 0, w, n);
  elen[n] = -2;  // node n: dummy root collecting dense nodes
  pe[n] = -1;
  w[n] = 0;

  int64_t nel = 0;
  for (int i = 0; i < n; ++i) {
    int64_t d = degree[i];
    if (d == 0) {  // isolated node: eliminate now
      elen[i] = -2;
      ++nel;
      pe[i] = -1;
      w[i] = 0;
    } else if (d > dense) {  // dense node: absorb into the dummy root, ordered last
      nv[i] = 0;
      elen[i] = -1;
      ++nel;
      pe[i] = flip(n);
      nv[n]++;
    } else {
      if (head[d] != -1) last[head[d]] = i;
      next[i] = head[d];
      head[d] = i;
    }
  }

  int64_t mindeg = 0, lemax = 0;
  // flops lower bound of the pivots eliminated so far: pivot k's element Lk is its exact pattern
  // (dense nodes left out: they only add), so its nvk columns count dk + nvk, ..., dk + 1 entries
  double lb = 0.0;
  int64_t npiv = 0;
  while (nel < n) {
    // ---- select a node of minimum approximate degree
    int k = -1;
    for (; mindeg < n && (k = head[mindeg]) == -1; ++mindeg) {
    }
    if (next[k] != -1) last[next[k]] = -1;
    head[mindeg] = next[k];
    int64_t elenk = elen[k];
    int64_t nvk = nv[k];
    nel += nvk;

    // ---- garbage collection of the quotient-graph workspace
    if (elenk > 0 && cnz + mindeg >= nzmax) {
      for (int j = 0; j < n; ++j) {
        int64_t p = pe[j];
        if (p >= 0) {
          pe[j] = iw[p];
          iw[p] = (int32_t)flip(j);
        }
      }
      int64_t q = 0, p = 0;
      while (p < cnz) {
        int64_t j = flip(iw[p++]);
        if (j >= 0) {
          iw[q] = (int32_t)pe[j];
          pe[j] = q++;
          for (int64_t k3 = 0; k3 < len[j] - 1; ++k3) iw[q++] = iw[p++];
        }
      }
      cnz = q;
    }

    // ---- construct the new element Lk
    int64_t dk = 0;
    nv[k] = (int32_t)-nvk;
    int64_t p = pe[k];
    int64_t pk1 = (elenk == 0) ? p : cnz;
    int64_t pk2 = pk1;
    for (int64_t k1 = 1; k1 <= elenk + 1; ++k1) {
      int64_t e, pj, ln;
      if (k1 > elenk) {
        e = k;
        pj = p;
        ln = len[k] - elenk;
      } else {
        e = iw[p++];
        pj = pe[e];
        ln = len[e];
      }
      for (int64_t k2 = 1; k2 <= ln; ++k2) {
        int i = iw[pj++];
        int64_t nvi = nv[i];
        if (nvi <= 0) continue;
        dk += nvi;
        nv[i] = (int32_t)-nvi;
        iw[pk2++] = i;
        if (next[i] != -1) last[next[i]] = last[i];
        if (last[i] != -1)
          next[last[i]] = next[i];
        else
          head[degree[i]] = next[i];
      }
      if (e != k) {
        pe[e] = flip(k);
        w[e] = 0;
      }
    }
    if (elenk != 0) cnz = pk2;
    degree[k] = dk;
    pe[k] = pk1;
    len[k] = (int32_t)(pk2 - pk1);
    elen[k] = -2;

    // ---- |Le \ Lk| for every element e adjacent to a variable of Lk
    mark = reset_marks(mark, lemax, w, n);
    for (int64_t pk = pk1; pk < pk2; ++pk) {
      int i = iw[pk];
      int64_t eln = elen[i];
      if (eln <= 0) continue;
      int64_t nvi = -nv[i];
      int64_t wnvi = mark - nvi;
      for (int64_t q = pe[i]; q <= pe[i] + eln - 1; ++q) {
        int e = iw[q];
        if (w[e] >= mark)
          w[e] -= nvi;
        else if (w[e] != 0)
          w[e] = degree[e] + wnvi;
      }
    }

    // ---- approximate degree update, element absorption, hashing
    for (int64_t pk = pk1; pk < pk2; ++pk) {
      int i = iw[pk];
      int64_t p1 = pe[i], p2 = p1 + elen[i] - 1, pn = p1;
      uint64_t h = 0;
      int64_t d = 0;
      for (int64_t q = p1; q <= p2; ++q) {
        int e = iw[q];
        if (w[e] != 0) {
          int64_t dext = w[e] - mark;
          if (dext > 0) {
            d += dext;
            iw[pn++] = e;
            h += (uint64_t)e;
          } else {  // aggressive absorption: Le is a subset of Lk
            pe[e] = flip(k);
            w[e] = 0;
          }
        }
      }
      elen[i] = (int32_t)(pn - p1 + 1);
      int64_t p3 = pn, p4 = p1 + len[i];
      for (int64_t q = p2 + 1; q < p4; ++q) {
        int j = iw[q];
        int64_t nvj = nv[j];
        if (nvj <= 0) continue;
        d += nvj;
        iw[pn++] = j;
        h += (uint64_t)j;
      }
      if (d == 0) {  // mass elimination: i is only adjacent to k
        pe[i] = flip(k);
        int64_t nvi = -nv[i];
        dk -= nvi;
        nvk += nvi;
        nel += nvi;
        nv[i] = 0;
        elen[i] = -1;
      } else {
        degree[i] = std::min(degree[i], d);
        iw[pn] = iw[p3];
        iw[p3] = iw[p1];
        iw[p1] = k;
        len[i] = (int32_t)(pn - p1 + 1);
        h %= (uint64_t)n;
        next[i] = hhead[h];
        hhead[h] = i;
        last[i] = (int32_t)h;
      }
    }
    degree[k] = dk;
    lemax = std::max(lemax, dk);
    mark = reset_marks(mark + lemax, lemax, w, n);

    // ---- supervariable detection
    for (int64_t pk = pk1; pk < pk2; ++pk) {
      int i = iw[pk];
      if (nv[i] >= 0) continue;
      int64_t h = last[i];
      i = hhead[h];
      hhead[h] = -1;
      for (; i != -1 && next[i] != -1; i = next[i], ++mark) {
        int64_t ln = len[i], eln = elen[i];
        for (int64_t q = pe[i] + 1; q <= pe[i] + ln - 1; ++q) w[iw[q]] = mark;
        int jlast = i;
        for (int j = next[i]; j != -1;) {
          bool ok = (len[j] == ln) && (elen[j] == eln);
          for (int64_t q = pe[j] + 1; ok && q <= pe[j] + ln - 1; ++q)
            if (w[iw[q]] != mark) ok = false;
          if (ok) {  // j is indistinguishable from i: absorb
            pe[j] = flip(i);
            nv[i] += nv[j];
            nv[j] = 0;
            elen[j] = -1;
            j = next[j];
            next[jlast] = j;
          } else {
            jlast = j;
            j = next[j];
          }
        }
      }
    }

    // ---- finalize the new element, reinsert variables in degree lists
    int64_t q = pk1;
    for (int64_t pk = pk1; pk < pk2; ++pk) {
      int i = iw[pk];
      int64_t nvi = -nv[i];
      if (nvi <= 0) continue;
      nv[i] = (int32_t)nvi;
      int64_t d = degree[i] + dk - nvi;
      d = std::min<int64_t>(d, n - nel - nvi);
      if (head[d] != -1) last[head[d]] = i;
      next[i] = head[d];
      last[i] = -1;
      head[d] = i;
      mindeg = std::min(mindeg, d);
      degree[i] = d;
      iw[q++] = i;
    }
    nv[k] = (int32_t)nvk;
    if (cap) {
      const double a = (double)dk + 1.0, b = (double)(dk + nvk);  // sum over c in [a, b] of c^2 + c - 2
      auto s2 = [](double x) { return x * (x + 1.0) * (2.0 * x + 1.0) / 6.0; };
      lb += (s2(b) - s2(a - 1.0)) + (b * (b + 1.0) - (a - 1.0) * a) / 2.0 - 2.0 * (b - a + 1.0);
      if ((++npiv & 255) == 0 && lb > cap->load(std::memory_order_relaxed)) {
        perm.clear();
        return false;
      }
    }
    if ((len[k] = (int32_t)(q - pk1)) == 0) {
      pe[k] = -1;
      w[k] = 0;
    }
    if (elenk != 0) cnz = q;
  }

  // ---- postorder the assembly tree
  std::vector<int32_t> par(n + 1);
  for (int i = 0; i < n; ++i) par[i] = (pe[i] >= 0) ? -1 : (int32_t)flip(pe[i]);
  par[n] = -1;
  for (int j = 0; j <= n; ++j) head[j] = -1;
  for (int j = n; j >= 0; --j) {  // non-principal variables into their representative's list
    if (nv[j] > 0) continue;
    next[j] = head[par[j]];
    head[par[j]] = j;
  }
  for (int e = n; e >= 0; --e) {  // elements into their parent's list
    if (nv[e] <= 0) continue;
    if (par[e] != -1) {
      next[e] = head[par[e]];
      head[par[e]] = e;
    }
  }
  std::vector<int32_t> post(n + 1), stack(n + 1);
  int64_t k = 0;
  for (int i = 0; i <= n; ++i)
    if (par[i] == -1) k = tree_dfs(i, k, head, next, post, stack);
  // post holds n+1 entries; the dummy root n comes last.
  int64_t o = 0;
  for (int64_t t = 0; t <= n && o < n; ++t)
    if (post[t] != n) perm[o++] = post[t];
  return true;
}

}  // namespace madipm
