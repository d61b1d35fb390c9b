// Nested-dissection fill-reducing ordering (multilevel vertex separators), host side.
//
// The reference's GPU linear solver (cuDSS, scripts/benchmarks_gpu.jl:41-42) orders with a
// METIS-style nested dissection; its CPU solvers (LDLFactorizations, MA57) use minimum-degree
// variants.  SymbolicOptions::ordering selects AMD (csrc/amd.cpp), this ND, or "auto" = both,
// keeping the one with fewer factorisation flops (symbolic.cpp) — SURVEY §8 a12.
//
// Algorithm (written for this project): recursive bisection.  Each connected subgraph larger than
// a leaf is bisected by a multilevel scheme — heavy-edge matching coarsening, greedy graph-growing
// initial partitions on the coarsest graph (several seeds), boundary Fiduccia–Mattheyses refinement
// while uncoarsening — and the edge cut is turned into a minimum vertex separator (König: maximum
// bipartite matching on the cut edges, Hopcroft–Karp).  Order = [part A][part B][separator],
// recursively; disconnected subgraphs are ordered component by component with no separator;
// leaves, and subgraphs without a good separator (|S| > sep_ratio |V|), are ordered by AMD.
// Host-parallel: the two sides of a separator, runs of components and the bisection tries of a
// large subgraph are independent and run on threads of their own (NDOptions::threads); every
// subproblem's random stream is seeded from its position in the recursion, so the order is the same
// whatever the thread count.
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <queue>
#include <thread>
#include <cstdlib>
#include <utility>
#include <memory>
#include <vector>

#include "common.hpp"
#include "symbolic.hpp"

namespace madipm {

namespace {

// std::allocator whose value-less construct leaves the element uninitialised: resize() of the big
// per-level arrays then costs no zero pass, and their pages first fault in on the threads that fill them
template <class T>
struct UninitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = UninitAlloc<U>;
  };
  UninitAlloc() = default;
  template <class U>
  UninitAlloc(const UninitAlloc<U>&) noexcept {}
  template <class U, class... A>
  void construct(U* q, A&&... a) {
    ::new ((void*)q) U(std::forward<A>(a)...);
  }
  template <class U>
  void construct(U* q) noexcept {
    ::new ((void*)q) U;
  }
};
template <class T>
using RawVec = std::vector<T, UninitAlloc<T>>;

struct Graph {
  int n = 0;
  std::vector<int64_t> p;
  RawVec<int32_t> adj, ew;
  std::vector<int32_t> vw;
  bool unit_ew = false;  // every edge weight 1 (an induced subgraph; coarse graphs: false)
  int64_t total_vw() const { return std::accumulate(vw.begin(), vw.end(), (int64_t)0); }
};

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
  uint32_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (uint32_t)(s >> 11);
  }
};

// Heavy-edge matching and contraction.  Returns false when the graph hardly shrinks.
bool coarsen(const Graph& g, Graph& c, std::vector<int32_t>& cmap, RawVec<uint64_t>& scratch, Rng& rng,
             int threads) {
  const int n = g.n;
  std::vector<int32_t> match(n, -1), order(n);
  std::iota(order.begin(), order.end(), 0);
  for (int i = n - 1; i > 0; --i) std::swap(order[i], order[rng.next() % (i + 1)]);
  for (int v : order) {
    if (match[v] != -1) continue;
    int best = -1, bw = -1;
    if (g.unit_ew) {  // the heaviest edge is the first one to an unmatched neighbour (ties: the first)
      for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e)
        if (match[g.adj[e]] == -1) {
          best = g.adj[e];
          break;
        }
    } else {
      for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e) {
        const int u = g.adj[e];
        if (match[u] == -1 && g.ew[e] > bw) {
          bw = g.ew[e];
          best = u;
        }
      }
    }
    if (best == -1) {
      match[v] = -2;  // no unmatched neighbour left: alone
    } else {
      match[v] = best;
      match[best] = v;
    }
  }
  for (int v = 0; v < n; ++v)
    if (match[v] == -2) match[v] = v;
  cmap.assign(n, -1);
  int nc = 0;
  for (int v = 0; v < n; ++v)
    if (cmap[v] == -1) cmap[v] = cmap[match[v]] = nc++;
  if (nc > 0.92 * n) return false;
  c.n = nc;
  c.vw.assign(nc, 0);
  c.p.assign(nc + 1, 0);
  std::vector<int32_t> rep(nc, -1);
  for (int v = 0; v < n; ++v)
    if (rep[cmap[v]] == -1) rep[cmap[v]] = v;
  // Contraction: a coarse vertex's list is its members' neighbours in adjacency order, duplicates
  // merged.  Each coarse vertex is written at its upper-bound offset (its members' degrees: the
  // offsets sum to g's adjacency) into the scratch, ranges of coarse vertices on threads of their
  // own, then packed.  The scratch lives for the whole bisection (sized by its finest level), so its
  // pages fault in once: fresh per-thread buffers per level faulting in concurrently measured 2-4x
  // slower than one thread.  The result does not depend on the thread count.
  std::vector<int64_t> off(nc + 1, 0);
  for (int cv = 0; cv < nc; ++cv) {
    const int v = rep[cv], u = match[v];
    off[cv + 1] = off[cv] + (g.p[v + 1] - g.p[v]) + (u == v ? 0 : g.p[u + 1] - g.p[u]);
  }
  if (scratch.size() < (size_t)off[nc]) scratch.resize(off[nc]);  // (first level: the largest)
  uint64_t* tmp = scratch.data();  // (neighbour, weight) pairs
  auto contract = [&](int cv0, int cv1) {
    std::vector<int64_t> pos(nc, -1);
    for (int cv = cv0; cv < cv1; ++cv) {
      const int v = rep[cv];
      const int u = match[v];
      const int members[2] = {v, u};
      const int64_t start = off[cv];
      int64_t cur = start;
      int32_t w = 0;
      for (int k = 0; k < (u == v ? 1 : 2); ++k) {
        const int x = members[k];
        w += g.vw[x];
        for (int64_t e = g.p[x]; e < g.p[x + 1]; ++e) {
          const int cu = cmap[g.adj[e]];
          if (cu == cv) continue;
          const int64_t q = pos[cu];
          if (q >= start) {
            tmp[q] += (uint64_t)(uint32_t)g.ew[e] << 32;
          } else {
            pos[cu] = cur;
            tmp[cur++] = (uint32_t)cu | ((uint64_t)(uint32_t)g.ew[e] << 32);
          }
        }
      }
      c.vw[cv] = w;
      c.p[cv + 1] = cur - start;
    }
  };
  const int T = std::max(1, std::min(threads, (int)(off[nc] / 200000)));
  std::vector<int> cut(T + 1, nc);
  cut[0] = 0;
  for (int t = 1; t < T; ++t)
    cut[t] = (int)(std::lower_bound(off.begin(), off.end(), off[nc] * t / T) - off.begin());
  auto on_threads = [&](auto&& f) {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(f, cut[t], cut[t + 1]);
    f(cut[0], cut[1]);
    for (auto& x : th) x.join();
  };
  on_threads(contract);
  for (int cv = 0; cv < nc; ++cv) c.p[cv + 1] += c.p[cv];
  c.adj.resize(c.p[nc]);
  c.ew.resize(c.p[nc]);
  on_threads([&](int cv0, int cv1) {
    for (int cv = cv0; cv < cv1; ++cv) {
      const uint64_t* src = tmp + off[cv];
      int32_t* a = c.adj.data() + c.p[cv];
      int32_t* ew = c.ew.data() + c.p[cv];
      const int64_t d = c.p[cv + 1] - c.p[cv];
      for (int64_t k = 0; k < d; ++k) {
        a[k] = (int32_t)(uint32_t)src[k];
        ew[k] = (int32_t)(src[k] >> 32);
      }
    }
  });
  return true;
}

int64_t cut_weight(const Graph& g, const std::vector<uint8_t>& part) {
  int64_t cut = 0;
  for (int v = 0; v < g.n; ++v)
    for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e)
      if (part[v] != part[g.adj[e]]) cut += g.ew[e];
  return cut / 2;
}

// Greedy graph growing from `seed`: vertices join side 0 by best gain until half the weight.
void grow(const Graph& g, int seed, std::vector<uint8_t>& part) {
  const int64_t W = g.total_vw();
  part.assign(g.n, 1);
  std::vector<int64_t> gain(g.n, 0);  // (edges to side 0) - (edges to side 1), for side-1 vertices
  for (int v = 0; v < g.n; ++v)
    for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e) gain[v] -= g.ew[e];
  std::priority_queue<std::pair<int64_t, int>> pq;
  int64_t w0 = 0;
  int next_seed = seed;
  std::vector<uint8_t> inq(g.n, 0);
  while (2 * w0 < W) {
    int v = -1;
    while (!pq.empty()) {
      auto t = pq.top();
      pq.pop();
      if (part[t.second] == 1 && t.first == gain[t.second]) {
        v = t.second;
        break;
      }
    }
    if (v == -1) {  // empty frontier (disconnected coarse graph): next unassigned vertex
      while (next_seed < g.n && part[next_seed] == 0) ++next_seed;
      if (next_seed >= g.n) {
        for (v = 0; v < g.n && part[v] == 0; ++v) {
        }
        if (v >= g.n) break;
      } else {
        v = next_seed;
      }
    }
    part[v] = 0;
    w0 += g.vw[v];
    for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e) {
      const int u = g.adj[e];
      if (part[u] == 1) {
        gain[u] += 2 * g.ew[e];
        pq.push({gain[u], u});
      }
    }
  }
}

// Boundary FM refinement with a balance bound; a few passes, best prefix kept.  Each pass starts
// from every vertex's gain (external - internal edge weight) and the boundary vertices, one scan of
// the edges split over `threads` (the moves themselves are few: ~64-80 per pass, 2-3 % of a pass's
// time on ex10's levels, the scan the rest).  The heap is built from the boundary in one go: pops
// follow the (gain, vertex) order alone, whatever the push order.
void refine(const Graph& g, std::vector<uint8_t>& part, double imbalance, int threads) {
  const int64_t W = g.total_vw();
  const int64_t maxw = (int64_t)((0.5 + imbalance) * W) + 1;
  const int T = std::max(1, std::min(threads, (int)(g.adj.size() / 250000)));
  std::vector<int> cut_v(T + 1, g.n);
  cut_v[0] = 0;
  for (int t = 1; t < T; ++t)
    cut_v[t] = (int)(std::lower_bound(g.p.begin(), g.p.end(), (int64_t)g.adj.size() * t / T) - g.p.begin());
  std::vector<int64_t> gain(g.n), ext(T);
  std::vector<uint8_t> bnd(g.n);
  auto scan = [&](int t) {
    int64_t x = 0;
    for (int v = cut_v[t]; v < cut_v[t + 1]; ++v) {
      int64_t gv = 0, xv = 0;
      bool b = false;
      for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e) {
        const bool c = part[g.adj[e]] != part[v];
        gv += c ? g.ew[e] : -g.ew[e];
        xv += c ? g.ew[e] : 0;
        b |= c;
      }
      gain[v] = gv;
      bnd[v] = b;
      x += xv;
    }
    ext[t] = x;
  };
  int64_t cut = -1;  // the cut weight after the pass (its change is tracked by the moves: cur)
  for (int pass = 0; pass < 4; ++pass) {
    int64_t wside[2] = {0, 0};
    for (int v = 0; v < g.n; ++v) wside[part[v]] += g.vw[v];
    {
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t) th.emplace_back(scan, t);
      scan(0);
      for (auto& x : th) x.join();
    }
    if (cut < 0) {  // the cut before the first pass: half the external weight
      cut = 0;
      for (int64_t x : ext) cut += x;
      cut /= 2;
    }
    std::vector<std::pair<int64_t, int>> init;
    for (int v = 0; v < g.n; ++v)
      if (bnd[v]) init.emplace_back(gain[v], v);
    std::priority_queue<std::pair<int64_t, int>> pq(std::less<std::pair<int64_t, int>>(), std::move(init));
    std::vector<uint8_t> locked(g.n, 0);
    std::vector<int> moves;
    int64_t cur = 0, best = 0;
    size_t best_len = 0;
    int since_best = 0;
    while (!pq.empty() && since_best < 64) {
      auto t = pq.top();
      pq.pop();
      const int v = t.second;
      if (locked[v] || t.first != gain[v]) continue;
      const int from = part[v], to = 1 - from;
      if (wside[to] + g.vw[v] > maxw) continue;
      locked[v] = 1;
      part[v] = (uint8_t)to;
      wside[from] -= g.vw[v];
      wside[to] += g.vw[v];
      cur -= gain[v];
      moves.push_back(v);
      for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e) {
        const int u = g.adj[e];
        gain[u] += (part[u] == to) ? -2 * g.ew[e] : 2 * g.ew[e];
        if (!locked[u]) pq.push({gain[u], u});
      }
      gain[v] = -gain[v];
      if (cur < best) {
        best = cur;
        best_len = moves.size();
        since_best = 0;
      } else {
        ++since_best;
      }
    }
    for (size_t k = moves.size(); k > best_len; --k) part[moves[k - 1]] ^= 1;  // roll back
    if (best == 0) break;
    cut += best;  // (each move changes the cut by exactly -gain: cur tracks it)
    if (-best * 200 < cut) break;  // converged (< 0.5 % gain)
  }
}

// Multilevel bisection of a connected graph; returns the partition of the finest graph.
void bisect(const Graph& g0, std::vector<uint8_t>& part, Rng& rng, int threads) {
  PhaseClock clk("  nd bisect");  // MADIPM_SYMBOLIC_TIMING: the phases of a bisection of > 1e5 vertices
  if (g0.n < 100000) clk.on = false;
  std::vector<Graph> coarse;  // levels 1, 2, ... (level 0: g0 itself)
  std::vector<std::vector<int32_t>> maps;
  RawVec<uint64_t> scratch;
  auto level = [&](int l) -> const Graph& { return l == 0 ? g0 : coarse[l - 1]; };
  while (level((int)coarse.size()).n > 120) {
    Graph c;
    std::vector<int32_t> cmap;
    if (!coarsen(level((int)coarse.size()), c, cmap, scratch, rng, threads)) break;
    coarse.push_back(std::move(c));
    maps.push_back(std::move(cmap));
  }
  RawVec<uint64_t>().swap(scratch);
  clk("coarsen");
  const Graph& gc = level((int)coarse.size());
  int64_t best = -1;
  std::vector<uint8_t> trial;
  for (int t = 0; t < 8; ++t) {
    grow(gc, (int)(rng.next() % gc.n), trial);
    refine(gc, trial, 0.05, 1);
    const int64_t cw = cut_weight(gc, trial);
    if (best < 0 || cw < best) {
      best = cw;
      part = trial;
    }
  }
  clk("initial partitions");
  for (int l = (int)coarse.size() - 1; l >= 0; --l) {
    std::vector<uint8_t> fine(level(l).n);
    for (int v = 0; v < level(l).n; ++v) fine[v] = part[maps[l][v]];
    part.swap(fine);
    refine(level(l), part, 0.05, threads);
  }
  clk("uncoarsen + refine");
}

// Minimum vertex cover of the cut edges (König), returned as sep[v] = 1.
void vertex_separator(const Graph& g, const std::vector<uint8_t>& part, std::vector<uint8_t>& sep) {
  const int n = g.n;
  sep.assign(n, 0);
  std::vector<int32_t> L, R, lid(n, -1), rid(n, -1);
  for (int v = 0; v < n; ++v)
    for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e)
      if (part[g.adj[e]] != part[v]) {
        if (part[v] == 0) {
          lid[v] = (int32_t)L.size();
          L.push_back(v);
        } else {
          rid[v] = (int32_t)R.size();
          R.push_back(v);
        }
        break;
      }
  const int nl = (int)L.size(), nr = (int)R.size();
  std::vector<int64_t> bp(nl + 1, 0);
  std::vector<int32_t> badj;
  for (int a = 0; a < nl; ++a) {
    const int v = L[a];
    for (int64_t e = g.p[v]; e < g.p[v + 1]; ++e)
      if (rid[g.adj[e]] >= 0) badj.push_back(rid[g.adj[e]]);
    bp[a + 1] = (int64_t)badj.size();
  }
  // Hopcroft–Karp
  std::vector<int32_t> ml(nl, -1), mr(nr, -1), dist(nl);
  const int INF = 1 << 30;
  std::vector<int32_t> bq;
  bq.reserve(nl);
  auto bfs = [&]() {
    std::vector<int32_t>& q = bq;
    q.clear();
    bool found = false;
    for (int a = 0; a < nl; ++a) {
      if (ml[a] == -1) {
        dist[a] = 0;
        q.push_back(a);
      } else {
        dist[a] = INF;
      }
    }
    for (size_t h = 0; h < q.size(); ++h) {
      const int a = q[h];
      for (int64_t e = bp[a]; e < bp[a + 1]; ++e) {
        const int b = badj[e];
        const int a2 = mr[b];
        if (a2 == -1) {
          found = true;
        } else if (dist[a2] == INF) {
          dist[a2] = dist[a] + 1;
          q.push_back(a2);
        }
      }
    }
    return found;
  };
  std::vector<int64_t> it(nl);
  std::vector<int32_t> stk;
  auto dfs = [&](int root) {  // iterative augmenting-path search along the BFS layers
    stk.assign(1, root);
    while (!stk.empty()) {
      const int a = stk.back();
      bool advanced = false;
      for (; it[a] < bp[a + 1]; ++it[a]) {
        const int b = badj[it[a]];
        const int a2 = mr[b];
        if (a2 == -1) {  // augment along the stack
          for (int k = (int)stk.size() - 1; k >= 0; --k) {
            const int aa = stk[k];
            const int bb = badj[it[aa]];
            const int prev = ml[aa];
            ml[aa] = bb;
            mr[bb] = aa;
            (void)prev;
          }
          return true;
        }
        if (dist[a2] == dist[a] + 1) {
          stk.push_back(a2);
          advanced = true;
          break;
        }
      }
      if (!advanced) {
        dist[a] = INF;
        stk.pop_back();
        if (!stk.empty()) ++it[stk.back()];
      }
    }
    return false;
  };
  while (bfs()) {
    for (int a = 0; a < nl; ++a) it[a] = bp[a];
    for (int a = 0; a < nl; ++a)
      if (ml[a] == -1) dfs(a);
  }
  // Z = reachable from unmatched left vertices by alternating paths; cover = (L \ Z) + (R & Z)
  std::vector<uint8_t> zl(nl, 0), zr(nr, 0);
  std::vector<int32_t> q;
  for (int a = 0; a < nl; ++a)
    if (ml[a] == -1) {
      zl[a] = 1;
      q.push_back(a);
    }
  for (size_t h = 0; h < q.size(); ++h) {
    const int a = q[h];
    for (int64_t e = bp[a]; e < bp[a + 1]; ++e) {
      const int b = badj[e];
      if (zr[b] || ml[a] == b) continue;
      zr[b] = 1;
      const int a2 = mr[b];
      if (a2 >= 0 && !zl[a2]) {
        zl[a2] = 1;
        q.push_back(a2);
      }
    }
  }
  for (int a = 0; a < nl; ++a)
    if (!zl[a]) sep[L[a]] = 1;
  for (int b = 0; b < nr; ++b)
    if (zr[b]) sep[R[b]] = 1;
}

// Per-thread scratch: global -> local id of the subgraph being built (-1 outside).  Every task that
// runs on a thread of its own gets its own map, so concurrent subgraphs never see each other's ids.
struct Ctx {
  std::vector<int32_t> loc;
  explicit Ctx(int n) : loc(n, -1) {}
};

// seeds of the subproblems: a fixed function of the parent's seed and the child's index, so the
// order does not depend on how the recursion is spread over threads
inline uint64_t child_seed(uint64_t s, uint64_t k) {
  uint64_t z = s + 0x9E3779B97F4A7C15ull * (k + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Dissector {
  const std::vector<int64_t>& Ap;
  const std::vector<int32_t>& Ai;
  const NDOptions& opt;
  const int n;
  // subgraphs below this size never get a thread of their own (the spawn costs more than the work)
  static constexpr int kParMin = 4096;

  Dissector(const std::vector<int64_t>& p, const std::vector<int32_t>& i, const NDOptions& o, int nn)
      : Ap(p), Ai(i), opt(o), n(nn) {}

  // (large subgraphs: degrees counted, then the lists filled, by vertex ranges on `par` threads)
  void induced(Ctx& cx, const std::vector<int32_t>& verts, Graph& g, int par = 1) const {
    std::vector<int32_t>& loc = cx.loc;
    for (size_t k = 0; k < verts.size(); ++k) loc[verts[k]] = (int32_t)k;
    g.n = (int)verts.size();
    g.p.assign(g.n + 1, 0);
    g.adj.clear();
    const int T = g.n >= 50000 ? std::max(1, std::min(par, g.n / 25000)) : 1;
    if (T == 1) {
      for (int k = 0; k < g.n; ++k) {
        const int v = verts[k];
        for (int64_t e = Ap[v]; e < Ap[v + 1]; ++e) {
          const int u = loc[Ai[e]];
          if (u >= 0 && u != k) g.adj.push_back(u);
        }
        g.p[k + 1] = (int64_t)g.adj.size();
      }
    } else {
      auto on_threads = [&](auto&& f) {
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(f, (int)((int64_t)g.n * t / T), (int)((int64_t)g.n * (t + 1) / T));
        f(0, g.n / T);
        for (auto& x : th) x.join();
      };
      on_threads([&](int k0, int k1) {
        for (int k = k0; k < k1; ++k) {
          const int v = verts[k];
          int64_t d = 0;
          for (int64_t e = Ap[v]; e < Ap[v + 1]; ++e) {
            const int u = loc[Ai[e]];
            d += u >= 0 && u != k;
          }
          g.p[k + 1] = d;
        }
      });
      for (int k = 0; k < g.n; ++k) g.p[k + 1] += g.p[k];
      g.adj.resize(g.p[g.n]);
      on_threads([&](int k0, int k1) {
        for (int k = k0; k < k1; ++k) {
          const int v = verts[k];
          int64_t q = g.p[k];
          for (int64_t e = Ap[v]; e < Ap[v + 1]; ++e) {
            const int u = loc[Ai[e]];
            if (u >= 0 && u != k) g.adj[q++] = u;
          }
        }
      });
    }
    g.ew.assign(g.adj.size(), 1);
    g.unit_ew = true;
    g.vw.assign(g.n, 1);
    for (int v : verts) loc[v] = -1;
  }

  void leaf(const std::vector<int32_t>& verts, const Graph& g, std::vector<int32_t>& out) const {
    std::vector<int32_t> lp;
    if (g.n > 2) {
      amd_order(g.n, g.p, std::vector<int32_t>(g.adj.begin(), g.adj.end()), lp, opt.dense_alpha);
    } else {
      lp.resize(g.n);
      std::iota(lp.begin(), lp.end(), 0);
    }
    for (int k : lp) out.push_back(verts[k]);
  }

  // Orders `parts` (disjoint vertex sets) one after another into `out`: in this thread when `par`
  // is 1, else split into two runs of about equal vertex count, the second on a thread of its own.
  void dissect_list(Ctx& cx, std::vector<std::vector<int32_t>>& parts, size_t p0, size_t p1, int depth,
                    uint64_t seed, int par, std::vector<int32_t>& out) const {
    int64_t tot = 0;
    for (size_t k = p0; k < p1; ++k) tot += (int64_t)parts[k].size();
    if (par <= 1 || p1 - p0 < 2 || tot < 2 * kParMin) {
      for (size_t k = p0; k < p1; ++k) dissect(cx, parts[k], depth, child_seed(seed, k), 1, out);
      return;
    }
    size_t mid = p0 + 1;
    int64_t acc = (int64_t)parts[p0].size();
    while (mid + 1 < p1 && 2 * (acc + (int64_t)parts[mid].size()) <= tot) acc += (int64_t)parts[mid++].size();
    std::vector<int32_t> out2;
    std::thread th([&] {
      Ctx c2(n);
      dissect_list(c2, parts, mid, p1, depth, seed, par / 2, out2);
    });
    dissect_list(cx, parts, p0, mid, depth, seed, par - par / 2, out);
    th.join();
    out.insert(out.end(), out2.begin(), out2.end());
  }

  void dissect(Ctx& cx, const std::vector<int32_t>& verts, int depth, uint64_t seed, int par,
               std::vector<int32_t>& out) const {
    PhaseClock clk("  nd top");  // MADIPM_SYMBOLIC_TIMING: the top bisection and the rest
    if (2 * verts.size() < (size_t)n) clk.on = false;  // the top bisection (below any component split)
    Graph g;
    induced(cx, verts, g, par);
    if (g.n <= opt.leaf_size || depth > 60) {
      leaf(verts, g, out);
      return;
    }
    // connected components
    std::vector<int32_t> comp(g.n, -1), q;
    int nc = 0;
    for (int s = 0; s < g.n; ++s) {
      if (comp[s] != -1) continue;
      q.assign(1, s);
      comp[s] = nc;
      for (size_t h = 0; h < q.size(); ++h)
        for (int64_t e = g.p[q[h]]; e < g.p[q[h] + 1]; ++e)
          if (comp[g.adj[e]] == -1) {
            comp[g.adj[e]] = nc;
            q.push_back(g.adj[e]);
          }
      ++nc;
    }
    if (nc > 1) {
      std::vector<std::vector<int32_t>> parts(nc);
      for (int k = 0; k < g.n; ++k) parts[comp[k]].push_back(verts[k]);
      g = Graph();
      dissect_list(cx, parts, 0, parts.size(), depth + 1, seed, par, out);
      return;
    }
    // best of a few multilevel bisections, scored by separator size and balance; the tries are
    // independent (a seed each) and run on threads of their own where the budget allows
    const int tries = g.n > 20000 ? opt.tries : 1;  // several tries only where separators matter most
    std::vector<std::vector<uint8_t>> parts(tries), seps(tries);
    auto one_try = [&](int t) {
      Rng rng(child_seed(seed, 1000 + (uint64_t)t));
      bisect(g, parts[t], rng, tries > 1 ? std::max(1, par / tries) : par);
      vertex_separator(g, parts[t], seps[t]);
    };
    auto sizes = [&](int t, int64_t& ns, int64_t& na, int64_t& nb) {
      ns = na = nb = 0;
      for (int k = 0; k < g.n; ++k) {
        if (seps[t][k])
          ++ns;
        else if (parts[t][k] == 0)
          ++na;
        else
          ++nb;
      }
    };
    if (tries > 1 && par > 1) {
      std::vector<std::thread> th;
      for (int t = 1; t < tries; ++t) th.emplace_back(one_try, t);
      one_try(0);
      for (auto& x : th) x.join();
    } else {
      one_try(0);
      int64_t ns0, na0, nb0;
      sizes(0, ns0, na0, nb0);
      // (the scoring below stops at a first try without a small separator: the others are not needed)
      const bool stop = na0 != 0 && nb0 != 0 && ns0 > 2.0 * opt.sep_ratio * g.n;
      for (int t = 1; t < tries && !stop; ++t) one_try(t);
    }
    clk("bisection tries");
    int best = -1;
    double bscore = 1e300;
    for (int t = 0; t < tries; ++t) {
      int64_t ns, na, nb;
      sizes(t, ns, na, nb);
      if (na == 0 || nb == 0) continue;
      if (t == 0 && ns > 2.0 * opt.sep_ratio * g.n) break;  // no small separator here: AMD
      const double score = (double)ns * (1.0 + 2.0 * std::abs((double)(na - nb)) / (double)g.n);
      if (score < bscore) {
        bscore = score;
        best = t;
      }
    }
    int64_t ns = 0;
    if (best >= 0)
      for (uint8_t s : seps[best]) ns += s;
    if (best < 0 || ns > opt.sep_ratio * g.n) {
      leaf(verts, g, out);
      return;
    }
    std::vector<std::vector<int32_t>> ab(2);
    std::vector<int32_t> S;
    for (int k = 0; k < g.n; ++k) (seps[best][k] ? S : ab[parts[best][k]]).push_back(verts[k]);
    g = Graph();
    parts.clear();
    seps.clear();
    // [A][B][separator]: A and B in parallel when both are large enough
    if (par > 1 && (int64_t)ab[0].size() >= kParMin && (int64_t)ab[1].size() >= kParMin) {
      std::vector<int32_t> outB;
      std::thread th([&] {
        Ctx c2(n);
        dissect(c2, ab[1], depth + 1, child_seed(seed, 2), par / 2, outB);
      });
      dissect(cx, ab[0], depth + 1, child_seed(seed, 1), par - par / 2, out);
      th.join();
      clk("both sides");
      out.insert(out.end(), outB.begin(), outB.end());
    } else {
      dissect(cx, ab[0], depth + 1, child_seed(seed, 1), 1, out);
      dissect(cx, ab[1], depth + 1, child_seed(seed, 2), 1, out);
    }
    out.insert(out.end(), S.begin(), S.end());
  }
};

}  // namespace

void nd_order(int n, const std::vector<int64_t>& Ap, const std::vector<int32_t>& Ai, std::vector<int32_t>& perm,
              const NDOptions& opt) {
  Dissector d(Ap, Ai, opt, n);
  std::vector<int32_t> out;
  // Dense vertices (degree above AMD's threshold, max(16, alpha sqrt(n))) are deferred and ordered
  // last, as AMD does: they would sit in every separator anyway, and leaving them in the graph makes
  // each level's induced subgraph / bisection cost O(their degree) -- for a dense-column QP (A dense,
  // H diagonal) that is every edge of the matrix at every level.  Dissection then runs on the rest.
  int64_t dense = (int64_t)std::max(16.0, opt.dense_alpha * std::sqrt((double)n));
  dense = std::min<int64_t>(n - 2, dense);
  if (opt.dense_alpha < 0) dense = n;
  // When more than half the vertices pass the threshold (a dense A block makes both its row and its
  // column vertices "dense"), the lowest degree class is put back until at most half are deferred:
  // for [H A'; A 0] with A dense m x n, m < n, that defers exactly the m constraint vertices.
  for (;;) {
    int64_t cnt = 0, lo = INT64_MAX;
    for (int v = 0; v < n; ++v) {
      const int64_t dg = Ap[v + 1] - Ap[v];
      if (dg > dense) ++cnt, lo = std::min(lo, dg);
    }
    if (2 * cnt <= n) break;
    dense = lo;
  }
  std::vector<int32_t> all, deferred;
  all.reserve(n);
  for (int v = 0; v < n; ++v) (Ap[v + 1] - Ap[v] > dense ? deferred : all).push_back(v);
  out.reserve(n);
  Ctx cx(n);
  PhaseClock clk("  nd order");
  d.dissect(cx, all, 0, opt.seed, std::max(1, opt.threads), out);
  clk("dissection");
  out.insert(out.end(), deferred.begin(), deferred.end());
  MADIPM_REQUIRE((int)out.size() == n, "nested dissection lost vertices");
  perm.swap(out);
}

}  // namespace madipm
