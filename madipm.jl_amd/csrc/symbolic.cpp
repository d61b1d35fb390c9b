// Symbolic analysis for the multifrontal supernodal LDL^T — see symbolic.hpp.
//
// Elimination tree: Liu's algorithm with path compression.  Column counts: Gilbert, Ng & Peyton
// (skeleton matrix / row-subtree leaves with least-common-ancestor compression).  Supernodes:
// fundamental supernodes in postorder, then relaxed amalgamation with the (nrelax, zrelax)
// thresholds popularised by CHOLMOD.  All written for this project.
#include "symbolic.hpp"

#include <algorithm>
#include <cstring>
#include <climits>
#include <cstdlib>
#include <numeric>
#include <chrono>
#include <cstdio>
#include <thread>
#include <atomic>
#include <limits>
#include <memory>

#include "common.hpp"

namespace madipm {

// Host threads for the O(nnz) passes of the analysis (MADIPM_ANALYSIS_THREADS, default: the
// hardware threads, at most 16).  Every parallel pass gives the sequential result bit for bit.
int analysis_threads() {
  static const int nt = [] {
    int t = (int)std::thread::hardware_concurrency();
    if (const char* e = std::getenv("MADIPM_ANALYSIS_THREADS")) t = std::atoi(e);
    return std::max(1, std::min(t, 16));
  }();
  return nt;
}

namespace {

constexpr int NT_FOLD = SymbolicPlan::kFoldThreads;  // threads of k_fact_tree (product-list chunks)

struct Pattern {
  // strictly-lower pattern of P K P^T: column lists (rows > col) and row lists (cols < row)
  std::vector<int64_t> cp, rp;
  hvec<int32_t> ci, ri;
};

// f(t, j0, j1) on T contiguous column ranges balanced by entries (colptr), one thread each
template <class F>
void par_columns(int N, const int64_t* colptr, int T, F f) {
  if (T <= 1) {
    f(0, 0, N);
    return;
  }
  std::vector<int> cut(T + 1, N);
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    const int64_t target = colptr[N] / T * t;
    cut[t] = (int)(std::lower_bound(colptr, colptr + N + 1, target) - colptr);
    cut[t] = std::max(cut[t], cut[t - 1]);
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(f, t, cut[t], cut[t + 1]);
  for (auto& x : th) x.join();
}

// Twin leaves: columns j with an empty row list (no neighbour to their left: etree leaves, L's
// column j = the column list of P K P^T, no fill) whose column list is the same row set as an
// earlier such column's (its representative; twin[j] = that column, else -1).  A twin adds to the
// graph only the clique its representative already adds, so the etree and the other columns' counts
// are those of the pattern without the twins' entries; a twin's parent is its representative's (the
// least row of the shared set) and its count is the representative's.  A QP with a diagonal Hessian
// and dense A in natural order: all x columns but one are twins (dense 50k x 10k: 5e8 of the
// 5e8 entries skipped by the etree's path compression and the column counts).
// Candidates by (length, two order-free hashes); the set equality is then checked exactly.
void find_twins(int N, const Pattern& P, const std::vector<uint8_t>& leaf, std::vector<int32_t>& twin) {
  twin.assign(N, -1);
  auto mix = [](uint64_t x) {  // splitmix64 finaliser
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
  };
  struct Key {
    int64_t len;
    uint64_t h1, h2;
    int32_t j;
  };
  std::vector<Key> keys;
  for (int j = 0; j < N; ++j)
    if (leaf[j] && P.cp[j + 1] - P.cp[j] >= 2) keys.push_back({P.cp[j + 1] - P.cp[j], 0, 0, j});
  if (keys.size() < 2) return;
  {
    const int T = std::max(1, std::min<int>(analysis_threads(), (int)(keys.size() / 256)));
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        for (size_t q = t; q < keys.size(); q += T) {
          uint64_t a = 0, b = 0;
          for (int64_t p = P.cp[keys[q].j]; p < P.cp[keys[q].j + 1]; ++p) {
            const uint64_t h = mix((uint64_t)P.ci[p]);
            a += h;
            b ^= mix(h ^ 0x5bd1e9955bd1e995ull);
          }
          keys[q].h1 = a;
          keys[q].h2 = b;
        }
      });
    for (auto& x : th) x.join();
  }
  std::sort(keys.begin(), keys.end(), [](const Key& x, const Key& y) {
    if (x.len != y.len) return x.len < y.len;
    if (x.h1 != y.h1) return x.h1 < y.h1;
    if (x.h2 != y.h2) return x.h2 < y.h2;
    return x.j < y.j;
  });
  // exact check per candidate group: the representative's rows marked, each member's rows must hit
  // distinct marks (a mark is cleared on its hit and restored after the member)
  std::vector<uint8_t> mark(N, 0);
  for (size_t g0 = 0, g1; g0 < keys.size(); g0 = g1) {
    g1 = g0 + 1;
    while (g1 < keys.size() && keys[g1].len == keys[g0].len && keys[g1].h1 == keys[g0].h1 &&
           keys[g1].h2 == keys[g0].h2)
      ++g1;
    if (g1 - g0 < 2) continue;
    const int rep = keys[g0].j;
    for (int64_t p = P.cp[rep]; p < P.cp[rep + 1]; ++p) mark[P.ci[p]] = 1;
    const int T = std::max(1, std::min<int>(analysis_threads(), (int)((g1 - g0) / 64)));
    std::vector<std::thread> th;
    std::vector<std::vector<uint8_t>> tm(T > 1 ? T : 0);
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        std::vector<uint8_t>& m = T > 1 ? tm[t] : mark;
        if (T > 1) m = mark;
        for (size_t q = g0 + 1 + t; q < g1; q += T) {
          const int j = keys[q].j;
          int64_t p = P.cp[j];
          for (; p < P.cp[j + 1] && m[P.ci[p]]; ++p) m[P.ci[p]] = 0;
          const bool same = p == P.cp[j + 1];
          for (int64_t r = P.cp[j]; r < p; ++r) m[P.ci[r]] = 1;
          if (same) twin[j] = rep;
        }
      });
    for (auto& x : th) x.join();
    for (int64_t p = P.cp[rep]; p < P.cp[rep + 1]; ++p) mark[P.ci[p]] = 0;
  }
}

// Strictly-lower pattern of P K P^T by column and by row: a counting sort of the entries into
// column / row buckets.  Threaded over column ranges when the matrix is dense enough to pay (private
// bucket counts per thread, offsets in thread order: the same bucket order as one pass).  The row
// lists leave out the entries of twin leaves (find_twins, from the column lists): no pass reads them.
void build_pattern(int N, const int64_t* colptr, const int32_t* rowval, const std::vector<int32_t>& pinv,
                   Pattern& P, std::vector<int32_t>& twin) {
  const int64_t nnz = colptr[N];
  int T = analysis_threads();
  if (nnz < 16 * (int64_t)N || (int64_t)T * N > (int64_t)1 << 27 || nnz < ((int64_t)1 << 22)) T = 1;
  std::vector<std::vector<int64_t>> cc(T, std::vector<int64_t>(N + 1, 0)), rc(T, std::vector<int64_t>(N + 1, 0));
  par_columns(N, colptr, T, [&](int t, int j0, int j1) {
    int64_t* c = cc[t].data();
    int64_t* r = rc[t].data();
    for (int j = j0; j < j1; ++j) {
      const int b = pinv[j];
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
        const int i = rowval[p];
        if (i == j) continue;
        const int a = pinv[i];
        c[std::min(a, b)]++;
        r[std::max(a, b)]++;
      }
    }
  });
  // bucket starts, then each thread's offset inside each bucket
  auto offsets = [&](std::vector<std::vector<int64_t>>& cnt, std::vector<int64_t>& ptr) {
    ptr.assign(N + 1, 0);
    for (int k = 0; k < N; ++k) {
      int64_t sum = 0;
      for (int t = 0; t < T; ++t) {
        const int64_t c = cnt[t][k];
        cnt[t][k] = sum;
        sum += c;
      }
      ptr[k + 1] = ptr[k] + sum;
    }
  };
  std::vector<uint8_t> leaf(N, 1);
  for (int t = 0; t < T; ++t)
    for (int k = 0; k < N; ++k)
      if (rc[t][k]) leaf[k] = 0;
  offsets(cc, P.cp);
  P.ci.resize(P.cp[N]);
  par_columns(N, colptr, T, [&](int t, int j0, int j1) {
    int64_t* c = cc[t].data();
    for (int j = j0; j < j1; ++j) {
      const int b = pinv[j];
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
        const int i = rowval[p];
        if (i == j) continue;
        const int a = pinv[i];
        const int lo = std::min(a, b);
        P.ci[P.cp[lo] + c[lo]++] = std::max(a, b);
      }
    }
  });
  find_twins(N, P, leaf, twin);
  // row lists without the twins' entries (a twin has no left neighbour: its whole input column is
  // its column list, skipped)
  for (int t = 0; t < T; ++t) std::fill(rc[t].begin(), rc[t].end(), 0);
  par_columns(N, colptr, T, [&](int t, int j0, int j1) {
    int64_t* r = rc[t].data();
    for (int j = j0; j < j1; ++j) {
      const int b = pinv[j];
      if (twin[b] >= 0) continue;
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
        const int i = rowval[p];
        if (i == j) continue;
        const int a = pinv[i];
        if (twin[std::min(a, b)] < 0) r[std::max(a, b)]++;
      }
    }
  });
  offsets(rc, P.rp);
  P.ri.resize(P.rp[N]);
  par_columns(N, colptr, T, [&](int t, int j0, int j1) {
    int64_t* r = rc[t].data();
    for (int j = j0; j < j1; ++j) {
      const int b = pinv[j];
      if (twin[b] >= 0) continue;
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
        const int i = rowval[p];
        if (i == j) continue;
        const int a = pinv[i];
        const int hi = std::max(a, b), lo = std::min(a, b);
        if (twin[lo] < 0) P.ri[P.rp[hi] + r[hi]++] = lo;
      }
    }
  });
}

// Liu's algorithm over the row lists (twins' entries left out by build_pattern), then the twins
// given their representative's parent
void etree(int N, const Pattern& P, const std::vector<int32_t>& twin, std::vector<int32_t>& parent) {
  parent.assign(N, -1);
  std::vector<int32_t> anc(N, -1);
  for (int k = 0; k < N; ++k)
    for (int64_t p = P.rp[k]; p < P.rp[k + 1]; ++p) {
      int i = P.ri[p];
      while (i != -1 && i < k) {
        int inext = anc[i];
        anc[i] = k;
        if (inext == -1) parent[i] = k;
        i = inext;
      }
    }
  for (int j = 0; j < N; ++j)
    if (twin[j] >= 0) parent[j] = parent[twin[j]];
}

// Postorder of the etree with every node's heaviest child subtree (most columns) visited LAST: the
// parent's first column then follows that child's last one, so relaxed amalgamation (step 4, which
// merges column-adjacent child -> parent pairs only) can merge a front with its main child — a chain
// of tree fronts under a separator becomes fewer, larger fronts (fewer dependent levels on the GPU).
// MADIPM_HEAVY_LAST=0: children in index order.
void postorder(int N, const std::vector<int32_t>& parent, std::vector<int32_t>& post) {
  std::vector<int32_t> head(N, -1), next(N, -1), stack(N);
  const char* hl = std::getenv("MADIPM_HEAVY_LAST");
  if (hl && hl[0] == '0') {
    for (int j = N - 1; j >= 0; --j)
      if (parent[j] != -1) {
        next[j] = head[parent[j]];
        head[parent[j]] = j;
      }
  } else {
    std::vector<int64_t> sz(N, 1);
    for (int j = 0; j < N; ++j)
      if (parent[j] != -1) sz[parent[j]] += sz[j];  // parent[j] > j: children are complete
    std::vector<int32_t> heavy(N, -1);
    for (int j = 0; j < N; ++j) {
      const int p = parent[j];
      if (p != -1 && (heavy[p] == -1 || sz[j] >= sz[heavy[p]])) heavy[p] = j;
    }
    // children in index order, the heavy one moved to the end of its parent's list
    for (int j = N - 1; j >= 0; --j)
      if (parent[j] != -1 && heavy[parent[j]] != j) {
        next[j] = head[parent[j]];
        head[parent[j]] = j;
      }
    std::vector<int32_t> tail(N, -1);
    for (int p = 0; p < N; ++p) {
      const int h = heavy[p];
      if (h == -1) continue;
      if (head[p] == -1) {
        head[p] = h;
      } else {
        int t = head[p];
        while (next[t] != -1) t = next[t];
        next[t] = h;
      }
      next[h] = -1;
    }
  }
  post.assign(N, 0);
  int k = 0;
  for (int j = 0; j < N; ++j) {
    if (parent[j] != -1) continue;
    int top = 0;
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
  }
}

// Column counts of L (diagonal included) for a matrix whose labelling is a postorder of its etree.
// Twins (find_twins): their entries skipped (the other columns' counts are those of the pattern
// without them), their own count set to their representative's.
void column_counts(int N, const Pattern& P, const std::vector<int32_t>& parent, const std::vector<int32_t>& twin,
                   std::vector<int64_t>& cnt) {
  cnt.assign(N, 0);
  std::vector<int32_t> first(N, -1), maxfirst(N, -1), prevleaf(N, -1), anc(N);
  for (int k = 0; k < N; ++k) {
    int j = k;
    cnt[j] = (first[j] == -1) ? 1 : 0;
    for (; j != -1 && first[j] == -1; j = parent[j]) first[j] = k;
  }
  std::iota(anc.begin(), anc.end(), 0);
  for (int j = 0; j < N; ++j) {
    if (parent[j] != -1) cnt[parent[j]]--;
    for (int64_t p = twin[j] >= 0 ? P.cp[j + 1] : P.cp[j]; p < P.cp[j + 1]; ++p) {
      int i = P.ci[p];  // i > j
      if (first[j] <= maxfirst[i]) continue;  // j is not a leaf of the i-th row subtree
      maxfirst[i] = first[j];
      int jprev = prevleaf[i];
      prevleaf[i] = j;
      if (jprev == -1) {
        cnt[j]++;  // first leaf: A(i,j) in the skeleton
      } else {
        int q = jprev;
        while (q != anc[q]) q = anc[q];
        for (int s = jprev, sp; s != q; s = sp) {
          sp = anc[s];
          anc[s] = q;
        }
        cnt[j]++;
        cnt[q]--;  // overlap at the least common ancestor
      }
    }
    if (parent[j] != -1) anc[j] = parent[j];
  }
  for (int j = 0; j < N; ++j)
    if (parent[j] != -1) cnt[parent[j]] += cnt[j];
  for (int j = 0; j < N; ++j)
    if (twin[j] >= 0) cnt[j] = cnt[twin[j]];
}

inline int64_t trap(int64_t w, int64_t r) { return w * r - w * (w - 1) / 2; }

// Everything the analysis needs about one fill-reducing order: the order relabelled as a postorder
// of its etree, the strictly-lower pattern in that labelling, the etree, the column counts of L and
// the factorisation flops sum_j (c_j - 1)(c_j + 2).  Candidate orders are compared by flops and the
// winner's analysis is kept (no second pass over the matrix for it).
struct OrderAnalysis {
  std::vector<int32_t> perm, pinv, parent, twin;
  std::vector<int64_t> cnt;
  Pattern P;
  double flops = 0.0;
};

void analyse_order(int N, const int64_t* colptr, const int32_t* rowval, std::vector<int32_t> perm,
                   OrderAnalysis& A) {
  const bool timing = std::getenv("MADIPM_SYMBOLIC_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  analyse_order %-20s %9.3f s\n", what, std::chrono::duration<double>(t - t_last).count());
    t_last = t;
  };
  A.pinv.assign(N, -1);
  for (int k = 0; k < N; ++k) {
    MADIPM_REQUIRE(perm[k] >= 0 && perm[k] < N && A.pinv[perm[k]] == -1, "ordering is not a permutation");
    A.pinv[perm[k]] = k;
  }
  std::vector<int32_t> post;
  std::vector<int32_t>& twin = A.twin;
  build_pattern(N, colptr, rowval, A.pinv, A.P, twin);
  stamp("pattern + twin leaves");
  etree(N, A.P, twin, A.parent);
  stamp("etree");
  postorder(N, A.parent, post);
  bool ident = true;  // the ordering is already a postorder (e.g. natural order of a QP's K2): no relabel
  for (int k = 0; k < N && ident; ++k) ident = post[k] == k;
  if (!ident) {
    std::vector<int32_t> perm2(N);
    for (int k = 0; k < N; ++k) perm2[k] = perm[post[k]];
    perm.swap(perm2);
    for (int k = 0; k < N; ++k) A.pinv[perm[k]] = k;
    build_pattern(N, colptr, rowval, A.pinv, A.P, twin);
    etree(N, A.P, twin, A.parent);
  }
  A.perm.swap(perm);
  stamp("postorder/relabel");
  column_counts(N, A.P, A.parent, twin, A.cnt);
  stamp("column counts");
  A.flops = 0.0;
  for (int64_t c : A.cnt) A.flops += (double)(c - 1) * (double)(c + 2);
}

}  // namespace

void symbolic_analyze(int N, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& opt,
                      const int32_t* user_perm, SymbolicPlan& S) {
  S = SymbolicPlan();
  MADIPM_REQUIRE(N >= 0, "negative dimension");
  // MADIPM_SYMBOLIC_TIMING=1: wall time of each step on stderr (diagnostics)
  const bool timing = std::getenv("MADIPM_SYMBOLIC_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "symbolic %-28s %9.3f s\n", what, std::chrono::duration<double>(t - t_last).count());
    t_last = t;
  };
  S.N = N;
  const int64_t nnz = colptr[N];
  S.nnzK = nnz;
  MADIPM_REQUIRE(colptr[0] == 0, "colptr[0] must be 0");
  std::vector<int64_t> diagcount(N, 0);
  // Either triangle is accepted (LDLFactorizations takes the upper one, MadNLP's aug_com the lower
  // one), even mixed, as long as every off-diagonal pair {i, j} is stored in one triangle only:
  // the factorisation maps each entry to its symmetric position, so a full symmetric matrix would
  // be counted twice and is rejected.
  bool has_upper = false;
  for (int j = 0; j < N; ++j) MADIPM_REQUIRE(colptr[j + 1] >= colptr[j], "colptr not monotone");
  {
    const int T = nnz < ((int64_t)1 << 22) ? 1 : analysis_threads();
    std::vector<uint8_t> up(T, 0), bad(T, 0);
    par_columns(N, colptr, T, [&](int t, int j0, int j1) {
      bool b = false, u = false;  // thread-local: no shared line written per entry
      for (int j = j0; j < j1; ++j) {
        int64_t d = 0;
        for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
          const int i = rowval[p];
          b |= i < 0 || i >= N;
          d += i == j;
          u |= i < j;
        }
        diagcount[j] = d;
      }
      bad[t] = b;
      up[t] = u;
    });
    for (int t = 0; t < T; ++t) {
      MADIPM_REQUIRE(!bad[t], "row index out of range");
      has_upper = has_upper || up[t];
    }
  }
  if (has_upper) {
    // pairs stored above the diagonal must not also be stored below it
    std::vector<int64_t> up_ptr(N + 1, 0);
    for (int j = 0; j < N; ++j)
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p)
        if (rowval[p] < j) up_ptr[rowval[p] + 1]++;  // (i, j), i < j  ->  bucket i, value j
    for (int i = 0; i < N; ++i) up_ptr[i + 1] += up_ptr[i];
    std::vector<int32_t> up(up_ptr[N]);
    std::vector<int64_t> fillu(up_ptr.begin(), up_ptr.end() - 1);
    for (int j = 0; j < N; ++j)
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p)
        if (rowval[p] < j) up[fillu[rowval[p]]++] = j;
    std::vector<int32_t> mark(N, -1);
    for (int j = 0; j < N; ++j) {  // column j's lower entries (i, j), i > j, vs the upper (j, i)
      for (int64_t q = up_ptr[j]; q < up_ptr[j + 1]; ++q) mark[up[q]] = j;
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p)
        MADIPM_REQUIRE(!(rowval[p] > j && mark[rowval[p]] == j),
                       "entry (" + std::to_string(rowval[p]) + "," + std::to_string(j) +
                           ") is stored in both triangles: pass one triangle of the symmetric matrix");
    }
  }
  if (N == 0) return;

  stamp("before 1");
  // ---------------- 1. fill-reducing ordering; 2. etree + postorder (relabel so that the labelling
  // is a postorder) and column counts of the chosen order
  OrderAnalysis OA;
  S.order_flops_amd = S.order_flops_nd = 0.0;
  if (opt.ordering == 1 || opt.ordering == 3 || opt.ordering == 4) {
    std::vector<int64_t> Ap(N + 1, 0);
    for (int j = 0; j < N; ++j)
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
        int i = rowval[p];
        if (i == j) continue;
        Ap[i + 1]++;
        Ap[j + 1]++;
      }
    for (int j = 0; j < N; ++j) Ap[j + 1] += Ap[j];
    std::vector<int32_t> Ai(Ap[N]);
    std::vector<int64_t> fill(Ap.begin(), Ap.end() - 1);
    for (int j = 0; j < N; ++j)
      for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
        int i = rowval[p];
        if (i == j) continue;
        Ai[fill[i]++] = j;
        Ai[fill[j]++] = i;
      }
    std::vector<int64_t>().swap(fill);
    // Nested dissection is randomised (matchings, initial partitions).  On graphs with more than
    // kBigAdj adjacency entries its fill varies with the seed far more than with anything else (neos
    // stand-in: 240-323 GFLOP over seeds; ex10 and supportcase10, below the bound: within 0.5 %), so
    // there it runs with kNdSeeds fixed seeds at once — each free to use all the analysis threads —
    // and the order with the fewest flops is kept (lowest seed on ties: the same choice whatever the
    // thread count).  ordering = auto adds AMD (one thread) beside ND and keeps the overall best; AMD
    // is skipped above kBigAdj, where it is the slowest step of the analysis and ND wins anyway on
    // the benchmark LPs (AMD vs ND flops: ex10 4.5e10 vs 2.6e8, supportcase10 6.0e8 vs 3.4e8, neos
    // 4.2e11 vs 2.5e11; the neos stand-in at scale 0.1: AMD 1.9e10 vs ND 3.6e10).  Once ND's order is
    // analysed, AMD stops as soon as a lower bound of its flops exceeds ND's (amd_order's cap: it
    // could only lose — the choice is the one without the stop; ex10's AMD took 0.62 s beside ~0.4 s
    // of ND).  Every candidate is analysed in full (etree + column counts).
    constexpr int kNdSeeds = 4;
    constexpr int64_t kBigAdj = 4000000, kNdSeedsMaxAdj = 40000000;
    std::vector<int32_t> pa;
    const bool use_nd = opt.ordering != 1;
    const bool use_amd = opt.ordering == 1 || (opt.ordering == 4 && Ap[N] <= kBigAdj);
    const int nseeds = use_nd ? (Ap[N] > kBigAdj && Ap[N] <= kNdSeedsMaxAdj ? kNdSeeds : 1) : 0;
    std::vector<OrderAnalysis> B(nseeds);
    OrderAnalysis A;
    const int T = analysis_threads();
    // every seed may use all the threads: the seeds finish ~0.5 s apart on neos, and a fixed share
    // each left the early finishers' cores idle (box, neos symbolic: 2.27-2.44 s with T / 4 threads
    // per seed, 2.03-2.13 s with T; the order does not depend on the thread count)
    const int per = std::max(1, T - (use_amd ? 1 : 0));
    auto run_nd = [&](int k) {
      NDOptions nopt;
      nopt.dense_alpha = opt.dense_alpha;
      nopt.threads = per;
      nopt.seed = 12345 + (uint64_t)k;
      // with several seeds, one bisection per subgraph: the seeds are the tries (neos: the same best
      // order with 1, 2 or 3 tries per seed, a third of the top-level work)
      if (nseeds > 1) nopt.tries = 1;
      std::vector<int32_t> pn;
      nd_order(N, Ap, Ai, pn, nopt);
      analyse_order(N, colptr, rowval, std::move(pn), B[k]);
    };
    std::vector<std::thread> th;
    std::atomic<double> amd_cap{std::numeric_limits<double>::infinity()};
    bool amd_done = true;
    if (use_amd)
      th.emplace_back([&] {
        amd_done = amd_order(N, Ap, Ai, pa, opt.dense_alpha, use_nd ? &amd_cap : nullptr);
        if (amd_done)
          analyse_order(N, colptr, rowval, std::move(pa), A);
        else
          A.flops = std::numeric_limits<double>::infinity();  // stopped: it could not beat ND
      });
    for (int k = 1; k < nseeds; ++k) th.emplace_back(run_nd, k);
    if (nseeds) {
      run_nd(0);
      if (nseeds == 1) amd_cap.store(B[0].flops);  // (seeds > 1: no AMD, kBigAdj)
    }
    for (auto& x : th) x.join();
    stamp("1: orderings (ND seeds, AMD) + analysis");
    std::vector<int64_t>().swap(Ap);
    std::vector<int32_t>().swap(Ai);
    int best = -1;
    for (int k = 0; k < nseeds; ++k)
      if (best < 0 || B[k].flops < B[best].flops) best = k;
    if (use_amd) S.order_flops_amd = A.flops;
    if (best >= 0) S.order_flops_nd = B[best].flops;
    if (best >= 0 && (!use_amd || B[best].flops < A.flops))
      std::swap(OA, B[best]);
    else
      std::swap(OA, A);
  } else if (opt.ordering == 2) {
    MADIPM_REQUIRE(user_perm != nullptr, "user permutation missing");
    analyse_order(N, colptr, rowval, std::vector<int32_t>(user_perm, user_perm + N), OA);
  } else {
    std::vector<int32_t> id(N);
    std::iota(id.begin(), id.end(), 0);
    analyse_order(N, colptr, rowval, std::move(id), OA);
  }
  stamp("2: etree, counts");
  const bool use_lb = opt.leaf_batch && !has_upper;
  struct SN {
    int first, w;
    int64_t r, zeros;
  };
  double bigm = opt.big_merge;
  if (const char* e = std::getenv("MADIPM_BIG_MERGE")) bigm = std::atof(e);
  // the trailing update's flops (2 w per entry of the (r - w) x (r - w) lower triangle)
  auto upd_flops = [](int64_t w, int64_t r) { return 2.0 * (double)w * (double)(r - w) * (double)(r - w + 1) / 2.0; };
  std::vector<int32_t> nchild;
  std::vector<uint8_t> lbcand;
  std::vector<SN> sn;
  // steps 3 - 4 (fundamental supernodes, batched-leaf candidates, relaxed amalgamation) of an order
  auto amalgamate = [&](const OrderAnalysis& A) {
    const std::vector<int32_t>& parent = A.parent;
    const std::vector<int64_t>& cnt = A.cnt;
    stamp("before 3");
    // ---------------- 3. fundamental supernodes
    nchild.assign(N, 0);
    for (int j = 0; j < N; ++j)
      if (parent[j] != -1) nchild[parent[j]]++;
    std::vector<SN> fund;
    fund.push_back({0, 1, cnt[0], 0});
    for (int j = 1; j < N; ++j) {
      if (parent[j - 1] == j && cnt[j - 1] == cnt[j] + 1 && nchild[j] == 1) {
        fund.back().w++;
      } else {
        fund.push_back({j, 1, cnt[j], 0});
      }
    }

    stamp("before 3b");
    // ---------------- 3b. batched-leaf candidates: single-column etree leaves with a large update,
    // many under the same parent column (a QP with a diagonal Hessian and dense A: every x_j).  They
    // are kept out of relaxed amalgamation; step 6b decides the groups.
    lbcand.assign(N, 0);
    // batched leaves read their K column as one contiguous CSC run (diagonal + rows below): lower only
    if (use_lb) {
      std::vector<int32_t> npar(N, 0);
      for (const SN& f : fund)
        if (f.w == 1 && nchild[f.first] == 0 && f.r - 1 >= opt.lb_min_rows && parent[f.first] != -1)
          npar[parent[f.first]]++;
      for (const SN& f : fund)
        if (f.w == 1 && nchild[f.first] == 0 && f.r - 1 >= opt.lb_min_rows && parent[f.first] != -1 &&
            npar[parent[f.first]] >= opt.lb_min_count)
          lbcand[f.first] = 1;
    }

    stamp("before 4");
    // ---------------- 4. relaxed amalgamation (merge a front with its column-adjacent child)
    sn.clear();
    sn.reserve(fund.size());
    for (const SN& f : fund) {
      SN p = f;
      while ((opt.relax || bigm > 0.0) && !sn.empty()) {
        const SN& c = sn.back();
        int clast = c.first + c.w - 1;
        if (clast + 1 != p.first) break;
        if (lbcand[c.first] || lbcand[p.first]) break;  // batched-leaf candidates stay single columns
        int par = parent[clast];
        if (par < p.first || par >= p.first + p.w) break;
        int64_t ncols = c.w + p.w;
        int64_t rnew = c.w + p.r;
        int64_t Enew = trap(ncols, rnew);
        int64_t zeros = Enew - (trap(c.w, c.r) - c.zeros) - (trap(p.w, p.r) - p.zeros);
        double frac = (double)zeros / (double)Enew;
        bool merge = opt.relax && (ncols <= opt.nrelax[0] || (ncols <= opt.nrelax[1] && frac < opt.zrelax[0]) ||
                                   (ncols <= opt.nrelax[2] && frac < opt.zrelax[1]) || frac < opt.zrelax[2]);
        if (!merge && bigm > 0.0 && c.r > opt.big_merge_rows) {
          // the child's update block: written once, read once by the parent's assembly; the zeros: written
          // by the factorisation, read by the two sweeps of each of ~2 solves
          const double u = (double)(c.r - c.w), saved = 16.0 * u * (u + 1) / 2.0, zbytes = 5.0 * 8.0 * (double)zeros;
          const double xfl = upd_flops(ncols, rnew) - upd_flops(c.w, c.r) - upd_flops(p.w, p.r);
          merge = saved - zbytes > xfl / bigm;
        }
        if (!merge) break;
        p.first = c.first;
        p.w = (int)ncols;
        p.r = rnew;
        p.zeros = zeros;
        sn.pop_back();
      }
      sn.push_back(p);
    }
  };
  amalgamate(OA);
  if (bigm > 0.0) {
    // 2b. sibling merges: relaxed amalgamation merges a front with its column-ADJACENT child only (the
    // last one in postorder), so of a parent's children with HBM-sized update blocks (more than
    // big_merge_rows rows) all but one would write their block for the parent to read back.  Reorder:
    // every such child's own columns (with those of its merged descendants) are moved to right before
    // its parent's, the largest last; the rest of its subtree stays where it was.  The order stays an
    // elimination order of the same etree (every column still follows its descendants: same fill,
    // counts and tree), and step 4's cost rule then merges the moved children one after the other.
    // A moved child that the rule does not merge would split its subtree's label range: those are
    // kept in place and the order is rebuilt (a few rounds), else the reorder is dropped.
    const std::vector<int32_t>& par0 = OA.parent;
    const std::vector<int64_t>& cnt0 = OA.cnt;
    std::vector<uint8_t> delay(N, 0);
    bool any = false;
    for (int j = 0; j < N; ++j)
      if (par0[j] != -1 && cnt0[j] > opt.big_merge_rows && !lbcand[j]) any = delay[j] = 1;
    std::vector<int32_t> chead(N, -1), cnext(N, -1), dhead(N, -1), dnext(N, -1), dl, order, newpos(N), stk;
    for (int attempt = 0; any && attempt < 4; ++attempt) {
      // children lists in label order; delayed children (also) in (count, label) order
      std::fill(chead.begin(), chead.end(), -1);
      std::fill(dhead.begin(), dhead.end(), -1);
      for (int c = N - 1; c >= 0; --c)
        if (par0[c] != -1) {
          cnext[c] = chead[par0[c]];
          chead[par0[c]] = c;
        }
      dl.clear();
      for (int c = 0; c < N; ++c)
        if (delay[c]) dl.push_back(c);
      std::stable_sort(dl.begin(), dl.end(), [&](int a, int b) { return cnt0[a] < cnt0[b]; });
      for (int q = (int)dl.size() - 1; q >= 0; --q) {
        const int c = dl[q];
        dnext[c] = dhead[par0[c]];
        dhead[par0[c]] = c;
      }
      // emission: full(v) = early(v) + late(v); early(v) = per child c: c delayed ? early(c) : full(c);
      // late(v) = late(d) per delayed child d (sorted), then v.  Explicit stack of (node, kind) tasks.
      enum { FULL = 0, EARLY = 1, LATE = 2, OUT = 3 };
      order.clear();
      order.reserve(N);
      for (int root = 0; root < N; ++root) {
        if (par0[root] != -1) continue;
        stk.push_back(root * 4 + FULL);
        while (!stk.empty()) {
          const int t = stk.back(), v = t >> 2, kind = t & 3;
          stk.pop_back();
          if (kind == OUT) {
            order.push_back(v);
          } else if (kind == FULL) {
            stk.push_back(v * 4 + LATE);
            stk.push_back(v * 4 + EARLY);
          } else if (kind == EARLY) {  // children pushed last-first: popped in label order
            size_t m = stk.size();
            for (int c = chead[v]; c != -1; c = cnext[c]) stk.push_back(c * 4 + (delay[c] ? EARLY : FULL));
            std::reverse(stk.begin() + m, stk.end());
          } else {
            stk.push_back(v * 4 + OUT);
            size_t m = stk.size();
            for (int d = dhead[v]; d != -1; d = dnext[d]) stk.push_back(d * 4 + LATE);
            std::reverse(stk.begin() + m, stk.end());
          }
        }
      }
      MADIPM_REQUIRE((int)order.size() == N && N < (1 << 29), "merge reorder");
      OrderAnalysis B;
      B.perm.resize(N);
      B.pinv.resize(N);
      for (int k = 0; k < N; ++k) {
        newpos[order[k]] = k;
        B.perm[k] = OA.perm[order[k]];
        B.pinv[B.perm[k]] = k;
      }
      B.parent.resize(N);
      B.cnt.resize(N);
      for (int k = 0; k < N; ++k) {
        const int p = par0[order[k]];
        B.parent[k] = p == -1 ? -1 : newpos[p];
        B.cnt[k] = cnt0[order[k]];
      }
      B.flops = OA.flops;
      build_pattern(N, colptr, rowval, B.pinv, B.P, B.twin);
      amalgamate(B);
      // every moved child merged into its parent's front?
      std::vector<int32_t> sof(N);
      for (int q = 0; q < (int)sn.size(); ++q)
        for (int j = sn[q].first; j < sn[q].first + sn[q].w; ++j) sof[j] = q;
      bool ok = true;
      for (int c = 0; c < N; ++c)
        if (delay[c] && sof[newpos[c]] != sof[newpos[par0[c]]]) {
          delay[c] = 0;
          ok = false;
        }
      if (ok) {
        std::swap(OA, B);
        break;
      }
      any = false;
      for (int c = 0; c < N && !any; ++c) any = delay[c];
      if (!any || attempt == 3) amalgamate(OA);  // back to the unmoved order
    }
    stamp("2b: sibling-merge order");
  }
  std::vector<int32_t>& perm = OA.perm;
  std::vector<int32_t>& pinv = OA.pinv;
  std::vector<int32_t>& parent = OA.parent;
  std::vector<int64_t>& cnt = OA.cnt;
  Pattern& P = OA.P;
  S.perm = perm;
  S.pinv = pinv;
  S.nnzL = std::accumulate(cnt.begin(), cnt.end(), (int64_t)0);
  S.colcnt.resize(N);
  S.kcol.resize(N);
  for (int j = 0; j < N; ++j) {
    S.colcnt[j] = (int32_t)cnt[j];
    S.kcol[j] = (int32_t)(P.cp[j + 1] - P.cp[j] + (diagcount[perm[j]] ? 1 : 0));
  }

  const int ns = (int)sn.size();
  S.nsuper = ns;
  S.first.resize(ns + 1);
  std::vector<int32_t> col2sn(N);
  for (int s = 0; s < ns; ++s) {
    S.first[s] = sn[s].first;
    for (int j = sn[s].first; j < sn[s].first + sn[s].w; ++j) col2sn[j] = s;
  }
  S.first[ns] = N;
  S.parent.assign(ns, -1);
  for (int s = 0; s < ns; ++s) {
    int last = S.first[s + 1] - 1;
    if (parent[last] != -1) S.parent[s] = col2sn[parent[last]];
    MADIPM_REQUIRE(S.parent[s] == -1 || S.parent[s] > s, "supernodal tree is not postordered");
  }
  S.child_ptr.assign(ns + 1, 0);
  for (int s = 0; s < ns; ++s)
    if (S.parent[s] != -1) S.child_ptr[S.parent[s] + 1]++;
  for (int s = 0; s < ns; ++s) S.child_ptr[s + 1] += S.child_ptr[s];
  S.child_list.resize(S.child_ptr[ns]);
  {
    std::vector<int32_t> fillc(S.child_ptr.begin(), S.child_ptr.end() - 1);
    for (int s = 0; s < ns; ++s)
      if (S.parent[s] != -1) S.child_list[fillc[S.parent[s]]++] = s;
  }

  // ---------------- 4b. batched-leaf groups, decided from the pattern before any row structure is
  // built: per parent, its candidate children whose K column is one CSC column of the caller
  // (diagonal + rows below, none to its left) and whose rows cover at least lb_min_density of the
  // union of their rows.  A member's rows are its L column's (a leaf: its K column's below the
  // diagonal, P's column list); the members keep only their pivot row as front structure (nrows 1):
  // their factor is the group's W, and on a dense-column QP their m-row lists were the analysis' bulk
  // (dense QP 50k x 10k: 5e8 row entries materialised, copied, relative-indexed and gathered).
  S.lb.clear();
  S.lb_of.assign(ns, -1);
  std::vector<std::vector<int32_t>> lb_members_of;  // per group: member fronts
  std::vector<std::vector<int32_t>> lb_union;       // per group: union of the members' rows (ascending)
  std::vector<int32_t> lb_group_of_parent(ns, -1);
  std::vector<uint8_t> has_left;
  if (use_lb) {
    has_left.assign(N, 0);
    {  // per-thread flags, OR-ed (order-free)
      const int T = nnz < ((int64_t)1 << 22) ? 1 : analysis_threads();
      std::vector<std::vector<uint8_t>> hl(T, std::vector<uint8_t>(N, 0));
      par_columns(N, colptr, T, [&](int t, int j0, int j1) {
        uint8_t* h = hl[t].data();
        for (int j = j0; j < j1; ++j)
          for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p)
            if (rowval[p] != j) h[rowval[p]] = 1;
      });
      for (int t = 0; t < T; ++t)
        for (int i = 0; i < N; ++i) has_left[i] |= hl[t][i];
    }
    std::vector<int32_t> seen(N, -1);
    std::vector<uint8_t> inmem(N, 0);
    for (int s = 0; s < ns; ++s) {
      std::vector<int32_t> mem;
      for (int64_t q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q) {
        const int c = S.child_list[q];
        const int oc = perm[S.first[c]];
        if (S.first[c + 1] - S.first[c] == 1 && lbcand[S.first[c]] && !has_left[oc] &&
            S.child_ptr[c + 1] == S.child_ptr[c])
          mem.push_back(c);
      }
      if ((int)mem.size() < opt.lb_min_count) continue;
      std::vector<int32_t> U;
      int64_t tot = 0;
      for (int c : mem) inmem[S.first[c]] = 1;
      for (int c : mem) {
        const int j = S.first[c];
        tot += P.cp[j + 1] - P.cp[j];
        if (OA.twin[j] >= 0 && inmem[OA.twin[j]]) continue;  // its rows are its representative's
        for (int64_t p = P.cp[j]; p < P.cp[j + 1]; ++p)
          if (seen[P.ci[p]] != s) {
            seen[P.ci[p]] = s;
            U.push_back(P.ci[p]);
          }
      }
      for (int c : mem) inmem[S.first[c]] = 0;
      const double dens = (double)tot / ((double)U.size() * (double)mem.size());
      if (dens < opt.lb_min_density) continue;
      std::sort(U.begin(), U.end());
      lb_group_of_parent[s] = (int32_t)lb_members_of.size();
      for (int c : mem) S.lb_of[c] = (int32_t)lb_members_of.size();
      lb_members_of.push_back(std::move(mem));
      lb_union.push_back(std::move(U));
    }
  }
  auto lb_member = [&](int s) { return !S.lb_of.empty() && S.lb_of[s] >= 0; };

  stamp("before 5");
  // ---------------- 5. frontal row structures
  S.row_ptr.assign(ns + 1, 0);
  S.nrows.resize(ns);
  std::vector<int32_t> marker(N, -1);
  std::vector<std::vector<int32_t>> R(ns);
  for (int s = 0; s < ns; ++s) {
    int f = S.first[s], l = S.first[s + 1];
    std::vector<int32_t>& rs = R[s];
    for (int j = f; j < l; ++j) {
      rs.push_back(j);
      marker[j] = s;
    }
    size_t nown = rs.size();
    if (lb_member(s)) {  // batched leaf: pivot row only (its rows are its group's business)
      S.nrows[s] = 1;
      S.row_ptr[s + 1] = S.row_ptr[s] + 1;
      continue;
    }
    for (int j = f; j < l; ++j)
      for (int64_t p = P.cp[j]; p < P.cp[j + 1]; ++p) {
        int i = P.ci[p];
        if (i >= l && marker[i] != s) {
          marker[i] = s;
          rs.push_back(i);
        }
      }
    if (lb_group_of_parent[s] >= 0)
      for (int i : lb_union[lb_group_of_parent[s]])
        if (i >= l && marker[i] != s) {
          marker[i] = s;
          rs.push_back(i);
        }
    for (int64_t q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q) {
      int c = S.child_list[q];
      if (lb_member(c)) continue;
      const std::vector<int32_t>& rc = R[c];
      int wc = S.first[c + 1] - S.first[c];
      for (size_t t = wc; t < rc.size(); ++t) {
        int i = rc[t];
        MADIPM_REQUIRE(i >= f, "child row structure escapes its parent");
        if (i >= l && marker[i] != s) {
          marker[i] = s;
          rs.push_back(i);
        }
      }
    }
    if (!std::is_sorted(rs.begin() + nown, rs.end())) std::sort(rs.begin() + nown, rs.end());
    S.nrows[s] = (int32_t)rs.size();
    S.row_ptr[s + 1] = S.row_ptr[s] + (int64_t)rs.size();
  }
  S.rows.resize(S.row_ptr[ns]);
  for (int s = 0; s < ns; ++s) std::copy(R[s].begin(), R[s].end(), S.rows.begin() + S.row_ptr[s]);

  stamp("before 6");
  // ---------------- 6. relative indices child -> parent
  S.rel_ptr.assign(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    int w = S.first[s + 1] - S.first[s];
    S.rel_ptr[s + 1] = S.rel_ptr[s] + (S.nrows[s] - w);
  }
  S.rel.resize(S.rel_ptr[ns]);
  std::vector<int32_t> pos(N, -1);
  for (int s = 0; s < ns; ++s) {
    for (int64_t t = S.row_ptr[s]; t < S.row_ptr[s + 1]; ++t) pos[S.rows[t]] = (int32_t)(t - S.row_ptr[s]);
    for (int64_t q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q) {
      int c = S.child_list[q];
      int wc = S.first[c + 1] - S.first[c];
      for (int t = wc; t < S.nrows[c]; ++t) {
        int row = S.rows[S.row_ptr[c] + t];
        int ps = pos[row];
        MADIPM_REQUIRE(ps >= 0 && S.rows[S.row_ptr[s] + ps] == row, "relative index lookup failed");
        S.rel[S.rel_ptr[c] + (t - wc)] = ps;
      }
    }
  }

  stamp("before 6b");
  // ---------------- 6b. batched-leaf group tables (groups decided in 4b): W rows = the union U in
  // parent-local positions (gpos), and for every entry of a member's caller CSC column its W row
  if (!lb_members_of.empty()) {
    std::vector<int32_t> pos_in_u;
    for (size_t gi = 0; gi < lb_members_of.size(); ++gi) {
      const std::vector<int32_t>& mem = lb_members_of[gi];
      const std::vector<int32_t>& U = lb_union[gi];
      const int s = S.parent[mem[0]];
      for (int64_t t = S.row_ptr[s]; t < S.row_ptr[s + 1]; ++t) pos[S.rows[t]] = (int32_t)(t - S.row_ptr[s]);
      SymbolicPlan::LBGroup g{};
      g.parent = s;
      g.m = (int32_t)U.size();
      g.n = (int32_t)mem.size();
      g.w_off = S.lb_wsize;
      g.mem_off = (int64_t)S.lb_mem.size();
      g.gpos_off = (int64_t)S.lb_gpos.size();
      S.lb_wsize += (int64_t)g.m * g.n;
      pos_in_u.assign(S.nrows[s], -1);
      for (int k = 0; k < g.m; ++k) {
        const int lr = pos[U[k]];
        MADIPM_REQUIRE(lr >= 0 && S.rows[S.row_ptr[s] + lr] == U[k], "batched leaf: row outside its parent");
        S.lb_gpos.push_back(lr);
        pos_in_u[lr] = k;
      }
      const size_t m0 = S.lb_mem.size();
      const int T = std::min<int>(analysis_threads(), std::max<int>(1, (int)(mem.size() / 64)));
      // a member whose CSC column has the previous member's rows (its own diagonal at the same
      // position) shares that member's W-row map (dense QP: one map of m + 1 entries, not 5e8)
      std::vector<uint8_t> same(mem.size(), 0);
      {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&, t]() {
            for (size_t k = 1 + t; k < mem.size(); k += T) {
              const int oa = perm[S.first[mem[k - 1]]], ob = perm[S.first[mem[k]]];
              const int64_t len = colptr[oa + 1] - colptr[oa];
              if (colptr[ob + 1] - colptr[ob] != len) continue;
              const int32_t* a = rowval + colptr[oa];
              const int32_t* b = rowval + colptr[ob];
              int64_t p = 0;
              for (; p < len && (a[p] == b[p] || (a[p] == oa && b[p] == ob)); ++p) {
              }
              same[k] = p == len;
            }
          });
        for (auto& x : th) x.join();
      }
      int64_t wtot = (int64_t)S.lb_wrow.size();
      for (size_t k = 0; k < mem.size(); ++k) {
        const int oc = perm[S.first[mem[k]]];
        S.lb_mem.push_back(S.first[mem[k]]);
        S.lb_cs.push_back(colptr[oc]);
        S.lb_ce.push_back(colptr[oc + 1]);
        if (same[k]) {
          S.lb_wbase.push_back(S.lb_wbase.back());
        } else {
          S.lb_wbase.push_back(wtot);
          wtot += colptr[oc + 1] - colptr[oc];
        }
      }
      S.lb_wrow.resize(wtot);  // once (the threads below fill it)
      // every entry of the distinct members' CSC columns -> its W row (threads over members)
      std::vector<std::thread> th;
      bool bad = false;
      std::vector<uint8_t> badt(T, 0);
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
          for (size_t q = m0 + t; q < m0 + mem.size(); q += T) {
            if (same[q - m0]) continue;
            const int oc = perm[S.lb_mem[q]];
            int32_t* wr = S.lb_wrow.data() + S.lb_wbase[q];
            for (int64_t e = colptr[oc]; e < colptr[oc + 1]; ++e) {
              const int i = rowval[e];
              int32_t v = -1;
              if (i != oc) {
                const int lr = pos[pinv[i]];
                if (lr < 0 || pos_in_u[lr] < 0) badt[t] = 1;
                v = lr >= 0 ? pos_in_u[lr] : -1;
              }
              wr[e - colptr[oc]] = v;
            }
          }
        });
      for (auto& x : th) x.join();
      for (uint8_t b : badt) bad = bad || b;
      MADIPM_REQUIRE(!bad, "batched leaf: row outside its parent");
      S.lb.push_back(g);
    }
  }

  stamp("before 7");
  // ---------------- 7. assembly map: caller's CSC entry -> (front, local offset)
  // (entries of batched-leaf members are read by the W build instead)
  // (threads: entries by column ranges with per-thread front counts, then fronts dealt to threads;
  // the same map as one pass)
  S.asm_ptr.assign(ns + 1, 0);
  // per entry (a, b) = (row, column) in the permuted lower triangle; uninitialised storage, touched
  // only for the entries of non-member columns (a batched-leaf member's column is all W entries)
  std::unique_ptr<int32_t[]> ea_buf(new int32_t[std::max<int64_t>(nnz, 1)]), eb_buf(new int32_t[std::max<int64_t>(nnz, 1)]);
  int32_t* ea = ea_buf.get();
  int32_t* eb = eb_buf.get();
  auto member_col = [&](int j) { return lb_member(col2sn[pinv[j]]); };
  int TA = analysis_threads();
  if (nnz < ((int64_t)1 << 19) || (int64_t)TA * (ns + N) > (int64_t)1 << 27) TA = 1;
  std::vector<std::vector<int64_t>> acnt(TA, std::vector<int64_t>(ns + 1, 0));
  par_columns(N, colptr, TA, [&](int t, int j0, int j1) {
    int64_t* cnt_t = acnt[t].data();
    for (int j = j0; j < j1; ++j)
      for (int64_t p = member_col(j) ? colptr[j + 1] : colptr[j]; p < colptr[j + 1]; ++p) {
        int a = pinv[rowval[p]], b = pinv[j];
        if (a < b) std::swap(a, b);
        ea[p] = a;
        eb[p] = b;
        if (lb_member(col2sn[b])) {
          eb[p] = -1;
          continue;
        }
        cnt_t[col2sn[b]]++;
      }
  });
  for (int s = 0; s < ns; ++s) {
    int64_t acc = 0;
    for (int t = 0; t < TA; ++t) {
      const int64_t c = acnt[t][s];
      acnt[t][s] = acc;
      acc += c;
    }
    S.asm_ptr[s + 1] = S.asm_ptr[s] + acc;
  }
  const int64_t nasm = S.asm_ptr[ns];
  S.asm_src.resize(nasm);
  S.asm_dst.resize(nasm);
  {
    std::vector<int64_t> byfront(nasm);
    par_columns(N, colptr, TA, [&](int t, int j0, int j1) {
      int64_t* off = acnt[t].data();
      for (int j = j0; j < j1; ++j) {
        if (member_col(j)) continue;
        for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p)
          if (eb[p] >= 0) {
            const int sf = col2sn[eb[p]];
            byfront[S.asm_ptr[sf] + off[sf]++] = p;
          }
      }
    });
    std::vector<std::thread> th;
    std::vector<uint8_t> bad_row(TA, 0), dup(TA, 0);
    for (int t = 0; t < TA; ++t)
      th.emplace_back([&, t]() {
        std::vector<int32_t> lpos(N, -1);
        std::vector<std::pair<int64_t, int64_t>> d;
        for (int s = t; s < ns; s += TA) {
          const int r = S.nrows[s];
          for (int64_t q = S.row_ptr[s]; q < S.row_ptr[s + 1]; ++q) lpos[S.rows[q]] = (int32_t)(q - S.row_ptr[s]);
          d.clear();
          for (int64_t q = S.asm_ptr[s]; q < S.asm_ptr[s + 1]; ++q) {
            const int64_t p = byfront[q];
            const int lc = eb[p] - S.first[s];
            const int lr = lpos[ea[p]];
            if (lr < 0) bad_row[t] = 1;
            d.emplace_back((int64_t)lc * r + lr, p);
          }
          // sort by destination (the big-front assembly binary-searches column ranges) and reject
          // duplicates, which would race in the parallel assembly
          std::sort(d.begin(), d.end());
          for (size_t u = 0; u < d.size(); ++u) {
            if (u > 0 && d[u].first == d[u - 1].first) dup[t] = 1;
            S.asm_dst[S.asm_ptr[s] + u] = d[u].first;
            S.asm_src[S.asm_ptr[s] + u] = d[u].second;
          }
          for (int64_t q = S.row_ptr[s]; q < S.row_ptr[s + 1]; ++q) lpos[S.rows[q]] = -1;
        }
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < TA; ++t) {
      MADIPM_REQUIRE(!bad_row[t], "assembly row not in front");
      MADIPM_REQUIRE(!dup[t], "duplicate entries in the CSC input (a pair {i, j} stored twice)");
    }
  }

  stamp("before 8");
  // ---------------- 8. level schedule (height in the supernodal tree)
  S.level.assign(ns, 0);
  int maxlev = 0;
  for (int s = 0; s < ns; ++s) {
    int lv = 0;
    for (int64_t q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q) lv = std::max(lv, S.level[S.child_list[q]] + 1);
    S.level[s] = lv;
    maxlev = std::max(maxlev, lv);
  }
  S.nlevels = maxlev + 1;
  S.level_ptr.assign(S.nlevels + 1, 0);
  for (int s = 0; s < ns; ++s) S.level_ptr[S.level[s] + 1]++;
  for (int l = 0; l < S.nlevels; ++l) S.level_ptr[l + 1] += S.level_ptr[l];
  S.level_list.resize(ns);
  {
    std::vector<int32_t> fl(S.level_ptr.begin(), S.level_ptr.end() - 1);
    for (int s = 0; s < ns; ++s) S.level_list[fl[S.level[s]]++] = s;
  }

  stamp("before 8b");
  // ---------------- 8b. subtree sharding (SURVEY §8 e).  cost(s) ~ factorisation flops + a per-front
  // latency term; sub(s) = cost of the subtree rooted at s.  Starting from the roots, the heaviest
  // splittable candidate subtree is moved to the "top" (its children become candidates) while the
  // candidates are dealt to the shards by LPT; the cut with the least (top cost + largest shard)
  // wins.  Every shard computes the same partition (deterministic, shard-independent).
  S.nshards = std::max(1, opt.nshards);
  S.shard = opt.shard;
  MADIPM_REQUIRE(S.shard >= 0 && S.shard < S.nshards, "shard id out of range");
  if (S.nshards > 1) {
    std::vector<double> cost(ns), sub(ns);
    for (int s = 0; s < ns; ++s) {
      const double r = S.nrows[s], w = S.first[s + 1] - S.first[s];
      double f = 0.0;
      for (int t = 0; t < (int)w; ++t) f += (r - t) * (r - t);
      cost[s] = f + 4096.0 + 64.0 * r;
      sub[s] = cost[s];
      for (int64_t q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q) sub[s] += sub[S.child_list[q]];
    }
    std::vector<int32_t> cands, popped;
    for (int s = 0; s < ns; ++s)
      if (S.parent[s] == -1) cands.push_back(s);
    auto lpt = [&](const std::vector<int32_t>& cs, std::vector<int32_t>* bin_of) {
      std::vector<int32_t> o(cs);
      std::sort(o.begin(), o.end(), [&](int a, int b) { return sub[a] > sub[b] || (sub[a] == sub[b] && a < b); });
      std::vector<double> load(S.nshards, 0.0);
      for (int c : o) {
        const int b = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        load[b] += sub[c];
        if (bin_of) (*bin_of)[c] = b;
      }
      return *std::max_element(load.begin(), load.end());
    };
    double topc = 0.0, best = lpt(cands, nullptr);
    size_t best_pops = 0;
    // every pop adds to the top cost, so the search ends once the top alone costs more than the best
    // cut found (or after a bounded number of pops)
    const size_t max_pops = std::min<size_t>((size_t)ns, 4096);
    while (popped.size() < max_pops && topc < best) {
      int bi = -1;
      for (size_t k = 0; k < cands.size(); ++k) {
        const int c = cands[k];
        if (S.child_ptr[c + 1] > S.child_ptr[c] && (bi < 0 || sub[c] > sub[cands[bi]])) bi = (int)k;
      }
      if (bi < 0) break;
      const int c = cands[bi];
      cands.erase(cands.begin() + bi);
      for (int64_t q = S.child_ptr[c]; q < S.child_ptr[c + 1]; ++q) cands.push_back(S.child_list[q]);
      popped.push_back(c);
      topc += cost[c];
      const double obj = topc + lpt(cands, nullptr);
      if (obj < best) {
        best = obj;
        best_pops = popped.size();
      }
    }
    // replay the best cut
    S.owner.assign(ns, -2);
    cands.clear();
    for (int s = 0; s < ns; ++s)
      if (S.parent[s] == -1) cands.push_back(s);
    S.top_cost = 0.0;
    for (size_t k = 0; k < best_pops; ++k) {
      const int c = popped[k];
      S.owner[c] = -1;
      S.top_cost += cost[c];
      cands.erase(std::find(cands.begin(), cands.end(), c));
      for (int64_t q = S.child_ptr[c]; q < S.child_ptr[c + 1]; ++q) cands.push_back(S.child_list[q]);
    }
    std::vector<int32_t> bin(ns, -1);
    S.shard_cost_max = lpt(cands, &bin);
    S.shard_cost_sum = 0.0;
    for (int c : cands) {
      S.owner[c] = bin[c];
      S.shard_cost_sum += sub[c];
    }
    for (int s = ns - 1; s >= 0; --s)
      if (S.owner[s] == -2) {
        MADIPM_REQUIRE(S.parent[s] >= 0, "sharding: unassigned root");
        S.owner[s] = S.owner[S.parent[s]];
      }
    // batched-leaf groups keep this shard's members only (compacted in place, member order kept).  A
    // group under a subtree front lies wholly on that subtree's shard; under a top front its members
    // are dealt like any subtree roots, and each shard's SYRK adds its members' W D^-1 W^T to the top
    // front's external part (all-reduced with it) and its GEMV forward contribution to the exchanged
    // external forward sums.  A group with no member here vanishes on this shard.
    if (!S.lb.empty()) {
      size_t ng = 0, nm = 0, nw = 0;
      int64_t wsize = 0, moved_from = -1, moved_to = 0;
      for (size_t gi = 0; gi < S.lb.size(); ++gi) {
        SymbolicPlan::LBGroup g = S.lb[gi];
        const int64_t m0 = g.mem_off;
        int n = 0;
        const size_t nm0 = nm;
        for (int j = 0; j < S.lb[gi].n; ++j) {
          const size_t q = (size_t)(m0 + j);
          if (S.owner[col2sn[S.lb_mem[q]]] != S.shard) continue;
          const int64_t len = S.lb_ce[q] - S.lb_cs[q], wb = S.lb_wbase[q];
          S.lb_mem[nm] = S.lb_mem[q];
          S.lb_cs[nm] = S.lb_cs[q];
          S.lb_ce[nm] = S.lb_ce[q];
          // shared maps (6b) are consecutive: moved once, for their first kept member (a destination
          // never passes a later map's source, so the maps not moved yet stay intact)
          if (wb != moved_from) {
            std::memmove(S.lb_wrow.data() + nw, S.lb_wrow.data() + wb, sizeof(int32_t) * (size_t)len);
            moved_from = wb;
            moved_to = (int64_t)nw;
            nw += (size_t)len;
          }
          S.lb_wbase[nm] = moved_to;
          ++nm;
          ++n;
        }
        if (n == 0) continue;
        g.mem_off = (int64_t)nm0;
        g.n = n;
        g.w_off = wsize;
        wsize += (int64_t)g.m * n;
        S.lb[ng++] = g;
      }
      S.lb.resize(ng);
      S.lb_mem.resize(nm);
      S.lb_cs.resize(nm);
      S.lb_ce.resize(nm);
      S.lb_wbase.resize(nm);
      S.lb_wrow.resize(nw);
      S.lb_wsize = wsize;
    }
  } else {
    S.owner.clear();  // unsharded: every front belongs to the (only) shard
  }

  stamp("before 9");
  // ---------------- 9. storage layout + statistics (top fronts last, contiguous, full F)
  S.l_off.resize(ns);
  S.u_off.resize(ns);
  S.u_ld.resize(ns);
  S.uvec_off.resize(ns);
  S.is_big.resize(ns);
  int64_t cur = 0, ucur = 0;
  std::vector<int32_t> storage_order;
  for (int s = 0; s < ns; ++s)
    if (!S.top(s)) storage_order.push_back(s);
  const size_t ntop_begin = storage_order.size();
  for (int s = 0; s < ns; ++s)
    if (S.top(s)) storage_order.push_back(s);
  for (size_t so = 0; so < storage_order.size(); ++so) {
    const int s = storage_order[so];
    if (so == ntop_begin) S.top_lo = cur;
    // a batched-leaf member keeps only its pivot row as front structure: its L column (the group's W
    // column) has colcnt entries, which the statistics count
    int64_t r = lb_member(s) ? (int64_t)S.colcnt[S.first[s]] : S.nrows[s], w = S.first[s + 1] - S.first[s];
    S.max_front = std::max<int>(S.max_front, (int)r);
    S.nnzL_super += trap(w, r);
    for (int64_t t = 0; t < w; ++t) {
      double cc = (double)(r - t);
      S.flops += (cc - 1.0) * (cc + 2.0);
    }
    S.uvec_off[s] = ucur;
    if (lb_member(s)) {  // batched leaf: factor lives in its group's W (no front storage, no update vector)
      S.is_big[s] = 0;
      S.l_off[s] = S.u_off[s] = cur;
      S.u_ld[s] = 1;
      continue;
    }
    ucur += r - w;
    if (r <= opt.small_front_max && !S.top(s)) {
      S.is_big[s] = 0;
      S.l_off[s] = cur;
      cur += r * w;
      S.u_off[s] = cur;
      S.u_ld[s] = (int32_t)(r - w);
      cur += (r - w) * (r - w);
    } else {
      S.is_big[s] = 1;
      S.nbig++;
      S.l_off[s] = cur;
      S.u_off[s] = cur + w * r + w;
      S.u_ld[s] = (int32_t)r;
      cur += r * r;
    }
    cur = (cur + 1) & ~(int64_t)1;  // 16-byte alignment of every front
  }
  if (ntop_begin == storage_order.size()) S.top_lo = cur;
  S.top_hi = cur;
  for (auto& g : S.lb) {  // the groups' forward update vectors (gathered by the parent like a child's)
    g.uvec_off = ucur;
    ucur += g.m;
  }
  if (S.nshards > 1) cur += 4 * S.nshards;  // status slots, all-reduced with the top fronts
  S.arena_size = cur;
  S.uvec_size = ucur;

  stamp("before 10");
  // ---------------- 10. assembly plan.  Each task is one 64x64 lower tile of a front's F: its entries
  // are the sums of their gather lists (original K entries first, then the small children's update
  // entries in child order), then the big children's update blocks are added child by child.  A
  // workgroup owns a tile, so the sums are parallel, conflict-free and deterministic.
  // Sharded: a top front is assembled in two parts — "external" (original entries on shard 0 + this
  // shard's subtree-root children; written, zeros included, then all-reduced) and "internal" (its top
  // children, accumulated after the all-reduce at the front's level).
  const int gather_max = opt.gather_max;
  // factorisation tree (k_fact_tree): phase-1 fronts of <= kFactTreeMax rows whose children are all
  // pre-leaves (leaves of <= 32 rows, factorised by the level-0 launches) or tree fronts.  Their
  // original entries and pre-leaf children are pre-assembled into scratch by ONE gather pass after
  // the level-0 launches (group 2 NL + 1); tree children are added inside the tree kernel.
  S.ftree.assign(ns, 0);
  {
    const char* ev = std::getenv("MADIPM_TREE_FACT");
    const bool on = opt.fact_tree && !(ev && ev[0] == '0');
    int fanin_max = SymbolicPlan::kFactTreeFanIn;
    if (const char* e = std::getenv("MADIPM_TREE_FANIN")) fanin_max = std::atoi(e);  // A/B knob
    std::vector<char> lbpar(ns, 0);
    for (const auto& g : S.lb) lbpar[g.parent] = 1;
    for (int s = 0; on && s < ns; ++s) {  // postorder: children first
      if (S.top(s) || !S.mine(s) || lb_member(s) || lbpar[s] || S.nrows[s] > SymbolicPlan::kFactTreeMedMax) continue;
      if (S.child_ptr[s] == S.child_ptr[s + 1] && S.nrows[s] <= 32) continue;  // pre-leaf
      bool ok = true;
      int fanin = 0;  // tree children are added one after another by one workgroup: bound the fan-in
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1] && ok; ++qc) {
        const int c = S.child_list[qc];
        fanin += S.ftree[c];
        ok = S.ftree[c] || (S.child_ptr[c] == S.child_ptr[c + 1] && S.nrows[c] <= 32 && !lb_member(c));
      }
      S.ftree[s] = ok && fanin <= fanin_max;
    }
  }
  // leaf folding (SymbolicPlan::absorb): a tree front whose pre-leaf children are all micro leaves
  // (w <= 2, r <= 32) factorises them itself inside k_fact_tree and subtracts their rank-1/2 updates
  // from its LDS front through destination-sorted product lists, replacing the micro launch and the
  // gather pre-assembly for that front (MADIPM_FOLD=0 disables it).
  const int ns_all = ns;
  S.absorb.assign(ns_all, 0);
  S.fold_pk.assign(ns_all, 0);
  S.mc_ptr.assign(ns_all + 1, 0);
  S.mc_list.clear();
  S.fold_bptr.assign(ns_all + 1, 0);
  S.fold_rmax.assign(ns_all, 0);
  S.fold_lmax.assign(ns_all, 0);
  S.fold_bat.clear();
  S.fold_row0.clear();
  S.fold_poff.clear();
  S.fold_plen.clear();
  S.fold_prod.clear();
  S.fold_chead.clear();
  S.ab_first.clear();
  S.ab_src0.clear();
  S.ab_src1.clear();
  S.ab_k.clear();
  S.ab_f0.clear();
  S.ab_wrc.clear();
  {
    const char* ev = std::getenv("MADIPM_FOLD");
    const bool on = !(ev && ev[0] == '0');
    constexpr int64_t LMAX = SymbolicPlan::kFoldLdsMax;
    constexpr int64_t RB = SymbolicPlan::kFoldRowBytes, LB = SymbolicPlan::kFoldLeafBytes;
    auto micro_leaf = [&](int c) {
      return S.child_ptr[c] == S.child_ptr[c + 1] && S.nrows[c] <= 32 && S.first[c + 1] - S.first[c] <= 2 &&
             S.nrows[c] > S.first[c + 1] - S.first[c];
    };
    auto sq_bytes = [](int64_t r) { return 8 * ((r * (r | 1) + 1) & ~1LL); };
    auto pk_bytes = [](int64_t r) { return 8 * ((r * (r + 1) / 2 + 1) & ~1LL); };
    struct Prod {
      uint32_t dst, q1, q2;
    };
    {
      // k_fact_tree's ticket order: by level (children before parents, so a workgroup waiting on its
      // children never blocks the tickets they need), and within a level by descending tail — the
      // estimated work from the front up to the root — so the fronts of the longest chains take the
      // first CUs.  Every tree front folds its micro leaves (r3: leaving the leaves of the fronts past
      // the first 256 tickets to a micro launch + gather pre-assembly measured 1547 vs 1593 iters/s)
      std::vector<double> tail(ns_all, 0.0);
      for (int s = ns_all - 1; s >= 0; --s) {  // parents have larger indices (postorder)
        const double r = S.nrows[s], w = S.first[s + 1] - S.first[s];
        tail[s] = r * r + r * w + (S.parent[s] >= 0 ? tail[S.parent[s]] : 0.0);
      }
      std::vector<int> ord;
      for (int lev = 0; lev < S.nlevels; ++lev) {
        const size_t o0 = ord.size();
        for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q)
          if (S.ftree[S.level_list[q]]) ord.push_back(S.level_list[q]);
        std::stable_sort(ord.begin() + o0, ord.end(), [&](int a, int b) { return tail[a] > tail[b]; });
      }
      S.ft_order.assign(ord.begin(), ord.end());
    }
    // One front's fold tables, with part-local offsets: the fronts are independent, so they run on
    // the analysis threads and the parts are appended in front order afterwards (offsets shifted —
    // the tables are the sequential ones bit for bit).
    struct FoldPart {
      std::vector<int32_t> mc_list, ab_src0, ab_src1, ab_k, ab_wrc, fold_bat, fold_plen;
      std::vector<int64_t> ab_first, ab_f0, fold_row0, fold_poff;
      std::vector<uint32_t> fold_prod, fold_chead;
    };
    struct FoldScratch {
      std::vector<int64_t> col0 = std::vector<int64_t>(32), col1 = std::vector<int64_t>(32);
      std::vector<Prod> pr, pr2;
      std::vector<int64_t> cnt;
      std::vector<std::vector<uint32_t>> enc;
    };
    auto fold_front = [&](int s, FoldPart& P, FoldScratch& X) {
      auto& pr = X.pr;
      auto& enc = X.enc;
      auto& col0 = X.col0;
      auto& col1 = X.col1;
      if (!on || !S.ftree[s] || S.nrows[s] > SymbolicPlan::kFactTreeMax) return;  // medium fronts: no folding
      const int64_t r = S.nrows[s];
      int64_t nmc = 0, nrow = 0;
      bool ok = true;
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1] && ok; ++qc) {
        const int c = S.child_list[qc];
        if (S.ftree[c]) continue;
        ok = micro_leaf(c);
        ++nmc;
        nrow += S.nrows[c];
      }
      if (!ok || nmc == 0) return;
      // storage: square (r <= 128) when the front and all its leaf rows fit, else packed lower;
      // leaves in batches when even that does not fit
      int pk;
      int64_t budget;
      if (r <= 128 && sq_bytes(r) + RB * nrow + LB * nmc <= LMAX) {
        pk = 0;
        budget = LMAX - sq_bytes(r);
      } else {
        pk = 1;
        budget = LMAX - pk_bytes(r);
      }
      if (budget < RB * 32 + LB) return;  // not even one leaf fits beside the front
      // a batch of `rows` leaf rows and `nl` leaves fits when the front's LDS carve — sized by the
      // largest batch's rows and the largest batch's leaf count, possibly two different batches —
      // stays within the budget
      // stays within the budget; and at most 2 kFoldThreads leaves per batch (k_fact_tree's fold_leaves
      // holds a batch's leaf table in two registers per thread: a bigger batch is a carve error there)
      auto fits = [&](int64_t rows, int64_t nl, int64_t rmax, int64_t lmax) {
        return RB * std::max(rows, rmax) + LB * std::max(nl, lmax) <= budget && rows <= SymbolicPlan::kFoldRowsMax &&
               nl <= SymbolicPlan::kFoldLeavesMax;
      };
      {  // the batch table lives in LDS: fronts needing more batches leave their leaves unfolded
        int nb = 0;
        int64_t rows = 0, nl = 0, rmax = 0, lmax = 0;
        bool ok2 = true;
        for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1] && ok2; ++qc) {
          const int c = S.child_list[qc];
          if (S.ftree[c]) continue;
          if (nl == 0 || !fits(rows + S.nrows[c], nl + 1, rmax, lmax)) {
            ++nb, rows = 0, nl = 0;
            ok2 = fits(S.nrows[c], 1, rmax, lmax);
          }
          rows += S.nrows[c];
          ++nl;
          rmax = std::max(rmax, rows);
          lmax = std::max(lmax, nl);
        }
        if (!ok2 || nb > SymbolicPlan::kFoldMaxBatches) return;
      }
      S.absorb[s] = 1;
      S.fold_pk[s] = (uint8_t)pk;
      const int64_t ld = r | 1;
      auto fidx = [&](int64_t i, int64_t j) -> uint32_t {
        return (uint32_t)(pk ? (j * (2 * r - j - 1)) / 2 + i : i + j * ld);
      };
      const int k0 = 0;  // part-local leaf indices (shifted when the parts are appended)
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1]; ++qc)
        if (!S.ftree[S.child_list[qc]]) P.mc_list.push_back(S.child_list[qc]);
      const int k1 = (int)P.mc_list.size();
      // flat leaf rows (child order)
      for (int k = k0; k < k1; ++k) {
        const int c = P.mc_list[k];
        const int rc = S.nrows[c], wc = S.first[c + 1] - S.first[c];
        P.ab_first.push_back((int64_t)P.ab_src0.size());
        P.ab_f0.push_back(S.first[c]);
        P.ab_wrc.push_back(wc | (rc << 8));
        std::fill(col0.begin(), col0.end(), -1);
        std::fill(col1.begin(), col1.end(), -1);
        for (int64_t q = S.asm_ptr[c]; q < S.asm_ptr[c + 1]; ++q) {
          const int64_t d = S.asm_dst[q];
          const int lc = (int)(d / rc), lr = (int)(d % rc);
          (lc == 0 ? col0 : col1)[lr] = S.asm_src[q];
        }
        for (int i = 0; i < rc; ++i) {
          MADIPM_REQUIRE(col0[i] < INT32_MAX && col1[i] < INT32_MAX, "folded leaf: CSC index beyond int32");
          P.ab_src0.push_back((int32_t)col0[i]);
          P.ab_src1.push_back((int32_t)col1[i]);
          P.ab_k.push_back(k);
        }
      }
      // batches and their product lists
      int kb = k0;
      while (kb < k1) {
        int ke = kb;
        int64_t rows = 0;
        while (ke < k1 && fits(rows + S.nrows[P.mc_list[ke]], ke - kb + 1, S.fold_rmax[s], S.fold_lmax[s]))
          rows += S.nrows[P.mc_list[ke++]];
        MADIPM_REQUIRE(ke > kb, "fold: a leaf does not fit the batch budget");
        P.fold_bat.push_back(kb);
        P.fold_row0.push_back(P.ab_first[kb]);
        S.fold_rmax[s] = std::max<int32_t>(S.fold_rmax[s], (int32_t)rows);
        S.fold_lmax[s] = std::max<int32_t>(S.fold_lmax[s], ke - kb);
        const int64_t row0 = P.ab_first[kb];
        pr.clear();
        for (int k = kb; k < ke; ++k) {
          const int c = P.mc_list[k];
          const int rc = S.nrows[c], wc = S.first[c + 1] - S.first[c];
          const int32_t* rl = S.rel.data() + S.rel_ptr[c];
          const uint32_t qb0 = (uint32_t)(P.ab_first[k] - row0);
          for (int a = wc; a < rc; ++a)
            for (int b = wc; b <= a; ++b)  // rel ascending: parent row of b <= that of a
              pr.push_back({fidx(rl[a - wc], rl[b - wc]), qb0 + a, qb0 + b});
        }
        {  // counting sort by destination: stable (leaf order within a destination), O(products)
          uint32_t dmax = 0;
          for (const Prod& x : pr) dmax = std::max(dmax, x.dst);
          auto& cnt = X.cnt;
          cnt.assign((size_t)dmax + 2, 0);
          for (const Prod& x : pr) cnt[x.dst + 1]++;
          for (size_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
          X.pr2.resize(pr.size());
          for (const Prod& x : pr) X.pr2[cnt[x.dst]++] = x;
          pr.swap(X.pr2);
        }
        // NCH chunks of equal length (a run split where a cut falls), each encoded with its running
        // destination (SymbolicPlan: one word per entry, kFoldPad steps for jumps beyond 127)
        constexpr int NCH = NT_FOLD;
        constexpr uint32_t PAD = SymbolicPlan::kFoldPad;
        const int64_t NP = (int64_t)pr.size();
        enc.assign(NCH, {});
        // (fewer products than chunks: one per chunk, the empty chunks last — the parts of a split
        // run always lie in adjacent chunks, which the kernel's left-to-right tail sum relies on)
        for (int t = 0; t < NCH; ++t) {
          const int64_t q0 = NP < NCH ? std::min<int64_t>(t, NP) : NP * t / NCH;
          const int64_t q1 = NP < NCH ? std::min<int64_t>(t + 1, NP) : NP * (t + 1) / NCH;
          std::vector<uint32_t>& E = enc[t];
          uint32_t head = 0;
          if (q0 < q1) {
            uint32_t d = pr[q0].dst;
            head = d | ((q0 > 0 && pr[q0 - 1].dst == d) ? SymbolicPlan::kFoldCont : 0u);
            for (int64_t q = q0; q < q1; ++q) {
              MADIPM_REQUIRE(pr[q].dst < 65536 && pr[q].q1 < PAD && pr[q].q2 < PAD, "fold: index beyond its field");
              uint32_t dd = pr[q].dst - d;
              for (; dd > 127; dd -= 127) E.push_back(PAD | (127u << 24));
              d = pr[q].dst;
              const bool end = q + 1 == q1 || pr[q + 1].dst != d;
              E.push_back(pr[q].q1 | (pr[q].q2 << 12) | (dd << 24) | (end ? SymbolicPlan::kFoldRunEnd : 0u));
            }
          }
          P.fold_chead.push_back(head);
        }
        int64_t len = 0;
        for (int t = 0; t < NCH; ++t) len = std::max<int64_t>(len, (int64_t)enc[t].size());
        const int64_t off = (int64_t)P.fold_prod.size();
        P.fold_poff.push_back(off);
        P.fold_plen.push_back((int32_t)len);
        P.fold_prod.resize(off + len * NCH, PAD);  // padding: no product, no step, no run end
        for (int t = 0; t < NCH; ++t)
          for (size_t k = 0; k < enc[t].size(); ++k) P.fold_prod[off + (int64_t)k * NCH + t] = enc[t][k];
        kb = ke;
      }
      MADIPM_REQUIRE(RB * S.fold_rmax[s] + LB * S.fold_lmax[s] <= budget, "fold: LDS carve beyond the budget");
    };
    {
      std::vector<FoldPart> fparts(ns_all);
      std::atomic<int> next{0};
      const int T = std::max(1, std::min<int>(analysis_threads(), ns_all / 256));
      auto worker = [&] {
        FoldScratch X;
        for (int s0; (s0 = next.fetch_add(64)) < ns_all;)
          for (int s = s0; s < std::min(ns_all, s0 + 64); ++s) fold_front(s, fparts[s], X);
      };
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t) th.emplace_back(worker);
      worker();
      for (auto& x : th) x.join();
      stamp("10a: fold tables per front (threads)");
      // the parts appended in front order: offsets by prefix sums, copies (with the shifts) on threads
      std::vector<int64_t> om(ns_all + 1), oa(ns_all + 1), op(ns_all + 1), ob(ns_all + 1);
      om[0] = (int64_t)S.mc_list.size();
      oa[0] = (int64_t)S.ab_src0.size();
      op[0] = (int64_t)S.fold_prod.size();
      ob[0] = (int64_t)S.fold_bat.size();
      const int64_t f0 = (int64_t)S.ab_first.size() - om[0], h0 = (int64_t)S.fold_chead.size() - ob[0] * NT_FOLD;
      for (int s = 0; s < ns_all; ++s) {
        const FoldPart& P = fparts[s];
        om[s + 1] = om[s] + (int64_t)P.mc_list.size();
        oa[s + 1] = oa[s] + (int64_t)P.ab_src0.size();
        op[s + 1] = op[s] + (int64_t)P.fold_prod.size();
        ob[s + 1] = ob[s] + (int64_t)P.fold_bat.size();
        S.mc_ptr[s + 1] = (int32_t)om[s + 1];
        S.fold_bptr[s + 1] = (int32_t)ob[s + 1];
      }
      S.mc_list.resize(om[ns_all]);
      S.ab_first.resize(f0 + om[ns_all]);
      S.ab_f0.resize(om[ns_all]);
      S.ab_wrc.resize(om[ns_all]);
      S.ab_src0.resize(oa[ns_all]);
      S.ab_src1.resize(oa[ns_all]);
      S.ab_k.resize(oa[ns_all]);
      S.fold_bat.resize(ob[ns_all]);
      S.fold_row0.resize(ob[ns_all]);
      S.fold_poff.resize(ob[ns_all]);
      S.fold_plen.resize(ob[ns_all]);
      S.fold_chead.resize(h0 + ob[ns_all] * NT_FOLD);
      S.fold_prod.resize(op[ns_all]);
      next = 0;
      auto copier = [&] {
        for (int s0; (s0 = next.fetch_add(64)) < ns_all;)
          for (int s = s0; s < std::min(ns_all, s0 + 64); ++s) {
            FoldPart& P = fparts[s];
            const int32_t mbase = (int32_t)om[s];
            const int64_t abase = oa[s], pbase = op[s], m = om[s], bb = ob[s];
            for (size_t k = 0; k < P.mc_list.size(); ++k) {
              S.mc_list[m + k] = P.mc_list[k];
              S.ab_first[f0 + m + k] = P.ab_first[k] + abase;
              S.ab_f0[m + k] = (int32_t)P.ab_f0[k];
              S.ab_wrc[m + k] = P.ab_wrc[k];
            }
            for (size_t k = 0; k < P.ab_src0.size(); ++k) {
              S.ab_src0[abase + k] = P.ab_src0[k];
              S.ab_src1[abase + k] = P.ab_src1[k];
              S.ab_k[abase + k] = P.ab_k[k] + mbase;
            }
            for (size_t k = 0; k < P.fold_bat.size(); ++k) {
              S.fold_bat[bb + k] = P.fold_bat[k] + mbase;
              S.fold_row0[bb + k] = P.fold_row0[k] + abase;
              S.fold_poff[bb + k] = P.fold_poff[k] + pbase;
              S.fold_plen[bb + k] = P.fold_plen[k];
            }
            std::copy(P.fold_chead.begin(), P.fold_chead.end(), S.fold_chead.begin() + h0 + bb * NT_FOLD);
            std::copy(P.fold_prod.begin(), P.fold_prod.end(), S.fold_prod.begin() + pbase);
            P = FoldPart();
          }
      };
      th.clear();
      for (int t = 1; t < T; ++t) th.emplace_back(copier);
      copier();
      for (auto& x : th) x.join();
    }
    S.ab_first.push_back((int64_t)S.ab_src0.size());
    // sentinels: the batch after a front's last one starts at that front's end (leaves and rows are
    // appended front by front), so batch b always ends where batch b + 1 begins
    S.fold_bat.push_back((int32_t)S.mc_list.size());
    S.fold_row0.push_back(S.ab_first.back());
    if (std::getenv("MADIPM_FOLD_STATS")) {  // diagnostics: per level, the folded leaves and products
      std::vector<double> acc((size_t)S.nlevels * 6, 0.0);
      for (int s = 0; s < ns_all; ++s) {
        if (!S.absorb[s]) continue;
        double* a = &acc[(size_t)S.level[s] * 6];
        a[0] += 1;
        a[1] += S.mc_ptr[s + 1] - S.mc_ptr[s];
        a[2] += (double)(S.ab_first[S.mc_ptr[s + 1]] - S.ab_first[S.mc_ptr[s]]);
        for (int b = S.fold_bptr[s]; b < S.fold_bptr[s + 1]; ++b)
          a[3] += (double)S.fold_plen[b] * NT_FOLD;
        a[4] += S.fold_bptr[s + 1] - S.fold_bptr[s];
        a[5] += S.nrows[s];
      }
      for (int lv = 0; lv < S.nlevels; ++lv)
        if (acc[lv * 6] > 0)
          fprintf(stderr, "fold level %d: %d fronts  r %.1f  leaves %.1f  leaf rows %.1f  product slots %.1f  batches %.2f\n", lv,
                  (int)acc[lv * 6], acc[lv * 6 + 5] / acc[lv * 6], acc[lv * 6 + 1] / acc[lv * 6], acc[lv * 6 + 2] / acc[lv * 6],
                  acc[lv * 6 + 3] / acc[lv * 6], acc[lv * 6 + 4] / acc[lv * 6]);
    }
  }
  stamp("10a: fold product lists");
  // the folded micro leaves never write an update block (their products go straight into the parent's
  // LDS front): lay the arena out again without their (r - w)^2 blocks, so the leaves' L panels are
  // contiguous in postorder (ex10: 138 MB of the arena were unused leaf blocks between 272-byte L
  // panels — the leaf solves and the fold's L stores touched a cache line per panel piece)
  if (!S.mc_list.empty()) {
    std::vector<uint8_t> folded(ns, 0);
    for (int c : S.mc_list) folded[c] = 1;
    int64_t cur2 = 0;
    for (size_t so = 0; so < storage_order.size(); ++so) {
      const int s = storage_order[so];
      if (so == ntop_begin) S.top_lo = cur2;
      if (lb_member(s)) {
        S.l_off[s] = S.u_off[s] = cur2;
        continue;
      }
      const int64_t r = S.nrows[s], w = S.first[s + 1] - S.first[s];
      S.l_off[s] = cur2;
      if (!S.is_big[s]) {
        S.u_off[s] = cur2 + r * w;
        cur2 += r * w + (folded[s] ? 0 : (r - w) * (r - w));
      } else {
        S.u_off[s] = cur2 + w * r + w;
        cur2 += r * r;
      }
      cur2 = (cur2 + 1) & ~(int64_t)1;
    }
    if (ntop_begin == storage_order.size()) S.top_lo = cur2;
    S.top_hi = cur2;
    if (S.nshards > 1) cur2 += 4 * S.nshards;
    S.arena_size = cur2;
  }
  S.fs_off.assign(ns, -1);
  S.fs_size = 0;
  for (int s = 0; s < ns; ++s)
    if ((S.ftree[s] && !S.absorb[s] && S.nrows[s] <= SymbolicPlan::kFactTreeMax) ||
        (!S.ftree[s] && !S.is_big[s] && S.child_ptr[s + 1] > S.child_ptr[s] && S.mine(s))) {
      // (medium tree fronts are pre-assembled in place, in the arena: no scratch)
      S.fs_off[s] = S.fs_size;
      // fronts staged into LDS are pre-assembled as their LDS image (square ld r | 1, or packed
      // lower for r > 128): room for r (r | 1) doubles
      S.fs_size += (int64_t)S.nrows[s] * (S.nrows[s] | 1);
    }
  S.atiles.clear();
  S.g_ptr.clear();
  S.g_src.clear();
  S.bt.clear();
  S.atile_lev.assign(2 * S.nlevels + 3, 0);
  S.chunk_lev.assign(2 * S.nlevels + 3, 0);
  S.g_chunk.clear();
  {
    // children of s whose update blocks this assembly reads: 0 all, 1 top children only, 2 this
    // shard's subtree children only
    auto child_ok = [&](int c, int which) {
      if (lb_member(c)) return false;  // batched leaves: absorbed by the group SYRK
      if (which == 0) return true;
      if (which == 1) return S.top(c);
      if (which == 3) return !S.ftree[c];  // tree front: pre-leaf children only
      return !S.top(c) && S.owner[c] == S.shard;
    };
    // One emit = the tiles of one front, written into a part of its own with part-local offsets (the
    // fronts are independent, so the emits run on the analysis threads; the parts are appended in
    // emit order afterwards, offsets shifted — the plan is the sequential one bit for bit).
    struct Part {
      std::vector<SymbolicPlan::AsmTile> atiles;
      std::vector<int32_t> g_ptr, bt;
      std::vector<int64_t> g_chunk, g_src;
    };
    struct Scratch {
      std::vector<int32_t> key, tcnt, cnt = std::vector<int32_t>(4097), bykey;
      std::vector<int64_t> src, bysrc, sorted;
    };
    // tsel: 0 every tile, 1 the tiles of column block 0 only, 2 the others only
    auto emit = [&](Part& P, Scratch& X, int s, bool orig, int which, bool acc, bool emit_empty, int tsel) {
      auto& key = X.key;
      auto& tcnt = X.tcnt;
      auto& cnt = X.cnt;
      auto& bykey = X.bykey;
      auto& src = X.src;
      auto& bysrc = X.bysrc;
      auto& sorted = X.sorted;
      const int r = S.nrows[s];
      const int nt = (r + 63) / 64;
      const int ntile = nt * (nt + 1) / 2;
      auto tkey = [&](int row, int col) {
        const int ti = row >> 6, tj = col >> 6;
        return (int32_t)((ti * (ti + 1) / 2 + tj) * 4096 + (row & 63) + (col & 63) * 64);
      };
      key.clear();
      src.clear();
      if (orig)
        for (int64_t qa = S.asm_ptr[s]; qa < S.asm_ptr[s + 1]; ++qa) {
          const int64_t d = S.asm_dst[qa];
          key.push_back(tkey((int)(d % r), (int)(d / r)));
          src.push_back(~S.asm_src[qa]);
        }
      std::vector<int32_t> bigch;
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1]; ++qc) {
        const int c = S.child_list[qc];
        if (!child_ok(c, which)) continue;
        const int uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
        if (uc > gather_max && which != 3) {
          bigch.push_back(c);
          continue;
        }
        const int32_t* relc = S.rel.data() + S.rel_ptr[c];
        for (int bb = 0; bb < uc; ++bb)
          for (int aa = bb; aa < uc; ++aa) {
            key.push_back(tkey(relc[aa], relc[bb]));
            src.push_back(S.u_off[c] + aa + (int64_t)bb * S.u_ld[c]);
          }
      }
      // stable counting sort by key (keeps originals-then-children order per entry), in two passes:
      // by tile, then inside each tile with entries by its 4096 positions — O(entries + tiles), not
      // O(r^2) per front (neos' 1257 big fronts: 13.7 -> 0.5 s)
      tcnt.assign(ntile + 1, 0);
      for (int32_t k : key) tcnt[(k >> 12) + 1]++;
      for (int t = 0; t < ntile; ++t) tcnt[t + 1] += tcnt[t];
      bykey.resize(key.size());
      bysrc.resize(src.size());
      {
        std::vector<int32_t> fill(tcnt.begin(), tcnt.end() - 1);
        for (size_t e = 0; e < key.size(); ++e) {
          const int32_t q = fill[key[e] >> 12]++;
          bykey[q] = key[e] & 4095;
          bysrc[q] = src[e];
        }
      }
      sorted.resize(src.size());
      for (int ti = 0; ti < nt; ++ti)
        for (int tj = 0; tj <= ti; ++tj) {
          if ((tsel == 1 && tj != 0) || (tsel == 2 && tj == 0)) continue;
          const int t = ti * (ti + 1) / 2 + tj;
          SymbolicPlan::AsmTile at{};
          at.front = s;
          at.tij = ti | (tj << 16) | (acc ? SymbolicPlan::kAccumulate : 0);
          const int64_t e0 = tcnt[t], e1 = tcnt[t + 1];
          const bool has_g = e1 > e0;
          if (has_g) {
            std::fill(cnt.begin(), cnt.end(), 0);
            for (int64_t e = e0; e < e1; ++e) cnt[bykey[e] + 1]++;
            for (int k = 0; k < 4096; ++k) cnt[k + 1] += cnt[k];
            {
              std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
              for (int64_t e = e0; e < e1; ++e) sorted[e0 + fill[bykey[e]]++] = bysrc[e];
            }
            // the tile's entry list: ne, then per nonempty entry its position | first chunk << 12,
            // then the chunk count << 12 (a dense 4097-offset table per tile was 1.5 GB on neos,
            // mostly for tree-front tiles of ~40 nonempty entries)
            at.gptr = (int64_t)P.g_ptr.size();
            at.gchk = (int64_t)P.g_chunk.size();
            int32_t nchk = 0, ne = 0;
            const int64_t sbase = (int64_t)P.g_src.size();
            P.g_ptr.push_back(0);
            for (int k = 0; k < 4096; ++k) {
              if (cnt[k + 1] == cnt[k]) continue;
              P.g_ptr.push_back(k | nchk << 12);
              ++ne;
              for (int64_t c = cnt[k]; c < cnt[k + 1]; c += SymbolicPlan::kChunk, ++nchk) P.g_chunk.push_back(sbase + c);
            }
            MADIPM_REQUIRE(nchk < (1 << 19), "assembly: more than 2^19 chunks on one tile");
            P.g_ptr.push_back(nchk << 12);
            P.g_ptr[at.gptr] = ne;
            P.g_src.insert(P.g_src.end(), sorted.begin() + e0, sorted.begin() + e1);
          } else {
            at.gptr = -1;
            at.gchk = 0;
          }
          at.bt0 = (int32_t)(P.bt.size() / 5);
          const int I0 = ti * 64, I1 = std::min(r, I0 + 64), J0 = tj * 64, J1 = std::min(r, J0 + 64);
          for (int c : bigch) {
            const int uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
            const int32_t* relc = S.rel.data() + S.rel_ptr[c];
            const int b0 = (int)(std::lower_bound(relc, relc + uc, J0) - relc);
            const int b1 = (int)(std::lower_bound(relc + b0, relc + uc, J1) - relc);
            const int a0 = (int)(std::lower_bound(relc, relc + uc, I0) - relc);
            const int a1 = (int)(std::lower_bound(relc + a0, relc + uc, I1) - relc);
            if (b0 < b1 && a0 < a1 && a1 - 1 >= b0) {
              const int32_t e[5] = {c, b0, b1, a0, a1};
              P.bt.insert(P.bt.end(), e, e + 5);
            }
          }
          at.bt1 = (int32_t)(P.bt.size() / 5);
          if (has_g || at.bt1 > at.bt0 || emit_empty) P.atiles.push_back(at);
        }
    };
    // the plan as a sequence of operations: emits, and marks recording where a group / the fused
    // fronts' tiles begin (mark kinds: 0 close_group(g), 1 atile_fz0[g], 2 atile_fz1[g])
    struct Op {
      int s, which, tsel;
      bool orig, acc, emit_empty;
      int mark, g;
    };
    std::vector<Op> ops;
    auto op_emit = [&](int s, bool orig, int which, bool acc, bool emit_empty, int tsel = 0) {
      ops.push_back(Op{s, which, tsel, orig, acc, emit_empty, -1, 0});
    };
    auto op_mark = [&](int kind, int g) { ops.push_back(Op{0, 0, 0, false, false, false, kind, g}); };
    const int NL = S.nlevels;
    // phase 1: this shard's fronts (all fronts when unsharded), level by level.  Single-panel big
    // fronts (w <= 64; SymbolicPlan::fused) last: their column block 0 (the panel, assembled before the
    // panel factorisation), then their other tiles, which k_asm_update assembles after the panel's
    // L is known and writes once, updated (C - L_I D L_J^T) — the tiles of column block 0 join that
    // launch too for their columns >= w.  The group: [plain..., fused block 0..., fused rest...).
    S.fused.assign(ns, 0);
    {
      const char* ev = std::getenv("MADIPM_FUSED_UPDATE");
      const bool on = !(ev && ev[0] == '0');
      std::vector<char> lbpar(ns, 0);
      for (const auto& g : S.lb) lbpar[g.parent] = 1;
      for (int s = 0; on && s < ns; ++s) {
        const int w = S.first[s + 1] - S.first[s];
        S.fused[s] = S.is_big[s] && !S.top(s) && S.mine(s) && !lb_member(s) && !S.ftree[s] && !lbpar[s] &&
                     S.fs_off[s] < 0 && w <= 64 && S.nrows[s] > w;
      }
    }
    S.atile_fz0.assign(NL, 0);
    S.atile_fz1.assign(NL, 0);
    for (int lev = 0; lev < NL; ++lev) {
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) {
        const int s = S.level_list[q];
        if (S.top(s) || !S.mine(s) || lb_member(s) || S.ftree[s] || S.fused[s]) continue;
        if (!S.is_big[s] && S.fs_off[s] < 0) continue;
        op_emit(s, true, 0, false, true);
      }
      op_mark(1, lev);
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q)
        if (S.fused[S.level_list[q]]) op_emit(S.level_list[q], true, 0, false, true, 1);
      op_mark(2, lev);
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q)
        if (S.fused[S.level_list[q]]) op_emit(S.level_list[q], true, 0, false, true, 2);
      op_mark(0, lev);
    }
    // top fronts, external part (before the all-reduce; zeros included)
    for (int s = 0; s < ns; ++s)
      if (S.top(s)) op_emit(s, S.shard == 0, 2, false, true);
    op_mark(0, NL);
    // phase 2: top fronts, internal part (their top children), level by level
    for (int lev = 0; lev < NL; ++lev) {
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) {
        const int s = S.level_list[q];
        if (S.top(s)) op_emit(s, false, 1, true, false);
      }
      op_mark(0, NL + 1 + lev);
    }
    // factorisation-tree pre-assembly (after the level-0 launches), tree fronts in level order
    for (int lev = 0; lev < NL; ++lev)
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q)
        if (S.ftree[S.level_list[q]] && !S.absorb[S.level_list[q]]) op_emit(S.level_list[q], true, 3, false, true);
    op_mark(0, 2 * NL + 1);
    // the emits, dealt dynamically to the analysis threads (heaviest fronts vary a lot in cost)
    std::vector<Part> parts(ops.size());
    stamp("10b: plan ops");
    {
      std::atomic<size_t> next{0};
      int64_t work = 0;
      for (const Op& o : ops)
        if (o.mark < 0) work += (int64_t)S.nrows[o.s] * S.nrows[o.s];
      const int T = std::max(1, std::min<int>(analysis_threads(), (int)(work / 200000)));
      // heaviest emits first (longest-processing-time order: neos' 16 block separators take 0.15-0.6 s
      // each and, dealt in level order, finished last on a few threads).  Each emit fills its own part:
      // the order they run in changes nothing in the plan.
      std::vector<int64_t> cost(ops.size(), -1);
      for (size_t k = 0; k < ops.size(); ++k) {
        const Op& o = ops[k];
        if (o.mark >= 0) continue;
        int64_t e = o.orig ? S.asm_ptr[o.s + 1] - S.asm_ptr[o.s] : 0;  // its sources (entries) estimate
        for (int64_t qc = S.child_ptr[o.s]; qc < S.child_ptr[o.s + 1]; ++qc) {
          const int c = S.child_list[qc];
          if (!child_ok(c, o.which)) continue;
          const int64_t uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
          if (uc <= gather_max || o.which == 3) e += uc * (uc + 1) / 2;
        }
        cost[k] = e + (int64_t)S.nrows[o.s] * S.nrows[o.s] / 64;  // + its tiles
      }
      std::vector<size_t> order(ops.size());
      std::iota(order.begin(), order.end(), (size_t)0);
      std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return cost[a] > cost[b]; });
      auto worker = [&] {
        Scratch X;
        for (size_t q; (q = next.fetch_add(1)) < ops.size();) {
          const size_t k = order[q];
          const Op& o = ops[k];
          if (o.mark < 0) emit(parts[k], X, o.s, o.orig, o.which, o.acc, o.emit_empty, o.tsel);
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t) th.emplace_back(worker);
      worker();
      for (auto& x : th) x.join();
    }
    stamp("10b: plan emits");
    // append the parts in emit order, offsets shifted: every part's place from prefix sums, then the
    // copies on the analysis threads (neos: ~1.4 GB of sources and 0.5 GB of chunk offsets, 0.4 s
    // single-threaded)
    {
      const size_t nop = ops.size();
      std::vector<int64_t> oa(nop + 1, 0), opp(nop + 1, 0), ob(nop + 1, 0), oc(nop + 1, 0), os(nop + 1, 0);
      for (size_t k = 0; k < nop; ++k) {
        const Op& o = ops[k];
        const Part& P = parts[k];
        const bool e = o.mark < 0;
        oa[k + 1] = oa[k] + (e ? (int64_t)P.atiles.size() : 0);
        opp[k + 1] = opp[k] + (e ? (int64_t)P.g_ptr.size() : 0);
        ob[k + 1] = ob[k] + (e ? (int64_t)P.bt.size() : 0);
        oc[k + 1] = oc[k] + (e ? (int64_t)P.g_chunk.size() : 0);
        os[k + 1] = os[k] + (e ? (int64_t)P.g_src.size() : 0);
        if (o.mark == 0) {
          S.atile_lev[o.g + 1] = (int32_t)oa[k];
          S.chunk_lev[o.g + 1] = oc[k];
        } else if (o.mark == 1) {
          S.atile_fz0[o.g] = (int32_t)oa[k];
        } else if (o.mark == 2) {
          S.atile_fz1[o.g] = (int32_t)oa[k];
        }
      }
      MADIPM_REQUIRE(os[nop] < (int64_t)INT32_MAX * 2 && oa[nop] < (int64_t)INT32_MAX, "assembly plan too large");
      S.atiles.resize(oa[nop]);
      S.g_ptr.resize(opp[nop]);
      S.bt.resize(ob[nop]);
      S.g_chunk.resize(oc[nop]);
      S.g_src.resize(os[nop]);
      stamp("10b: plan parts placed");
      std::atomic<size_t> next{0};
      auto worker = [&] {
        for (size_t k; (k = next.fetch_add(1)) < nop;) {
          if (ops[k].mark >= 0) continue;
          Part& P = parts[k];
          const int64_t pbase = opp[k], cbase = oc[k], sbase = os[k];
          const int32_t bbase = (int32_t)(ob[k] / 5);
          for (size_t t = 0; t < P.atiles.size(); ++t) {
            SymbolicPlan::AsmTile at = P.atiles[t];
            if (at.gptr >= 0) {
              at.gptr += pbase;
              at.gchk += cbase;
            }
            at.bt0 += bbase;
            at.bt1 += bbase;
            S.atiles[oa[k] + t] = at;
          }
          std::copy(P.g_ptr.begin(), P.g_ptr.end(), S.g_ptr.begin() + pbase);
          for (size_t t = 0; t < P.g_chunk.size(); ++t) S.g_chunk[cbase + t] = P.g_chunk[t] + sbase;
          std::copy(P.g_src.begin(), P.g_src.end(), S.g_src.begin() + sbase);
          std::copy(P.bt.begin(), P.bt.end(), S.bt.begin() + ob[k]);
          Part().atiles.swap(P.atiles);  // release as we go
          std::vector<int32_t>().swap(P.g_ptr);
          std::vector<int32_t>().swap(P.bt);
          std::vector<int64_t>().swap(P.g_src);
          std::vector<int64_t>().swap(P.g_chunk);
        }
      };
      const int T = std::max(1, std::min<int>(analysis_threads(), (int)(os[nop] / 1000000) + 1));
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t) th.emplace_back(worker);
      worker();
      for (auto& x : th) x.join();
    }
    S.g_chunk.push_back((int64_t)S.g_src.size());  // sentinel
  }

  stamp("10b: assembly plan");
  if (std::getenv("MADIPM_ASM_STATS")) {  // diagnostics: per assembly group, tiles, big-child blocks, chunks
    for (size_t g = 0; g + 1 < S.atile_lev.size(); ++g) {
      const int32_t t0 = S.atile_lev[g], t1 = S.atile_lev[g + 1];
      if (t1 <= t0) continue;
      double bc = 0, bmax = 0, ch = 0, chmax = 0, nent = 0, nne = 0, nsrc = 0, c1 = 0, smax = 0, s16 = 0, s64 = 0;
      for (int32_t t = t0; t < t1; ++t) {
        const auto& A = S.atiles[t];
        const double nb = (A.bt1 - A.bt0);
        bc += nb;
        bmax = std::max(bmax, nb);
        if (A.gptr >= 0) {
          const int32_t ne = S.g_ptr[A.gptr];
          const double c = S.g_ptr[A.gptr + ne + 1] >> 12;
          ch += c;
          chmax = std::max(chmax, c);
          nent += 4096;
          nne += ne;
          for (int64_t k = 0; k < (int64_t)c; ++k) {
            const int64_t q = A.gchk + k, ns = S.g_chunk[q + 1] - S.g_chunk[q];
            nsrc += (double)ns;
            c1 += ns == 1;
          }
          for (int32_t e = 0; e < ne; ++e) {
            const int32_t ce = (S.g_ptr[A.gptr + 2 + e] >> 12) - (S.g_ptr[A.gptr + 1 + e] >> 12);
            const int64_t se = S.g_chunk[A.gchk + (S.g_ptr[A.gptr + 1 + e] >> 12) + ce] - S.g_chunk[A.gchk + (S.g_ptr[A.gptr + 1 + e] >> 12)];
            smax = std::max(smax, (double)se);
            s16 += se > 16;
            s64 += se > 64;
          }
        }
      }
      fprintf(stderr, "asm group %zu: %d tiles  big-child blocks %.1f/tile (max %.0f)  chunks %.2f/entry (tile max %.0f)"
              "  nonempty entries %.0f/tile  sources %.2f/chunk  single-source chunks %.0f%%  entry sources max %.0f, >16 %.0f, >64 %.0f\n", g,
              t1 - t0, bc / (t1 - t0), bmax, nent > 0 ? ch / nent : 0.0, chmax, nne / (t1 - t0), ch > 0 ? nsrc / ch : 0.0,
              ch > 0 ? 100.0 * c1 / ch : 0.0, smax, s16, s64);
    }
  }

  // ---------------- 11. forward-solve gather lists (child order).  Sharded: a top front's rows list
  // only its top children (sv); its subtree-root children of this shard are listed in sx (the
  // external forward contribution, exchanged before the top forward solve).
  auto sv_child_ok = [&](int s, int c) { return !lb_member(c) && (!S.top(s) || S.top(c)); };
  S.sv_ptr.assign(S.row_ptr[ns] + 1, 0);
  for (int s = 0; s < ns; ++s)
    for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1]; ++qc) {
      const int c = S.child_list[qc];
      if (!sv_child_ok(s, c)) continue;
      const int uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
      for (int aa = 0; aa < uc; ++aa) S.sv_ptr[S.row_ptr[s] + S.rel[S.rel_ptr[c] + aa] + 1]++;
    }
  // a group under a top front (sharded) contributes to the external forward sums (sx) instead
  for (const auto& g : S.lb)
    if (!S.top(g.parent))
      for (int k = 0; k < g.m; ++k) S.sv_ptr[S.row_ptr[g.parent] + S.lb_gpos[g.gpos_off + k] + 1]++;
  for (int64_t t = 0; t < S.row_ptr[ns]; ++t) S.sv_ptr[t + 1] += S.sv_ptr[t];
  S.sv_src.assign(S.sv_ptr[S.row_ptr[ns]], 0);
  {
    std::vector<int64_t> fill(S.sv_ptr.begin(), S.sv_ptr.end() - 1);
    for (int s = 0; s < ns; ++s)
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1]; ++qc) {
        const int c = S.child_list[qc];
        if (!sv_child_ok(s, c)) continue;
        const int uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
        for (int aa = 0; aa < uc; ++aa) S.sv_src[fill[S.row_ptr[s] + S.rel[S.rel_ptr[c] + aa]]++] = S.uvec_off[c] + aa;
      }
    for (const auto& g : S.lb)  // after the regular children (fixed order)
      if (!S.top(g.parent))
        for (int k = 0; k < g.m; ++k) S.sv_src[fill[S.row_ptr[g.parent] + S.lb_gpos[g.gpos_off + k]]++] = g.uvec_off + k;
  }
  S.xoff.assign(ns, -1);
  S.xlen = 0;
  for (int s = 0; s < ns; ++s)
    if (S.top(s)) {
      S.xoff[s] = S.xlen;
      S.xlen += S.nrows[s];
    }
  S.sx_ptr.assign(S.xlen + 1, 0);
  S.sx_src.clear();
  if (S.xlen) {
    for (int s = 0; s < ns; ++s) {
      if (!S.top(s)) continue;
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1]; ++qc) {
        const int c = S.child_list[qc];
        if (S.top(c) || S.owner[c] != S.shard) continue;
        const int uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
        for (int aa = 0; aa < uc; ++aa) S.sx_ptr[S.xoff[s] + S.rel[S.rel_ptr[c] + aa] + 1]++;
      }
    }
    for (const auto& g : S.lb)  // this shard's members of groups under top fronts
      if (S.top(g.parent))
        for (int k = 0; k < g.m; ++k) S.sx_ptr[S.xoff[g.parent] + S.lb_gpos[g.gpos_off + k] + 1]++;
    for (int64_t t = 0; t < S.xlen; ++t) S.sx_ptr[t + 1] += S.sx_ptr[t];
    S.sx_src.assign(S.sx_ptr[S.xlen], 0);
    std::vector<int64_t> fill(S.sx_ptr.begin(), S.sx_ptr.end() - 1);
    for (int s = 0; s < ns; ++s) {
      if (!S.top(s)) continue;
      for (int64_t qc = S.child_ptr[s]; qc < S.child_ptr[s + 1]; ++qc) {
        const int c = S.child_list[qc];
        if (S.top(c) || S.owner[c] != S.shard) continue;
        const int uc = S.nrows[c] - (S.first[c + 1] - S.first[c]);
        for (int aa = 0; aa < uc; ++aa) S.sx_src[fill[S.xoff[s] + S.rel[S.rel_ptr[c] + aa]]++] = S.uvec_off[c] + aa;
      }
    }
    for (const auto& g : S.lb)  // after the regular children (fixed order)
      if (S.top(g.parent))
        for (int k = 0; k < g.m; ++k) S.sx_src[fill[S.xoff[g.parent] + S.lb_gpos[g.gpos_off + k]]++] = g.uvec_off + k;
  }
  stamp("11 (end)");
}

}  // namespace madipm
