// Multifrontal supernodal LDL^T for gfx950: numeric factorisation and triangular solves.
//
// Fronts are processed level by level (children before parents).  Per level:
//  * small fronts (r <= 128): ONE workgroup per front, the whole r x r front in LDS:
//    assemble (original entries + extend-add of the children's update blocks, children in a
//    fixed order -> deterministic), right-looking LDL^T of the w pivot columns, write the L panel,
//    D and the (r-w)^2 update block;
//  * big fronts (r > 128): the front lives in HBM (ld r).  Batched launches over all big fronts of
//    the level: column-block assembly, then per 64-column panel a panel kernel (diagonal block
//    factorised in LDS, rows below solved by forward substitution) and a trailing-update kernel
//    C -= (L D) L^T on 64x64 tiles with v_mfma_f64_16x16x4_f64.
// Quasi-definite KKT matrices (FixedRegularization(1e-8,-1e-8)) admit static
// pivoting in any symmetric order; zero / non-finite pivots are reported (is_factorized=false).
#include <algorithm>
#include <atomic>
#include <thread>
#include <array>
#include <map>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdio>

#include "ldl.hpp"

namespace madipm {
namespace {

constexpr int NT = 256;
typedef double dbl4 __attribute__((ext_vector_type(4)));

// Pin loaded values (an empty asm that "modifies" them) so the compiler keeps clamped loads
// unconditional instead of sinking them into the branch of their conditional use.  The asm needs the
// value, so it waits for the load: pin a batch only after ALL its loads are issued (pinning each load
// right after it serialised the LDS loads of the MFMA loops on the LDS latency).
#define LDL_PIN(x) asm volatile("" : "+v"(x))
#define LDL_PIN4(a) asm volatile("" : "+v"((a)[0]), "+v"((a)[1]), "+v"((a)[2]), "+v"((a)[3]))

__device__ __forceinline__ bool bad_pivot(double d, double tol) { return !(fabs(d) > tol) || isinf(d); }

// wave-synchronous LDS hand-off: LDS ops of one wave complete in order; keep the compiler from
// moving them across this point
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

template <class T>
__device__ __forceinline__ int64_t lower_bound_dev(const T* a, int64_t lo, int64_t hi, T key) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// initial forward value of row i of front s: own right-hand side entry, or (sharded top fronts) the
// exchanged sum of b and the other shards' subtree updates
__device__ __forceinline__ double fwd_init(const FrontTab& T, int s, int i, int w, int f0, const double* __restrict__ b) {
  // the caller's entry loaded unconditionally (clamped row): its two dependent loads issue beside the
  // xoff load instead of after it (a load under a branch waits for everything before it)
  const double bv = b[T.perm[f0 + min(i, max(w - 1, 0))]];
  const int64_t xo = T.xoff[s];
  if (xo >= 0) return T.xch[xo + i];
  return (i < w) ? bv : 0.0;
}

// Destination of update entry a of front s: its slot in the tree parent's contiguous gather range
// (T.upos >= 0) or the front's own update vector (read by the level kernels through sv_src).
__device__ __forceinline__ double* uvec_dst(const FrontTab& T, int s, int a, double* uvec) {
  const int64_t p = T.upos[T.rel_ptr[s] + a];
  return p >= 0 ? T.gbuf + p : uvec + T.uvec_off[s] + a;
}

// uvec_dst of the rows lane + 64 h (h < NH) of front s for a whole wave at once: the front's words
// once (uniform), every row's slot loaded unconditionally from a clamped row, then selected — uvec_dst
// per row under its row mask was three dependent round trips per row (k_fwd_tree: nine before the
// wait of every front, ~10 us of the level-1 fronts' start)
template <int NH>
__device__ __forceinline__ void uvec_dsts(const FrontTab& T, int s, int w, int r, int f0, bool act, int lane,
                                          double* uvec, double* xi, double* (&dst)[NH]) {
  const int64_t rp = T.rel_ptr[s], uo = T.uvec_off[s];
  const int amax = r - w - 1;  // (uniform) the front's last update row
  int64_t p[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) p[h] = amax >= 0 ? T.upos[rp + min(max(lane + 64 * h - w, 0), amax)] : -1;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int i = lane + 64 * h;
    dst[h] = (act && i >= w && i < r) ? (p[h] >= 0 ? T.gbuf + p[h] : uvec + uo + (i - w)) : xi + f0 + min(i, max(w - 1, 0));
  }
}

// HBM panel (r x w, ld r) -> LDS (ld rl), all threads, 16 independent loads per thread per batch
// (one HBM round trip per 4096 doubles: a 128 x 128 front is 4 round trips)
// (i, j) of the column-major indices q = q0, q0 + NT, q0 + 2 NT, ... of an r-row matrix: one integer
// division per thread instead of one per element (a division is ~15 VALU instructions, and the
// staging / write-out loops of a front are otherwise dominated by them)
struct ColWalk {
  int i, j, di, dj, r;
  __device__ __forceinline__ ColWalk(int q0, int r_, int stride = NT) : r(r_) {
    j = q0 / r_;
    i = q0 - j * r_;
    dj = stride / r_;
    di = stride - dj * r_;
  }
  __device__ __forceinline__ void next() {
    i += di;
    j += dj;
    if (i >= r) {
      i -= r;
      ++j;
    }
  }
};

__device__ __forceinline__ void stage_panel(const double* __restrict__ L, double* Ls, int r, int w, int rl) {
  const int nel = r * w;
  ColWalk wk(threadIdx.x, r);
  for (int base = 0; base < nel; base += NT * 16) {
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = base + k * NT + threadIdx.x;
      v[k] = (q < nel) ? L[q] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = base + k * NT + threadIdx.x;
      if (q < nel) Ls[wk.i + wk.j * rl] = v[k];
      wk.next();
    }
  }
}

__global__ void k_status_init(LDLStatus* st, int all = 0) {
  const uint64_t now = wall_clock64();
  if (all) {
    st->ticks = 0;
  } else if (st->t1 > st->t0) {
    st->ticks += st->t1 - st->t0;  // the previous factorisation
  }
  st->t0 = st->t1 = now;
  st->fail_pivot = INT_MAX;
  st->npos = st->nneg = st->nzero = 0;
  if (all) st->err = 0;
}

// ------------------------------------------------------------------ small fronts (LDS)
// Register-tiled right-looking LDL^T: the lower triangle of F is cut into 16 x 16 tiles of TS x TS
// entries (TS = 8 for r <= 128, 4 for r <= 64); thread q < 136 owns tile q in registers.  Step t:
// the owners of column t publish it through LDS (double-buffered), one barrier, every thread
// applies the rank-1 update to its tile.  The column loop is unrolled by TS so register indices
// are static.
template <int TS>
__global__ __launch_bounds__(NT) void k_small_factor(FrontTab T, const int32_t* __restrict__ fronts,
                                                     const double* __restrict__ Kx, double* __restrict__ arena,
                                                     const double* __restrict__ fscratch, double* __restrict__ D,
                                                     LDLStatus* st, double tol) {
  extern __shared__ __attribute__((aligned(16))) double F[];  // r x r, col-major, ld r (leaf fronts only)
  __shared__ double cb[2][16 * TS];
  __shared__ double dp[16 * TS];
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s];
  const int w = T.first[s + 1] - f0;
  const int r = T.nrows[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // tile of this thread: q -> (ti, tj), tj <= ti, 136 lower tiles of a 16 x 16 grid
  int ti = 0, tj = 0;
  {
    int q = tid;
    while (q > ti) {
      q -= ti + 1;
      ++ti;
    }
    tj = q;
  }
  const bool act = tid < 136 && ti * TS < r;
  const int i0 = ti * TS, j0 = tj * TS;
  double a[TS][TS];
  const int64_t fso = T.fs_off[s];
  if (fso >= 0) {
    // assembled by k_assemble (lower triangle, ld r): every thread loads its tile straight from HBM,
    // TS*TS independent loads in flight (no serialised staging copy); entries above the diagonal
    // are never read
    const double* __restrict__ Fs = fscratch + fso;
#pragma unroll
    for (int k = 0; k < TS; ++k)
#pragma unroll
      for (int c = 0; c < TS; ++c) {
        const int i = i0 + k, j = j0 + c;
        a[k][c] = (act && i < r && j <= i) ? Fs[i + (int64_t)j * r] : 0.0;
      }
  } else {  // leaf: original entries only, scattered into LDS
    for (int q = tid; q < r * r; q += NT) F[q] = 0.0;
    __syncthreads();
    for (int64_t q = T.asm_ptr[s] + tid; q < T.asm_ptr[s + 1]; q += NT) F[T.asm_dst[q]] = Kx[T.asm_src[q]];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TS; ++k)
#pragma unroll
      for (int c = 0; c < TS; ++c) a[k][c] = (act && i0 + k < r && j0 + c < r) ? F[(i0 + k) + (j0 + c) * r] : 0.0;
  }
  for (int t8 = 0; t8 < w; t8 += TS) {
#pragma unroll
    for (int c = 0; c < TS; ++c) {
      const int t = t8 + c;
      if (t < w) {  // block-uniform
        double* colb = cb[t & 1];
        if (act && tj == (t8 / TS)) {
#pragma unroll
          for (int k = 0; k < TS; ++k) colb[i0 + k] = a[k][c];
        }
        __syncthreads();
        const double dt = colb[t];
        if (tid == 0) dp[t] = dt;
        const double dinv = 1.0 / dt;
        double li[TS], cj[TS];
#pragma unroll
        for (int k = 0; k < TS; ++k) li[k] = (i0 + k > t) ? colb[i0 + k] * dinv : 0.0;
#pragma unroll
        for (int cc = 0; cc < TS; ++cc) cj[cc] = (j0 + cc > t) ? colb[j0 + cc] : 0.0;
#pragma unroll
        for (int k = 0; k < TS; ++k)
#pragma unroll
          for (int cc = 0; cc < TS; ++cc) a[k][cc] = fma(-li[k], cj[cc], a[k][cc]);
      }
    }
  }
  __syncthreads();
  // write-out: L panel (ld r; d on the diagonal, zeros above), D, lower triangle of U (ld r - w)
  double* __restrict__ L = arena + T.l_off[s];
  double* __restrict__ Uo = arena + T.u_off[s];
  const int u = r - w;
  if (act) {
#pragma unroll
    for (int c = 0; c < TS; ++c) {
      const int j = j0 + c;
      if (j >= r) continue;
      if (j < w) {
        const double dj = dp[j];
        const double dinv = 1.0 / dj;
#pragma unroll
        for (int k = 0; k < TS; ++k) {
          const int i = i0 + k;
          if (i < r) L[i + (int64_t)j * r] = (i > j) ? a[k][c] * dinv : (i == j ? dj : 0.0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < TS; ++k) {
          const int i = i0 + k;
          if (i < r && i >= j) Uo[(i - w) + (int64_t)(j - w) * u] = a[k][c];
        }
      }
    }
  }
  // upper part of the L panel (rows above the tile grid's lower triangle): zeros, so the solves can
  // read the r x w panel as stored
  for (int j = wv; j < w; j += NT / 64)
    for (int i = lane; i < j - (j % TS); i += 64) L[i + (int64_t)j * r] = 0.0;
  if (tid < w) {
    const double d = dp[tid];
    D[f0 + tid] = d;
    if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + tid + 1);
  }
}

// ------------------------------------------------------------------ micro fronts (w <= 2, r <= 32)
// The leaf level of the K2 trees (~1e5 fronts: one or two x columns and their rows).  16 lanes per
// front, 16 fronts per workgroup, lane l owns rows l and l + 16; no frontal matrix: a leaf's original
// entries live in its pivot columns only, so L = F(:, 0:w) D^-1 (2 x 2 block at most) and the update
// block is U = -L D L^T (rows >= w), written column by column, coalesced over the group's lanes.
constexpr int MG = 16;
__global__ __launch_bounds__(NT) void k_micro_factor(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                     const double* __restrict__ Kx, double* __restrict__ arena,
                                                     double* __restrict__ D, LDLStatus* st, double tol) {
  __shared__ double Fs[NT / MG][64];  // columns 0 / 1 of F (rows 0..31); later l_i0 d0 / l_i1 d1
  const int g = threadIdx.x / MG, l = threadIdx.x & (MG - 1);
  const int q = blockIdx.x * (NT / MG) + g;
  const bool live = q < nf;
  const int s = fronts[live ? q : nf - 1];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  double* F = Fs[g];
#pragma unroll
  for (int k = 0; k < 4; ++k) F[l + 16 * k] = 0.0;
  wave_sync();
  for (int64_t e = T.asm_ptr[s] + l; e < T.asm_ptr[s + 1]; e += MG) {
    // original entries lie in the front's own (w <= 2) columns: d < 2 r, no division
    const int d = (int)T.asm_dst[e];
    const int lc = d >= r ? 1 : 0, lr = d - lc * r;
    F[lr + 32 * lc] = Kx[T.asm_src[e]];
  }
  wave_sync();
  const double d0 = F[0];
  const double f10 = F[1];
  const double l10 = (w == 2) ? f10 / d0 : 0.0;
  const double d1 = (w == 2) ? F[33] - l10 * f10 : 0.0;
  double li0[2], li1[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = l + 16 * h;
    li0[h] = 0.0;
    li1[h] = 0.0;
    if (i >= w && i < r) {
      li0[h] = F[i] / d0;
      if (w == 2) li1[h] = (F[32 + i] - li0[h] * f10) / d1;
    }
  }
  wave_sync();
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // scaled columns for the update: U_ab = -(l_a0 (d0 l_b0) + l_a1 (d1 l_b1))
    const int i = l + 16 * h;
    F[i] = li0[h] * d0;
    F[32 + i] = li1[h] * d1;
  }
  wave_sync();
  if (!live) return;
  double* __restrict__ L = arena + T.l_off[s];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = l + 16 * h;
    if (i < r) {
      L[i] = (i == 0) ? d0 : (i >= w ? li0[h] : l10);
      if (w == 2) L[i + r] = (i == 0) ? 0.0 : (i == 1 ? d1 : li1[h]);
    }
  }
  if (l == 0) {
    D[f0] = d0;
    if (bad_pivot(d0, tol)) atomicMin(&st->fail_pivot, f0 + 1);
    if (w == 2) {
      D[f0 + 1] = d1;
      if (bad_pivot(d1, tol)) atomicMin(&st->fail_pivot, f0 + 2);
    }
  }
  const int u = r - w;
  double* __restrict__ Uo = arena + T.u_off[s];
  for (int b = 0; b < u; ++b) {
    const double sb0 = F[w + b], sb1 = F[32 + w + b];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int a = l + 16 * h - w;  // U row of this lane's row
      if (a >= b && a < u) Uo[a + (int64_t)b * u] = -(li0[h] * sb0 + li1[h] * sb1);
    }
  }
}

// forward / backward solves of micro fronts (same lane layout); x_0, x_1 broadcast within the group
__global__ __launch_bounds__(NT) void k_fwd_micro(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                  const double* __restrict__ arena, const double* __restrict__ b,
                                                  double* __restrict__ xi, double* __restrict__ uvec) {
  const int g = threadIdx.x / MG, l = threadIdx.x & (MG - 1);
  const int q = blockIdx.x * (NT / MG) + g;
  const bool live = q < nf;
  const int s = fronts[live ? q : nf - 1];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const double* __restrict__ L = arena + T.l_off[s];
  double v[2], c0[2], c1[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = l + 16 * h;
    double vi = 0.0, a0 = 0.0, a1 = 0.0;
    if (i < r) {
      vi = fwd_init(T, s, i, w, f0, b);
      const int64_t e = T.row_ptr[s] + i;
      const int64_t p1 = T.sv_ptr[e + 1];
      for (int64_t p = T.sv_ptr[e]; p < p1; ++p) vi += uvec[T.sv_src[p]];
      a0 = L[i];
      if (w == 2) a1 = L[i + r];
    }
    v[h] = vi;
    c0[h] = a0;
    c1[h] = a1;
  }
  const double x0 = __shfl(v[0], 0, MG);
  const double l10 = __shfl(c0[0], 1, MG);
  const double x1 = (w == 2) ? __shfl(v[0], 1, MG) - l10 * x0 : 0.0;
  if (!live) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = l + 16 * h;
    if (i < w) {
      xi[f0 + i] = (i == 0) ? x0 : x1;
    } else if (i < r) {
      *uvec_dst(T, s, i - w, uvec) = (v[h] - c0[h] * x0) - c1[h] * x1;
    }
  }
}

__global__ __launch_bounds__(NT) void k_bwd_micro(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                  const double* __restrict__ arena, const double* __restrict__ D,
                                                  double* __restrict__ xi, double* __restrict__ out) {
  const int g = threadIdx.x / MG, l = threadIdx.x & (MG - 1);
  const int q = blockIdx.x * (NT / MG) + g;
  const bool live = q < nf;
  const int s = fronts[live ? q : nf - 1];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const double* __restrict__ L = arena + T.l_off[s];
  const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
  double a0 = 0.0, a1 = 0.0, l10 = 0.0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = l + 16 * h;
    if (i >= w && i < r) {
      const double x = xi[rows[i]];  // final: ancestors
      a0 = fma(L[i], x, a0);
      if (w == 2) a1 = fma(L[i + r], x, a1);
    }
    if (i == 1 && w == 2) l10 = L[1];
  }
#pragma unroll
  for (int o = MG / 2; o > 0; o >>= 1) {
    a0 += __shfl_xor(a0, o, MG);
    a1 += __shfl_xor(a1, o, MG);
  }
  l10 = __shfl(l10, 1, MG);
  if (!live || l != 0) return;
  const double v1 = (w == 2) ? xi[f0 + 1] / D[f0 + 1] - a1 : 0.0;
  const double v0 = xi[f0] / D[f0] - a0 - l10 * v1;
  xi[f0] = v0;
  if (T.wout[s]) out[T.perm[f0]] = v0;
  if (w == 2) {
    xi[f0 + 1] = v1;
    if (T.wout[s]) out[T.perm[f0 + 1]] = v1;
  }
}

// Fronts with r <= 32: one WAVE per front, 4 fronts per workgroup (the leaf level has ~10^5 of them).
// Lane l works on row l & 31 and the columns of parity l >> 5; wave-synchronous right-looking LDL^T.
constexpr int TINY = 32;
__global__ __launch_bounds__(NT) void k_tiny_factor(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                    const double* __restrict__ Kx, double* __restrict__ arena,
                                                    const double* __restrict__ fscratch, double* __restrict__ D,
                                                    LDLStatus* st, double tol) {
  constexpr int LD = TINY + 1;
  __shared__ double Fs[4][TINY * LD];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = blockIdx.x * 4 + wv;
  if (q >= nf) return;
  const int s = fronts[q];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  double* F = Fs[wv];
  const int i = lane & 31, par = lane >> 5;
  for (int j = par; j < r; j += 2) F[i + j * LD] = 0.0;
  wave_sync();
  const int64_t fso = T.fs_off[s];
  if (fso < 0) {
    for (int64_t e = T.asm_ptr[s] + lane; e < T.asm_ptr[s + 1]; e += 64) {
      const int d = (int)T.asm_dst[e], dj = d / r;  // d < r^2: 32-bit division
      F[(d - dj * r) + dj * LD] = Kx[T.asm_src[e]];
    }
  } else {
    const double* __restrict__ Fg = fscratch + fso;
    for (int j = par; j < r; j += 2)
      if (i >= j && i < r) F[i + j * LD] = Fg[i + j * r];
  }
  wave_sync();
  for (int t = 0; t < w; ++t) {
    const double dinv = 1.0 / F[t + t * LD];
    const double lit = F[i + t * LD] * dinv;
    for (int j = t + 1 + par; j < r; j += 2)
      if (i >= j && i < r) F[i + j * LD] -= lit * F[j + t * LD];
    wave_sync();
  }
  double* __restrict__ L = arena + T.l_off[s];
  for (int t = par; t < w; t += 2) {
    const double d = F[t + t * LD];
    if (i < r) L[i + (int64_t)t * r] = (i > t) ? F[i + t * LD] / d : (i == t ? d : 0.0);
    if (i == 0) {
      D[f0 + t] = d;
      if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + t + 1);
    }
  }
  const int u = r - w;
  double* __restrict__ Uo = arena + T.u_off[s];
  for (int b = par; b < u; b += 2)
    if (i >= b && i < u) Uo[i + (int64_t)b * u] = F[(w + i) + (w + b) * LD];
}

// ------------------------------------------------------------------ assembly (all big fronts, small fronts with children)
// Phase 1 (flat, thread per chunk): part[c] = sum of the <= kChunk sources of chunk c, in order.
// Chunk sums: thread per chunk of <= kChunk sources, summed in source order.  Sources are int32
// when the arena and K fit (IDX = int32_t), else int64.
template <typename IDX>
__device__ __forceinline__ void asm_chunk_sum(const int64_t* __restrict__ ids, const int64_t* __restrict__ gchunk,
                                              const IDX* __restrict__ gsrc, int64_t c0, int64_t ci,
                                              const double* __restrict__ Kx, const double* __restrict__ arena,
                                              double* __restrict__ part, bool sc1) {
  const int64_t c = ids[c0 + ci];  // the chunks of the launch's chunk-path tiles (asm_chunks_lds)
  const int64_t p0 = gchunk[c], p1 = gchunk[c + 1];
  constexpr int KC = SymbolicPlan::kChunk;
  // every index, then every value operand in flight before the sum: unconditional loads (clamped
  // index, selected source pointer), masked at the sum — predicated loads compiled into branches
  // with a wait each
  int64_t q[KC];
#pragma unroll
  for (int u = 0; u < KC; ++u) q[u] = (int64_t)gsrc[min(p0 + u, max(p1 - 1, p0))];
  double x[KC];
#pragma unroll
  for (int u = 0; u < KC; ++u) x[u] = *((q[u] < 0) ? Kx + ~q[u] : arena + q[u]);
  double v = 0.0;
#pragma unroll
  for (int u = 0; u < KC; ++u)
    if (p0 + u < p1) v += x[u];
  if (sc1)
    __hip_atomic_store(part + c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    part[c] = v;
}
template <typename IDX>
__global__ __launch_bounds__(NT) void k_asm_chunks(const int64_t* __restrict__ ids, const int64_t* __restrict__ gchunk,
                                                   const IDX* __restrict__ gsrc, int64_t c0, int64_t n,
                                                   const double* __restrict__ Kx, const double* __restrict__ arena,
                                                   double* __restrict__ part, int32_t* cflag, int epoch) {
  const int64_t ci = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (ci < n) asm_chunk_sum(ids, gchunk, gsrc, c0, ci, Kx, arena, part, cflag != nullptr);
  if (cflag) {  // the root tail (LDLSolver::root_async_): handed to its k_assemble on the side stream
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // form R1: write-through sums drained, one flag
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(cflag + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Phase 2: one workgroup (1024 threads) per 64x64 lower tile of F (SymbolicPlan step 10), assembled
// in an LDS tile: entry = sum of its chunk sums in chunk order (asm_chunks_lds), then the big
// children's update blocks record by record in child order (asm_children_lds); thread t writes out
// the entries (row t & 63, columns t >> 6 + 16 k), k < 4.  No atomics, deterministic.  The tile is written to the front (big: arena, ld r; small: scratch, ld r).
constexpr int ANT = 1024;
// tiles of at most kAsmLdsWin windows of kAsmLdsSrc sources (one window in launches of < 256 tiles:
// their few workgroups would carry a root's whole gather — ex10's 3 root tiles of 32k sources took
// 1816 -> 1645 iters/s through the LDS path; the chunk pass spreads it over the chip) gather them into
// LDS and sum them there (asm_chunks_lds), without k_asm_chunks.  (r5_zi: the source count rode in gchk's top 16 bits and was read back with a signed
// shift — a tile of >= 2^15 sources read a negative count and summed nothing; unsigned now)
// The windows straddle: an entry whose sources cross a window boundary carries its running chunk
// sum to the next (the straddle branch below); MADIPM_ASM_LDS_WIN=n (tests) puts every tile of up to
// n windows on this path, whatever its launch size.  kAsmLdsWinMax bounds n: the count rides in 16
// bits of gchk, and the kernel checks it against FrontTab::asm_src_cap (kErrAsmSrc).
constexpr int kAsmLdsSrc = 5 * ANT, kAsmLdsWin = 4, kAsmLdsWinMax = 12;
static_assert(kAsmLdsSrc * kAsmLdsWinMax < 65536, "the tile's source count rides in 16 bits");
// The tile's chunk sums into the LDS tile Ts (64 x 64, column-major, ld 64; zeroed first): the
// tile's nonempty entries (its g_ptr list: ne, then position | first chunk << 12 per entry, then the
// chunk count << 12; ne also in the device tile's gptr >> 48, bit 47: the source path below) spread
// over the threads, up to 4 per thread, each entry's chunk sums added in
// chunk order, CU per entry and round in flight.  A wave past the list issues no load.  Ends with a
// barrier.  (r3-r5 read a dense 4097-offset table per tile: 32 KB of offset loads for a tree front's
// tile of ~40 nonempty entries, neos.)
template <int CU, typename IDX, int WS = 5 * 1024>
__device__ __forceinline__ void asm_chunks_lds(const SymbolicPlan::AsmTile& tl, const int32_t* __restrict__ gent,
                                               const double* __restrict__ part, const IDX* __restrict__ gsrc,
                                               const double* __restrict__ Kx, const double* __restrict__ arena,
                                               double* Ts, double* vals, int32_t* err, int src_cap) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
#pragma unroll
  for (int m = 0; m < 4; ++m) Ts[(wv + 16 * m) * 64 + lane] = 0.0;
  if (tl.gptr >= 0 && ((tl.gptr >> 47) & 1)) {  // uniform: a tile of <= kAsmLdsWin windows of sources
    // Its entry list holds source offsets (pos | first source << 12): the tile's sources are gathered
    // straight into LDS (thread per source, consecutive indices: coalesced), then each entry sums its
    // sources from LDS in 8-source chunks, in order — k_asm_chunks' partial sums, then their sum, as
    // the chunk path: the same bits, without the chunk launch and its partials in HBM.
    const int32_t* __restrict__ ge = gent + (tl.gptr & (((int64_t)1 << 47) - 1));
    const int ne = (int)(tl.gptr >> 48);
    const int64_t sb = tl.gchk & (((int64_t)1 << 48) - 1);
    int ns = (int)((uint64_t)tl.gchk >> 48);  // unsigned: a count >= 2^15 sets the sign bit
    if (ns > src_cap) {  // uniform: the plan promised at most kAsmLdsWinMax windows — never a silent sum
      if (tid == 0) __hip_atomic_fetch_or(err, kErrAsmSrc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ns = 0;
    }
    int pos[4], s0[4], s1[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      pos[m] = -1;
      s0[m] = s1[m] = 0;
      if (wbase + ANT * m < ne) {  // uniform
        const int k = tid + ANT * m, kk = min(k, ne - 1);
        const int e0 = ge[1 + kk], e1 = ge[2 + kk];
        s0[m] = e0 >> 12;
        s1[m] = k < ne ? e1 >> 12 : s0[m];
        pos[m] = k < ne ? (e0 & 4095) : -1;
      }
    }
    // windows of WS sources; an entry whose sources straddle a window carries its running
    // chunk sum to the next (the chunk boundaries stay every kChunk sources from the entry's first)
    double v[4] = {0.0, 0.0, 0.0, 0.0}, cs[4] = {0.0, 0.0, 0.0, 0.0};
    int nx[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) nx[m] = s0[m];
    for (int w0 = 0; w0 < ns; w0 += WS) {  // uniform
      const int wn = min(WS, ns - w0);
      int64_t q[WS / ANT];
#pragma unroll
      for (int u = 0; u < WS / ANT; ++u)
        q[u] = (wbase + ANT * u < wn) ? (int64_t)gsrc[sb + w0 + min(tid + ANT * u, wn - 1)] : 0;
      double x[WS / ANT];
#pragma unroll
      for (int u = 0; u < WS / ANT; ++u)
        x[u] = (wbase + ANT * u < wn) ? *((q[u] < 0) ? Kx + ~q[u] : arena + q[u]) : 0.0;
#pragma unroll
      for (int u = 0; u < WS / ANT; ++u)
        if (tid + ANT * u < wn) vals[tid + ANT * u] = x[u];
      __syncthreads();  // the window's sources (and the zeroed tile)
      const int we = w0 + wn;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (pos[m] < 0 || nx[m] >= s1[m] || nx[m] >= we) continue;
        if (nx[m] == s0[m] && s1[m] <= we) {  // the whole entry in this window (the common case)
          for (int c = s0[m]; c < s1[m]; c += SymbolicPlan::kChunk) {
            double ck = 0.0;
#pragma unroll
            for (int u = 0; u < SymbolicPlan::kChunk; ++u)
              if (c + u < s1[m]) ck += vals[c + u - w0];
            v[m] += ck;
          }
          nx[m] = s1[m];
        } else {
          const int e = min(s1[m], we);
          for (; nx[m] < e; ++nx[m]) {
            cs[m] += vals[nx[m] - w0];
            if (((nx[m] + 1 - s0[m]) % SymbolicPlan::kChunk) == 0 || nx[m] + 1 == s1[m]) {
              v[m] += cs[m];
              cs[m] = 0.0;
            }
          }
        }
      }
      __syncthreads();  // every entry done with the window before the next overwrites it
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (pos[m] >= 0) Ts[pos[m]] = v[m];
    __syncthreads();
    return;
  }
  __syncthreads();
  if (tl.gptr >= 0) {  // uniform
    const int32_t* __restrict__ ge = gent + (tl.gptr & (((int64_t)1 << 47) - 1));
    const double* __restrict__ pc = part + tl.gchk;
    const int ne = (int)(tl.gptr >> 48);
    int pos[4], c0[4], c1[4], len = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      pos[m] = -1;
      c0[m] = c1[m] = 0;
      if (wbase + ANT * m < ne) {  // uniform
        const int k = tid + ANT * m, kk = min(k, ne - 1);
        const int e0 = ge[1 + kk], e1 = ge[2 + kk];
        c0[m] = e0 >> 12;
        c1[m] = k < ne ? e1 >> 12 : c0[m];
        pos[m] = k < ne ? (e0 & 4095) : -1;
        len = max(len, c1[m] - c0[m]);
      }
    }
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < len; it += CU) {
      double x[4][CU];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int u = 0; u < CU; ++u) x[m][u] = pc[min(c0[m] + it + u, max(c1[m] - 1, c0[m]))];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int u = 0; u < CU; ++u)
          if (c0[m] + it + u < c1[m]) v[m] += x[m][u];
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (pos[m] >= 0) Ts[pos[m]] = v[m];
  }
  __syncthreads();
}

// The big children's blocks added into the LDS tile Ts (64 x 64, column-major, ld 64), record by
// record in child order (BigChildRec: a child's hits on the tile are the na x nb block of its U at
// (a0, b0), <= 1024 entries per record): thread e takes the record's entry e — consecutive threads
// read consecutive rows of the child's column, and a wave past the record's entries issues nothing —
// and a barrier separates the records.  The loads of ABR records are in flight before the first
// add.  r3-r5 had every thread pull its own four entries from every child through row / column maps:
// ~5% of those loads hit (neos), and the address unit was the bound (TA busy 83%, r6_b).
template <int ABR>
__device__ __forceinline__ void asm_children_lds(int bt0, int bt1, const BigChildRec* __restrict__ brec,
                                                 const double* __restrict__ arena, double* Ts) {
  const int tid = threadIdx.x;
  const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
  for (int kc = bt0; kc < bt1; kc += ABR) {  // uniform
    const int nk = min(ABR, bt1 - kc);
    // the batch's record headers first (scalar loads, none waited for alone), then its entry loads
    int4 h0[ABR], h1[ABR];
#pragma unroll
    for (int k = 0; k < ABR; ++k) {
      const int4* __restrict__ hp = reinterpret_cast<const int4*>(brec + kc + min(k, nk - 1));
      h0[k] = hp[0];
      h1[k] = hp[1];
    }
    // the loaded values are only combined at the adds: nothing inside the uniform branch waits
    double x[ABR];
    int rb[ABR], cbt[ABR];
    uint32_t ok = 0;
#pragma unroll
    for (int k = 0; k < ABR; ++k) {
      x[k] = 0.0;
      rb[k] = cbt[k] = 0;
      const int64_t uo = (int64_t)(((uint64_t)(uint32_t)h0[k].y << 32) | (uint32_t)h0[k].x);
      const int ldc = h0[k].z, a0 = h0[k].w, b0 = h1[k].x;
      const int na = h1[k].y & 0xffff, nab = na * ((uint32_t)h1[k].y >> 16);
      if (k < nk && wbase < nab) {  // uniform
        const int e = min(tid, nab - 1);
        const int j = (int)(((uint32_t)e * (uint32_t)h1[k].z) >> 16), i = e - j * na;
        const int ra = a0 + i, cb = b0 + j;
        x[k] = arena[uo + ra + (int64_t)cb * ldc];
        const BigChildRec* __restrict__ R = brec + kc + k;
        rb[k] = R->rows[i];
        cbt[k] = R->cols[j];
        ok |= (uint32_t)(tid < nab && ra >= cb) << k;
      }
    }
#pragma unroll
    for (int k = 0; k < ABR; ++k)
      if (k < nk) {  // uniform
        if ((ok >> k) & 1u) Ts[cbt[k] * 64 + rb[k]] += x[k];
        __syncthreads();
      }
  }
}

// k_assemble runs two tiles per CU (8 waves per SIMD, <= 64 VGPRs: 2 chunk sums per entry and
// round, 8 big-child records per batch; 32 KB of LDS each).  Launches of few tiles (a root's
// high-fan-in assembly: ex10's 3 root tiles, up to 8 chunks per entry) take the CU = 8 instance,
// one round of chunk loads per entry, one tile per CU.
template <int CU, typename IDX>
__global__ __launch_bounds__(ANT, CU == 2 ? 8 : 4) void k_assemble(FrontTab T, const SymbolicPlan::AsmTile* __restrict__ tiles,
                                                     const int32_t* __restrict__ gptr, const double* __restrict__ part,
                                                     const BigChildRec* __restrict__ brec, double* __restrict__ arena,
                                                     double* __restrict__ fscratch, const IDX* __restrict__ gsrc,
                                                     const double* __restrict__ Kx, int32_t* go, int go_epoch,
                                                     const int32_t* cwait, int ncw) {
  constexpr int WS = kAsmLdsSrc;
  __shared__ double Ts[64 * 64];
  extern __shared__ __attribute__((aligned(16))) double vals[];  // WS doubles (dynamic: past 64 KB of static LDS)
  if (ncw > 0) {  // the root tail's assembly on the side stream: the chunk pass's blocks (main stream) first
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      for (int q0 = 0; q0 < ncw; q0 += 64) {
        int spins = 0;
        for (;;) {
          const bool ok = q0 + lane >= ncw ||
                          __hip_atomic_load(cwait + q0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == go_epoch;
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1 << 25)) {
            if (lane == 0) atomicOr(T.err, kErrHandoff);
            break;
          }
        }
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the chunk sums, the children's blocks, K
  }
  const SymbolicPlan::AsmTile tl = tiles[blockIdx.x];
  const int s = tl.front, ti = tl.tij & 0xffff, tj = (tl.tij >> 16) & 0x7fff;
  const bool acc = tl.tij < 0;  // SymbolicPlan::kAccumulate: F += tile (sharded top fronts, phase 2)
  const int r = T.nrows[s];
  const int I0 = ti * 64, J0 = tj * 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  asm_chunks_lds<CU, IDX, WS>(tl, gptr, part, gsrc, Kx, arena, Ts, vals, T.err, T.asm_src_cap);
  asm_children_lds<8>(tl.bt0, tl.bt1, brec, arena, Ts);
  double v[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) v[m] = Ts[(wv + 16 * m) * 64 + lane];
  const int64_t fso = T.fs_off[s];
  double* __restrict__ F = (fso >= 0 ? fscratch + fso : arena + T.l_off[s]);
  const int i = I0 + lane;
  const int img = (fso >= 0) ? T.fs_img[s] : 0;  // tree front: write its LDS image
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = J0 + wv + 16 * m;
    if (i < r && j < r && i >= j) {
      const int64_t q = !img ? i + (int64_t)j * r : (r > 128 ? (int64_t)((j * (2 * r - j - 1)) >> 1) + i : i + (int64_t)j * (r | 1));
      const double x = acc ? F[q] + v[m] : v[m];
      if (go)
        __hip_atomic_store(F + q, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (st_sc1): to the root tail
      else
        F[q] = x;
    }
  }
  if (go) {  // the root tail's release (LDLSolver::root_async_): the last tile out raises go[0]
    // (form R1: write-through stores drained, one relaxed counter / flag per workgroup)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(go + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == (int)gridDim.x - 1) {
        __hip_atomic_store(go + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(go, go_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Single-panel big fronts (SymbolicPlan::fused, w <= 64): once k_big_diag / k_big_trsm have written
// the panel's L and D, ONE pass per 64x64 tile assembles the trailing entries (asm_chunks_lds and
// asm_children_lds, as k_assemble) and subtracts L_I D L_J^T (K = w, f64 MFMA 16x16x4) before the tile's only store.  The
// level path moved every trailing entry through HBM three times (k_assemble's store, k_big_upd128's
// load and store); neos' 1220 skinny big fronts (w <= 39, r up to 2.7k) are mostly trailing matrix.
// Each of the 16 waves owns one 16x16 block, and each thread assembles exactly the four entries its
// MFMA result holds (no result tile in LDS); the operands are staged [k][row] for the K = kmax rows
// the launch needs (dynamic LDS: 2 x kmax x 80 doubles, 51 KB at neos' w <= 39, beside the 32 KB
// assembled tile).  Column block 0's tiles (assembled for the panel by k_assemble) get their columns >= w here.
// Operands and MFMA order are k_big_upd128's (A = L_J, B = (L D)_I, K ascending, one accumulator):
// the same U bit for bit.
constexpr int AU_LDT = 80;  // [k][row] operand stride (conflict-free ds_read_b64 for the 16x4 pattern)
template <typename IDX>
__global__ __launch_bounds__(ANT) void k_asm_update(FrontTab T, const SymbolicPlan::AsmTile* __restrict__ tiles,
                                                    const int32_t* __restrict__ gptr, const double* __restrict__ part,
                                                    const BigChildRec* __restrict__ brec, double* __restrict__ arena,
                                                    const double* __restrict__ D, int kmax, const IDX* __restrict__ gsrc,
                                                    const double* __restrict__ Kx) {
  extern __shared__ __attribute__((aligned(16))) double AUs[];
  __shared__ double Ts[64 * 64];     // the assembled tile
  double* Wt = AUs;                  // (L D)[I rows], kmax x AU_LDT
  double* Lt = AUs + kmax * AU_LDT;  // L[J rows]
  double* vals = AUs + 2 * kmax * AU_LDT;  // the tile's sources (asm_chunks_lds), kAsmLdsSrc doubles
  const SymbolicPlan::AsmTile tl = tiles[blockIdx.x];
  const int s = tl.front, ti = tl.tij & 0xffff, tj = (tl.tij >> 16) & 0x7fff;
  const int r = T.nrows[s], f0 = T.first[s], w = T.first[s + 1] - f0;
  const int I0 = ti * 64, J0 = tj * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int bi = wv & 3, bj = wv >> 2;
  double* __restrict__ F = arena + T.l_off[s];
  // the panel rows of I and J, [k][row]: thread (row lane, k = wv + 16 q); clamped loads, masked stores
  {
    double a[4], b[4], d[4];
    const int ri = min(I0 + lane, r - 1), rj = min(J0 + lane, r - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kc = min(wv + 16 * q, w - 1);
      a[q] = F[ri + (int64_t)kc * r];
      b[q] = F[rj + (int64_t)kc * r];
      d[q] = D[f0 + kc];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = wv + 16 * q;
      if (k < kmax) {
        Wt[k * AU_LDT + lane] = (k < w && I0 + lane < r) ? a[q] * d[q] : 0.0;
        Lt[k * AU_LDT + lane] = (k < w && J0 + lane < r) ? b[q] : 0.0;
      }
    }
  }
  // this thread's entries = its MFMA result's: row 16 bi + (lane & 15), column 16 bj + (lane >> 4) + 4 g
  int ei[4], ej[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    ei[g] = 16 * bi + (lane & 15);
    ej[g] = 16 * bj + (lane >> 4) + 4 * g;
  }
  asm_chunks_lds<4, IDX, kAsmLdsSrc>(tl, gptr, part, gsrc, Kx, arena, Ts, vals, T.err, T.asm_src_cap);
  asm_children_lds<8>(tl.bt0, tl.bt1, brec, arena, Ts);
  double v[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) v[g] = Ts[ej[g] * 64 + ei[g]];
  __syncthreads();  // the operands in LDS
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  const int nks = (w + 3) >> 2;
  for (int ks = 0; ks < nks; ++ks) {  // wave-uniform
    const int kk = 4 * ks + (lane >> 4);
    const double a = Lt[kk * AU_LDT + 16 * bj + (lane & 15)];
    const double b = Wt[kk * AU_LDT + 16 * bi + (lane & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int i = I0 + ei[g], j = J0 + ej[g];
    if (i < r && j < r && i >= j && j >= w) F[i + (int64_t)j * r] = v[g] - acc[g];
  }
}

// ------------------------------------------------------------------ big fronts (HBM)
// Big-front kernels read their (front, item) pair from the launch's task list.
__device__ __forceinline__ void task_of(const int32_t* __restrict__ list, int& s, int& item) {
  const int2 t = reinterpret_cast<const int2*>(list)[blockIdx.x];
  s = t.x;
  item = t.y;
}


// ---- blocked 64x64 panel kernels (16x16 sub-blocks; wave w owns sub-block row w)
// Layout conventions: A64 = LDS 64x64 tile, col-major, ld 65.  MFMA f64 16x16x4 fragments:
// A operand lane l = (m = l & 15, k = l >> 4); B operand lane l = (k = l >> 4, n = l & 15);
// result D lane l, element g = (m = (l >> 4) + 4 g, n = l & 15).
constexpr int LDA = 65;
constexpr int LDM = 17;

// Blocked LDL^T of the LDS tile A64 (lower part valid) by 4 waves: after the call A64 holds the
// strictly-lower L (diagonal untouched), Dl the pivots and Ms[K] the four M_K blocks.
template <bool PK, bool RCP>
__device__ __forceinline__ void factor16r(double* A, int r, int ld, int k0, int kw, double* Dl, double* MK, int lane);
// (the pipelined schedule of blocked_factor_pipe on this tile was measured slower — supportcase10
// k_big_diag 18.1 -> 19.8 us, r3: four pivot blocks leave the other waves too little to overlap)
__device__ __forceinline__ void diag64(double* A64, double* Dl, double* Ms, int tid) {
  const int lane = tid & 63, w = tid >> 6;
  for (int K = 0; K < 4; ++K) {
    if (w == K) factor16r<false, true>(A64, 64, LDA, 16 * K, 16, Dl, Ms + K * 16 * LDM, lane);
    __syncthreads();
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    if (w > K) {  // L_wK = A_wK M_K
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + (lane >> 4);
        const double av = A64[(16 * w + (lane & 15)) + (16 * K + k) * LDA];
        const double bv = Ms[K * 16 * LDM + k * LDM + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
    }
    __syncthreads();  // every wave has read A_wK before it is overwritten
    if (w > K) {
#pragma unroll
      for (int g = 0; g < 4; ++g) A64[(16 * w + (lane >> 4) + 4 * g) + (16 * K + (lane & 15)) * LDA] = acc[g];
    }
    __syncthreads();
    if (w > K) {  // A_wJ -= (L_wK D_K) L_JK^T, K < J <= w
      for (int J = K + 1; J <= w; ++J) {
        dbl4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int k = 4 * ks + (lane >> 4);
          const double av = A64[(16 * w + (lane & 15)) + (16 * K + k) * LDA] * Dl[16 * K + k];
          const double bv = A64[(16 * J + (lane & 15)) + (16 * K + k) * LDA];
          u = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, u, 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) A64[(16 * w + (lane >> 4) + 4 * g) + (16 * J + (lane & 15)) * LDA] -= u[g];
      }
    }
    // next K: wave K+1 factors the block it just updated itself; the others read M_{K+1} after
    // the barrier at the top of the next iteration
  }
  __syncthreads();
}

// ------------------------------------------------------------------ small fronts, blocked (r <= 128)
// The front lives in LDS (ld = r | 1).  Pivots are taken 16 at a time: one wave factors the 16 x 16
// diagonal block (wave-synchronous, no barriers; identity-padded when fewer than 16 pivots remain),
// the rows below get L = A M_K on f64 MFMA, and the trailing lower triangle is updated tile by tile
// (16 x 16 tiles, C -= (L_I D) L_J^T, f64 MFMA 16x16x4) — 3 barriers per 16 pivots instead of one per
// pivot.  Row/column blocks of a step start right after its last pivot (not 16-aligned), exactly
// like the big-front path.
// Factor the kw (<= 16) pivots at (k0, k0) of A (ld) with ONE wave: strictly-lower L_KK into A,
// pivots into Dl[k0 + t], M_K = L_KK^{-T} D^{-1} (16 x 16, ld LDM, identity-padded) into MK.
template <bool PK>
__device__ __forceinline__ int fidx(int i, int j, int r, int ld) {
  return PK ? ((j * (2 * r - j - 1)) >> 1) + i : i + j * ld;
}


// PK = false: square storage, ld = r | 1 (r <= 128); PK = true: packed lower-triangular columns
// (r <= 192 fits LDS), element (i, j >= ...) at j (2r - j - 1) / 2 + i

// Factor the 16 x 16 diagonal block K at (k0, k0) of the front in LDS with ONE wave (identity-padded
// past kw): writes the strictly-lower unit L_KK into A, d into Dl[k0 + i] and M_K = L_KK^{-T} D^{-1}
// (ld LDM, zero above the diagonal) into MK — register-resident, no LDS hand-off per step (the LDS
// hand-off variant took ~3.8 us per block against ~2.6 us for this one, r3).
// Lane (i = lane & 15, g = lane >> 4) holds A(i, j) and X(i, j) for the four columns j = 4m + g in
// a[m], x[m]: column t lives in register t >> 2 of row group t & 3.  Step t:
//   d_t = A(t, t): v_readlane (wave-uniform);
//   A(i, t) to every row group: v_permlane16_swap + v_permlane32_swap (gfx950) of row group t & 3;
//   A(t, j), X(t, j) of the lane's columns: DPP row_newbcast:t inside the lane's 16-lane row.
// Every row i > t is updated with the mirrored row t (A(t, j), j > t).
template <int T>
__device__ __forceinline__ double dpp_row_bcast(double v) {  // lane T of every 16-lane row, to the row
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, 0x150 + T, 0xf, 0xf, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, 0x150 + T, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
template <int G>
__device__ __forceinline__ int xrow_bcast32(int v) {  // row G (16 lanes) of the wave, to every row
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // [r0 r0 r2 r2] | [r1 r1 r3 r3]
  const int y = (G & 1) ? (int)p[1] : (int)p[0];
  const auto q = __builtin_amdgcn_permlane32_swap(y, y, false, false);  // [rA rA rA rA] | [rB rB rB rB]
  return (G & 2) ? (int)q[1] : (int)q[0];
}
template <int G>
__device__ __forceinline__ double xrow_bcast(double v) {
  return __hiloint2double(xrow_bcast32<G>(__double2hiint(v)), xrow_bcast32<G>(__double2loint(v)));
}
// acc += acc[lane T of the lane's 16-lane row] * mul: ONE v_fmac_f64 with a DPP row_newbcast source
// (64-bit DPP, gfx90a+).  The s_nop covers the VALU-write -> DPP-read hazard (2 wait states) that the
// compiler does not track through inline asm.
template <int T>
__device__ __forceinline__ void fmac_row_bcast(double& acc, double mul) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(mul), "n"(T));
}
// RCP: l = A(i, t) * (1 / d_t) with the reciprocal from v_rcp_f64 + two Newton steps
// (within an ulp of the IEEE quotient; ~6 dependent instructions on the pivot chain instead of the
// ~10 of the IEEE division sequence)
__device__ __forceinline__ double recip_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  return fma(fma(-d, r, 1.0), r, r);
}
template <int T, bool RCP>
__device__ __forceinline__ void f16r_step(double (&a)[4], double (&x)[4], double& dmine, int i, int g) {
  constexpr int gt = T & 3, mt = T >> 2;
  const double dt = readlane_f64(a[mt], T + 16 * gt);
  const double ci = xrow_bcast<gt>(a[mt]);
  const double li = (i > T) ? (RCP ? ci * recip_nr(dt) : ci / dt) : 0.0;  // IEEE quotient unless RCP
  // A(i, j) -= l_i A(t, j) for j > t; X(i, j) -= l_i X(t, j) for j <= t (a zero multiplier elsewhere:
  // exact, the products are finite); the column ranges are static except for one register.  The
  // register holding the next pivot column goes first and the X updates (off the pivot chain) last:
  // the waves issue in order, so the next step's readlane then finds its operand ready (the same
  // operations as before, in another order: bitwise the same factor)
  constexpr int mn = (T + 1 < 16) ? ((T + 1) >> 2) : -1;
  if constexpr (mn >= 0) fmac_row_bcast<T>(a[mn], (4 * mn + g > T) ? -li : 0.0);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = 4 * m + g;
    if (m != mn && 4 * m + 3 > T) fmac_row_bcast<T>(a[m], (j > T) ? -li : 0.0);
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = 4 * m + g;
    if (4 * m <= T) fmac_row_bcast<T>(x[m], (j <= T) ? -li : 0.0);
  }
  if (i == T) dmine = dt;
  if (g == gt && i > T) a[mt] = li;
}
template <int T, bool RCP>
__device__ __forceinline__ void f16r_steps(double (&a)[4], double (&x)[4], double& dmine, int i, int g) {
  if constexpr (T < 16) {
    f16r_step<T, RCP>(a, x, dmine, i, g);
    f16r_steps<T + 1, RCP>(a, x, dmine, i, g);
  }
}
template <bool PK, bool RCP>
__device__ __forceinline__ void factor16r(double* A, int r, int ld, int k0, int kw, double* Dl, double* MK, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int ic = min(i, kw - 1);
  double a[4], x[4], v[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = 4 * m + g, jc = min(j, kw - 1);
    v[m] = A[fidx<PK>(k0 + max(ic, jc), k0 + min(ic, jc), r, ld)];  // mirrored: the full symmetric block
  }
  LDL_PIN4(v);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = 4 * m + g;
    a[m] = (i < kw && j < kw) ? v[m] : (i == j ? 1.0 : 0.0);
    x[m] = (i == j) ? 1.0 : 0.0;
  }
  double dmine = 1.0;
  f16r_steps<0, RCP>(a, x, dmine, i, g);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = 4 * m + g;
    if (j < i && i < kw) A[fidx<PK>(k0 + i, k0 + j, r, ld)] = a[m];
    MK[j * LDM + i] = (j <= i) ? x[m] / dmine : 0.0;
  }
  if (g == 0 && i < kw) Dl[k0 + i] = dmine;
  wave_sync();
}

// In-launch hand-offs between workgroups (MI355X_MICROARCH.md "inter-workgroup visibility", form R1):
// payload stored sc1 and drained before ONE lane stores the flag; consumers poll relaxed and load sc1.
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool poll_flag(int32_t* f, int epoch, int32_t* err) {
  int spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 25)) {
      atomicOr(err, kErrHandoff);
      return false;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only (sc1 loads follow)
  return true;
}
// wave 0: poll the flags of dep[q0 .. q1) together (one lane per dependency, 64 per pass)
__device__ __forceinline__ void poll_deps(const int32_t* __restrict__ dep, int q0, int q1, int32_t* flags, int epoch,
                                          int32_t* err) {
  const int lane = threadIdx.x & 63;
  for (int q = q0; q < q1; q += 64) {
    const int32_t* f = (q + lane < q1) ? flags + dep[q + lane] : nullptr;
    int spins = 0;
    for (;;) {
      const bool ok = !f || __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 25)) {
        if (lane == 0) atomicOr(err, kErrHandoff);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void publish_sc1(int32_t* f, int epoch) {  // the storing wave, after its sc1 stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Blocked right-looking LDL^T of the w pivots of a front held in LDS (lower part; square ld r|1 or
// packed), all 256 threads; pivots in Dl.
//
// Codegen notes (measured on gfx950 with tools/factor_bench.hip, tools/tile_bench.hip): one f64
// MFMA 16x16x4 issues every 64 cycles per SIMD, an LDS round trip is ~80 cycles, and a wave has
// nothing to hide them behind (one 256-thread workgroup per CU).  So every LDS operand of a step is
// loaded unconditionally (clamped indices, pinned so the compiler cannot sink a load into a branch
// with its own wait), a wave updates a STRIP of up to four 16 x 16 tiles sharing the (L_I D)
// operand (four independent accumulator chains back to back), and the next pivot block is
// factorised by one wave while the other three finish the trailing update (lookahead).

// L_R = A[R, k0:k0+kw] M_K for the 16-row blocks b = b0, b0 + bstep, ... below the pivots
template <bool PK>
__device__ __forceinline__ void panel_blocks(double* A, int r, int ld, int k0, int kw, int R0, int nbr, const double* MK,
                                             int b0, int bstep, int lane) {
  const int kl = lane >> 4, il = lane & 15;
  double bv[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) bv[ks] = MK[(4 * ks + kl) * LDM + il];
  for (int b = b0; b < nbr; b += 2 * bstep) {
    const bool two = b + bstep < nbr;  // wave-uniform
    double av[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int row = min(R0 + 16 * (b + u * bstep) + il, r - 1);
        av[u][ks] = A[fidx<PK>(row, k0 + min(4 * ks + kl, kw - 1), r, ld)];
      }
    LDL_PIN4(av[0]);
    LDL_PIN4(av[1]);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) av[u][ks] = (4 * ks + kl < kw) ? av[u][ks] : 0.0;
    dbl4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0][ks], bv[ks], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1][ks], bv[ks], acc1, 0, 0, 0);  // unpredicated
    }
    // acc[g] = D[m][n]: m = kl + 4 g (row in the block: the A operand carried the rows), n = il (pivot)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row0 = R0 + 16 * b + kl + 4 * g, row1 = row0 + 16 * bstep;
      if (row0 < r && il < kw) A[fidx<PK>(row0, k0 + il, r, ld)] = acc0[g];
      if (two && row1 < r && il < kw) A[fidx<PK>(row1, k0 + il, r, ld)] = acc1[g];
    }
  }
}

// One strip: tiles (I, J0 .. J0+NS-1).  NS is static so the MFMA sequence has no branches (a
// predicated MFMA makes the compiler drain the accumulators after every step).
template <bool PK, int NS>
__device__ __forceinline__ void trail_strip(double* A, int r, int ld, int k0, int kw, int R0, int I, int J0,
                                            const double (&dk)[4], int lane, int jend) {
  const int kl = lane >> 4, il = lane & 15;
  const int i0 = R0 + 16 * I;
  const int ri = min(i0 + il, r - 1);
  double bv[4], av[NS][4], cv[NS][4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int kc = k0 + min(4 * ks + kl, kw - 1);
    bv[ks] = A[fidx<PK>(ri, kc, r, ld)];
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int rj = min(R0 + 16 * (J0 + t) + il, r - 1);
      av[t][ks] = A[fidx<PK>(rj, kc, r, ld)];
    }
  }
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = min(R0 + 16 * (J0 + t) + kl + 4 * g, r - 1);
      cv[t][g] = A[fidx<PK>(max(ri, j), min(ri, j), r, ld)];
    }
  // pins in issue order, after every load (the MFMA operands first: their waits come first)
  LDL_PIN4(bv);
#pragma unroll
  for (int t = 0; t < NS; ++t) LDL_PIN4(av[t]);
#pragma unroll
  for (int t = 0; t < NS; ++t) LDL_PIN4(cv[t]);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) bv[ks] *= dk[ks];  // dk = 0 past kw
  dbl4 acc[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int t = 0; t < NS; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t][ks], bv[ks], acc[t], 0, 0, 0);
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = R0 + 16 * (J0 + t) + kl + 4 * g, i = i0 + il;
      if (i < r && j < jend && i >= j) A[fidx<PK>(i, j, r, ld)] = cv[t][g] - acc[t][g];
    }
}

// C_IJ -= L_J (L_I D)^T over the 16 x 16 tiles (I, J) of the trailing lower triangle with
// jlo <= J <= min(I, jhi), I < nbr; strips (I, J0 .. J0+3) dealt to waves w0, w0 + wstep, ...
template <bool PK>
__device__ __forceinline__ void trail_strips(double* A, int r, int ld, int k0, int kw, int R0, int nbr, int jlo, int jhi,
                                             const double (&dk)[4], int w0, int wstep, int lane, int jend, int i0 = 0) {
  if (jlo > jhi) return;
  int I = max(jlo, i0), J0 = jlo;  // rows I >= i0 only
  auto adv = [&]() {
    J0 += 4;
    if (J0 > min(I, jhi)) {
      ++I;
      J0 = jlo;
    }
  };
  for (int s = 0; s < w0; ++s) adv();
  while (I < nbr) {
    switch (min(4, min(I, jhi) - J0 + 1)) {  // tiles in this strip (wave-uniform)
      case 1: trail_strip<PK, 1>(A, r, ld, k0, kw, R0, I, J0, dk, lane, jend); break;
      case 2: trail_strip<PK, 2>(A, r, ld, k0, kw, R0, I, J0, dk, lane, jend); break;
      case 3: trail_strip<PK, 3>(A, r, ld, k0, kw, R0, I, J0, dk, lane, jend); break;
      default: trail_strip<PK, 4>(A, r, ld, k0, kw, R0, I, J0, dk, lane, jend); break;
    }
    for (int s = 0; s < wstep; ++s) adv();
  }
}

// Deferred Schur complement: U -= L_U D L_U^T over all w pivots in one pass (tiles of the lower
// triangle of A[w:, w:]).  K runs over the pivots in 16-column chunks with the accumulators held in
// registers, so each C tile is loaded and stored once (the per-block right-looking update touches it
// w/16 times); the next chunk's operands are loaded before the current chunk's MFMAs.
template <bool PK, int NS>
__device__ __forceinline__ void schur_strip(double* A, int r, int ld, int w, const double* Dl, int I, int J0, int lane) {
  const int kl = lane >> 4, il = lane & 15;
  const int i0 = w + 16 * I;
  const int ri = min(i0 + il, r - 1);
  int rj[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) rj[t] = min(w + 16 * (J0 + t) + il, r - 1);
  dbl4 acc[NS];
#pragma unroll
  for (int t = 0; t < NS; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  // raw operands of the next 16-pivot chunk: issued one chunk ahead, pinned (waited for) only at the
  // top of the iteration that consumes them, i.e. after the previous chunk's MFMAs
  double bn[4], an[NS][4];
  auto load = [&](int k0) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kc = min(k0 + 4 * ks + kl, w - 1);
      bn[ks] = A[fidx<PK>(ri, kc, r, ld)];
#pragma unroll
      for (int t = 0; t < NS; ++t) an[t][ks] = A[fidx<PK>(rj[t], kc, r, ld)];
    }
  };
  load(0);
  for (int k0 = 0; k0 < w; k0 += 16) {
    LDL_PIN4(bn);
#pragma unroll
    for (int t = 0; t < NS; ++t) LDL_PIN4(an[t]);
    double b2[4], a2[NS][4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = k0 + 4 * ks + kl;
      b2[ks] = (k < w) ? bn[ks] * Dl[min(k, w - 1)] : 0.0;  // pivots: LDS, read at the point of use
#pragma unroll
      for (int t = 0; t < NS; ++t) a2[t][ks] = an[t][ks];
    }
    if (k0 + 16 < w) load(k0 + 16);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int t = 0; t < NS; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[t][ks], b2[ks], acc[t], 0, 0, 0);
  }
  double cv[NS][4];
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = min(w + 16 * (J0 + t) + kl + 4 * g, r - 1);
      cv[t][g] = A[fidx<PK>(max(ri, j), min(ri, j), r, ld)];
    }
#pragma unroll
  for (int t = 0; t < NS; ++t) LDL_PIN4(cv[t]);
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = w + 16 * (J0 + t) + kl + 4 * g, i = i0 + il;
      if (i < r && j < r && i >= j) A[fidx<PK>(i, j, r, ld)] = cv[t][g] - acc[t][g];
    }
}

template <bool PK>
__device__ __forceinline__ void schur_strips(double* A, int r, int ld, int w, const double* Dl, int wv, int nw, int lane) {
  const int nbu = (r - w + 15) >> 4;
  int I = 0, J0 = 0;
  auto adv = [&]() {
    J0 += 4;
    if (J0 > I) {
      ++I;
      J0 = 0;
    }
  };
  for (int q = 0; q < wv; ++q) adv();
  while (I < nbu) {
    switch (min(4, I - J0 + 1)) {
      case 1: schur_strip<PK, 1>(A, r, ld, w, Dl, I, J0, lane); break;
      case 2: schur_strip<PK, 2>(A, r, ld, w, Dl, I, J0, lane); break;
      case 3: schur_strip<PK, 3>(A, r, ld, w, Dl, I, J0, lane); break;
      default: schur_strip<PK, 4>(A, r, ld, w, Dl, I, J0, lane); break;
    }
    for (int q = 0; q < nw; ++q) adv();
  }
}

// defer: the right-looking block steps update only the pivot columns (columns < w); the update
// block U gets its whole Schur complement afterwards in one pass (schur_strips)
// pt (diagnostics, MADIPM_TREE_DEBUG): thread 0 accumulates the phase times (first pivot block,
// panels, J = 0 strips, lookahead sections, Schur pass) into pt[0..4]
template <bool PK>
__device__ __forceinline__ void blocked_factor_lds(double* A, int r, int w, int ld, double* Dl, double* MK, double* cbuf,
                                                   int defer = 0, int64_t* pt = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  const int nblk = (w + 15) >> 4;
  defer = defer && w < r;
  const int jend = defer ? w : r;
  int64_t tp[5] = {0, 0, 0, 0, 0}, tl = (pt && tid == 0) ? wall_clock64() : 0;
  auto stamp = [&](int k) {
    if (pt && tid == 0) {
      const int64_t now = wall_clock64();
      tp[k] += now - tl;
      tl = now;
    }
  };
  const int64_t cyc0 = (pt && tid == 0) ? (int64_t)clock64() : 0;
  if (wv == 0) factor16r<PK, true>(A, r, ld, 0, min(16, w), Dl, MK, lane);
  __syncthreads();
  stamp(0);
  const int64_t cyc1 = (pt && tid == 0) ? (int64_t)clock64() : 0;
  for (int kb = 0; kb < nblk; ++kb) {
    const int k0 = 16 * kb, kw = min(16, w - k0);
    const int R0 = k0 + kw;                       // first row / column after the pivots
    const int nbr = (r - R0 + 15) >> 4;           // 16-row blocks below
    const int jhi = defer ? ((w - R0 + 15) >> 4) - 1 : nbr;  // last column block updated
    panel_blocks<PK>(A, r, ld, k0, kw, R0, nbr, MK, wv, nw, lane);
    __syncthreads();
    stamp(1);
    double dk[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = 4 * ks + (lane >> 4);
      dk[ks] = (k < kw) ? Dl[k0 + min(k, kw - 1)] : 0.0;
    }
    if (kb + 1 < nblk) {
      // the next pivot block's columns (J = 0: its diagonal block and panel rows) first ...
      trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 0, 0, dk, wv, nw, lane, jend);
      __syncthreads();
      stamp(2);
      // ... then one wave factorises it while the others update the rest (J >= 1)
      const int fw = (kb + 1) % nw;
      if (wv == fw)
        factor16r<PK, true>(A, r, ld, R0, min(16, w - R0), Dl, MK, lane);
      else
        trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 1, jhi, dk, (wv - fw + nw - 1) % nw, nw - 1, lane, jend);
    } else if (!defer) {
      trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 0, nbr, dk, wv, nw, lane, jend);
    }
    __syncthreads();
    stamp(3);
  }
  if (defer) {
    schur_strips<PK>(A, r, ld, w, Dl, wv, nw, lane);
    __syncthreads();
    stamp(4);
  }
  if (pt && tid == 0) {
    for (int k = 0; k < 5; ++k) pt[k] = tp[k];
    pt[5] = cyc1 - cyc0;  // shader clocks of the first pivot block (vs pt[0] in 100 MHz ticks)
  }
}

// ---- Pipelined schedule of the same factorisation (MADIPM_FACT_PIPE=1, default; needs factor16r).
// In blocked_factor_lds every pivot block costs panel + column-0 strips + max(next diagonal factor,
// trailing update), three workgroup barriers apart, and the diagonal factor (~2.6 us of division and
// lane-swap latency) dominates.  Here wave 0 runs the pivot chain alone: once block k is factorised it
// forms the panel tile of row block 0 below it (the next pivot rows), updates the next diagonal tile
// with it and factorises that tile at once — while waves 1.. form the rest of block k's panel and its
// trailing update.  Hand-offs are LDS counters (workgroup-scope release / acquire), not barriers, so
// the chain never waits for the trailing update of its own step:
//   mk     = k + 1  wave 0: block k's M_K (buffer k & 1), pivots and L_kk are in LDS
//   pt     = k + 1  wave 0: panel tile 0 of step k is in LDS
//   j0    += 1      each other wave, after its priority tiles of step k: column block 0 (tiles (I, 0),
//                   I >= 1) and the diagonal tile (1, 1) — everything wave 0 reads at step k + 1
//   ob    += 1      barrier among the other waves (panel rows complete before the trailing update)
// Tile (0, 0) of a non-final step is wave 0's alone.  Every tile and panel block is formed by the
// same MFMA sequence from the same operands as in blocked_factor_lds: the two schedules agree
// bitwise (test_ldl_fact_pipe_bitwise).  A wait that spins for ~2^20 polls sets `abort` (a schedule
// bug must not hang the GPU: the factor is then garbage and the tests fail).
struct PipeCtr {
  int mk, pt, j0, ob, abort;
  int64_t ow;  // diagnostics: wave 1's wait ticks
};
__device__ __forceinline__ PipeCtr& pipe_ctr() {
  __shared__ PipeCtr c;
  return c;
}
__device__ __forceinline__ void pipe_wait(int* f, int v, int* abort) {
  int spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) {
    if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 20)) {
      __hip_atomic_store(abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return;
    }
  }
}
// one lane per wave, after the wave's LDS writes (the release orders them before the counter)
__device__ __forceinline__ void pipe_set(int* f, int v) {
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void pipe_add(int* f) {
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool PK>
__device__ __forceinline__ void blocked_factor_pipe(double* A, int r, int w, int ld, double* Dl, double* MK0,
                                                    double* MK1, int defer, int64_t* pt, int32_t* err, int fault) {
  constexpr bool RCP = true;
  double* const MKall = nullptr;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  const int no = nw - 1;  // waves 1 .. nw - 1: panel rest + trailing update
  const int nblk = (w + 15) >> 4;
  // defer 2: the caller forms the update block's Schur complement itself (the medium fronts' panels,
  // whose trailing matrix lives in HBM): rows below the pivots get their L only
  const bool schur = defer == 1;
  defer = defer && w < r;
  const int jend = defer ? w : r;
  PipeCtr& pc = pipe_ctr();
  int64_t t0 = (pt && tid == 0) ? wall_clock64() : 0;
  if (tid == 0) pc = PipeCtr{0, 0, 0, 0, 0, 0};
  // diagnostics (pt): wave 0's wait / diagonal-factor ticks, wave 1's wait ticks
  const bool dbg = pt && (tid == 0 || tid == 64);
  int64_t tw = 0, tf = 0, tc = 0;
  auto lap = [&](int64_t& acc) {
    if (dbg) {
      const int64_t now = wall_clock64();
      acc += now - tc;
      tc = now;
    }
  };
  if (wv == 0) factor16r<PK, RCP>(A, r, ld, 0, min(16, w), Dl, MKall ? MKall : MK0, lane);
  __syncthreads();  // block 0 factorised; the counters are zero
  const int64_t t1 = (pt && tid == 0) ? wall_clock64() : 0;
  int gen = 0;  // O-barrier generation (waves 1..)
  for (int kb = 0; kb < nblk; ++kb) {
    const int k0 = 16 * kb, kw = min(16, w - k0);
    const int R0 = k0 + kw;
    const int nbr = (r - R0 + 15) >> 4;
    const int jhi = defer ? ((w - R0 + 15) >> 4) - 1 : nbr;
    const bool last = kb + 1 == nblk;
    const double* MKc = MKall ? MKall + kb * 16 * LDM : ((kb & 1) ? MK1 : MK0);
    double dk[4];
    int64_t tx = 0;
    if (dbg) tc = wall_clock64();
    if (wv == 0) {
      // the pivot chain: step kb - 1's priority tiles (this step's raw panel tile 0 and diagonal tile)
      if (kb > 0) pipe_wait(&pc.j0, no * kb, &pc.abort);
      lap(tw);
      if (nbr > 0) panel_blocks<PK>(A, r, ld, k0, kw, R0, 1, MKc, 0, 1, lane);
      pipe_set(&pc.pt, kb + 1);
      if (!last) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int k = 4 * ks + (lane >> 4);
          dk[ks] = (k < kw) ? Dl[k0 + min(k, kw - 1)] : 0.0;
        }
        trail_strip<PK, 1>(A, r, ld, k0, kw, R0, 0, 0, dk, lane, jend);  // the next diagonal tile
        wave_sync();
        lap(tx);
        factor16r<PK, RCP>(A, r, ld, R0, min(16, w - R0), Dl,
                           MKall ? MKall + (kb + 1) * 16 * LDM : ((kb & 1) ? MK0 : MK1), lane);
        if (!fault) pipe_set(&pc.mk, kb + 2);  // fault: MADIPM_DEBUG_PIPE_FAULT (tests only): never published
        lap(tf);
      }
    } else {
      const int ow = wv - 1;
      if (kb > 0) {
        pipe_wait(&pc.mk, kb + 1, &pc.abort);      // block kb's M_K and pivots
        pipe_wait(&pc.j0, no * kb, &pc.abort);     // every other wave's column-0 tiles of step kb - 1 (raw panel rows)
      }
      lap(tw);
      panel_blocks<PK>(A, r, ld, k0, kw, R0, nbr, MKc, 1 + ow, no, lane);  // rows 1 .. nbr - 1
      ++gen;
      lap(tx);
      pipe_add(&pc.ob);
      pipe_wait(&pc.ob, no * gen, &pc.abort);
      pipe_wait(&pc.pt, kb + 1, &pc.abort);
      lap(tw);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + (lane >> 4);
        dk[ks] = (k < kw) ? Dl[k0 + min(k, kw - 1)] : 0.0;
      }
      if (!last) {
        // priority: strip (1, 0..1) (tile (1, 1) only inside the update range), then (I, 0) for I >= 2
        const bool d11 = nbr > 1 && jhi >= 1;
        for (int it = ow; it < nbr - 1; it += no) {
          if (it == 0) {
            if (d11)
              trail_strip<PK, 2>(A, r, ld, k0, kw, R0, 1, 0, dk, lane, jend);
            else
              trail_strip<PK, 1>(A, r, ld, k0, kw, R0, 1, 0, dk, lane, jend);
          } else {
            trail_strip<PK, 1>(A, r, ld, k0, kw, R0, it + 1, 0, dk, lane, jend);
          }
        }
        pipe_add(&pc.j0);
        // the rest: rows I >= 2, column blocks 1 .. jhi
        trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 1, jhi, dk, ow, no, lane, jend, 2);
      } else if (!defer) {
        trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 0, nbr, dk, ow, no, lane, jend);
      }
    }
  }
  if (dbg && tid == 64) pc.ow = tw;
  __syncthreads();
  // a lost hand-off (a wait that timed out) leaves a wrong factor: raise the sticky status error that
  // status() turns into a failure (the flag polls between fronts do the same)
  if (tid == 0 && __hip_atomic_load(&pc.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) && err)
    __hip_atomic_fetch_or(err, kErrHandoff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t t2 = (pt && tid == 0) ? wall_clock64() : 0;
  if (defer && schur) {
    schur_strips<PK>(A, r, ld, w, Dl, wv, nw, lane);
    __syncthreads();
  }
  if (pt && tid == 0) {
    pt[0] = t1 - t0;
    pt[1] = t2 - t1;  // the pipelined block steps
    pt[2] = tw;       // wave 0 waiting for the other waves' priority tiles
    pt[3] = tf;       // wave 0 in factor16r
    pt[4] = wall_clock64() - t2;
    pt[5] = pc.ow;    // wave 1 waiting (M_K, barrier, panel tile 0, column-0 tiles)
  }
}

template <bool PK>
__device__ __forceinline__ void factor_lds(const FrontTab& T, double* A, int r, int w, int ld, double* Dl, double* MK,
                                           double* cbuf, int64_t* pt = nullptr) {
  if (T.fpipe && (blockDim.x >> 6) >= 2)
    blocked_factor_pipe<PK>(A, r, w, ld, Dl, MK, cbuf, 1, pt, T.err, T.pipe_fault);
  else
    blocked_factor_lds<PK>(A, r, w, ld, Dl, MK, cbuf, 1, pt);
}


// write-out: L panel (ld r; d on the diagonal, zeros above), lower triangle of U (ld uld), D and the
// pivot check.  SC1: U stored write-through (handed to a parent inside the same launch).
template <bool PK, bool SC1>
__device__ __forceinline__ void writeout_u(const double* A, int r, int w, int ld, double* Uo, int uld);
// offset of column b of a u x u update block: square ld uld, or packed lower (uld == 0: column b
// holds rows b .. u - 1, entry (a, b) at b (2u - b - 1) / 2 + a)
__device__ __forceinline__ int64_t ucol_off(int b, int u, int64_t uld) {
  return uld ? (int64_t)b * uld : ((int64_t)b * (2 * u - b - 1)) >> 1;
}
template <bool PK>
__device__ __forceinline__ void writeout_ld(const double* A, int r, int w, int ld, const double* Dl, double* L, double* D,
                                           int f0, LDLStatus* st, double tol) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  // L panel (ld r; d on the diagonal, zeros above): columns dealt to waves as in writeout_u
  for (int j0 = 4 * wv; j0 < w; j0 += 4 * nw) {
    double x[4][3], dd[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int j = min(j0 + cb, w - 1);
      const int base = PK ? ((j * (2 * r - j - 1)) >> 1) : j * ld;
      dd[cb] = Dl[j];
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int i = lane + 64 * h, ic = min(max(i, j), r - 1);
        x[cb][h] = A[base + ic];
      }
    }
    LDL_PIN4(dd);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      asm volatile("" : "+v"(x[cb][0]), "+v"(x[cb][1]), "+v"(x[cb][2]));
      const int j = min(j0 + cb, w - 1);
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int i = lane + 64 * h;
        x[cb][h] = (i > j) ? x[cb][h] : (i == j ? dd[cb] : 0.0);
      }
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int j = j0 + cb;
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int i = lane + 64 * h;
        if (j < w && i < r) L[i + (int64_t)j * r] = x[cb][h];
      }
    }
  }
  if (tid < w) {
    const double d = Dl[tid];
    D[f0 + tid] = d;
    if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + tid + 1);
  }
}
template <bool PK, bool SC1>
__device__ __forceinline__ void blocked_writeout(const double* A, int r, int w, int ld, const double* Dl, double* L,
                                                 double* Uo, int uld, double* D, int f0, LDLStatus* st, double tol) {
  writeout_ld<PK>(A, r, w, ld, Dl, L, D, f0, st, tol);
  writeout_u<PK, SC1>(A, r, w, ld, Uo, uld);
}
// lower triangle of the update block U (ld uld); SC1: stored write-through (handed to a parent
// inside the same launch)
// columns dealt to waves, NC per wave and round, NH 64-row chunks per column; a column's rows run
// over the lanes, so the LDS and global addresses are a wave-uniform column base + the row (no
// per-element index arithmetic: with one wave per SIMD that arithmetic bounded this loop)
template <bool PK, bool SC1, int NH, int NC>
__device__ __forceinline__ void writeout_u_cols(const double* A, int r, int w, int ld, double* Uo, int uld) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  const int u = r - w;
  for (int b0 = NC * wv; b0 < u; b0 += nw * NC) {
    double x[NC][NH];
#pragma unroll
    for (int cb = 0; cb < NC; ++cb) {
      const int b = min(b0 + cb, u - 1), j = w + b;
      const int base = PK ? ((j * (2 * r - j - 1)) >> 1) : j * ld;  // fidx(i, j) = base + i
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int a = min(b + lane + 64 * h, u - 1);
        x[cb][h] = A[base + w + a];
      }
    }
#pragma unroll
    for (int cb = 0; cb < NC; ++cb)
#pragma unroll
      for (int h = 0; h < NH; ++h) LDL_PIN(x[cb][h]);
#pragma unroll
    for (int cb = 0; cb < NC; ++cb) {
      const int b = b0 + cb;
      double* col = Uo + ucol_off(b, u, uld);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int a = b + lane + 64 * h;
        if (b < u && a < u) {
          if (SC1)
            __hip_atomic_store(col + a, x[cb][h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            col[a] = x[cb][h];
        }
      }
    }
  }
}
template <bool PK, bool SC1>
__device__ __forceinline__ void writeout_u(const double* A, int r, int w, int ld, double* Uo, int uld) {
  const int u = r - w;
  if (u <= 64)
    writeout_u_cols<PK, SC1, 1, 8>(A, r, w, ld, Uo, uld);
  else if (u <= 128)
    writeout_u_cols<PK, SC1, 2, 6>(A, r, w, ld, Uo, uld);
  else
    writeout_u_cols<PK, SC1, 3, 4>(A, r, w, ld, Uo, uld);
}

// lower part of an r x r front assembled in HBM scratch (ld r) -> LDS, 16 loads in flight per thread
template <bool PK, int NTH = NT>
__device__ __forceinline__ void stage_front(const double* __restrict__ Fs, double* A, int r, int ld) {
  const int tid = threadIdx.x;
  const int nel = r * r;
  ColWalk wk(tid, r, NTH);
  for (int base = 0; base < nel; base += NTH * 16) {
    double v[16];
    int dst[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = base + k * NTH + tid;
      const bool ok = q < nel && wk.i >= wk.j;
      v[k] = ok ? Fs[q] : 0.0;
      dst[k] = ok ? fidx<PK>(wk.i, wk.j, r, ld) : -1;
      wk.next();
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (dst[k] >= 0) A[dst[k]] = v[k];
  }
}

// k_small_blocked: 8 waves (2 per SIMD): twice the loads in flight of the staging copy and write-out,
// and 7 waves beside the pivot chain of the pipelined factorisation (the 120-column ex10 root)
constexpr int SBT = 512;
template <bool PK>
__global__ __launch_bounds__(SBT) void k_small_blocked(FrontTab T, const int32_t* __restrict__ fronts,
                                                      const double* __restrict__ Kx, double* __restrict__ arena,
                                                      const double* __restrict__ fscratch, double* __restrict__ D,
                                                      LDLStatus* st, double tol, LDLStatus* stamp, int32_t* go,
                                                      int go_epoch) {
  extern __shared__ __attribute__((aligned(16))) double A[];  // lower part of F (square ld r|1, or packed)
  __shared__ double Dl[192];
  __shared__ double MK[16 * LDM];
  __shared__ __attribute__((aligned(16))) double cbuf[2 * 16 * LDM];
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int ld = r | 1;
  const int tid = threadIdx.x;
  // the root tail (LDLSolver::root_async_): launched on the side stream ahead of time, it waits for
  // the root assembly's go[0] (k_assemble's last tile, main stream), then acquires its stores.  The
  // pivot chain runs beside the solve's kernels on this CU: its waves issue first
  if (go) {
    __builtin_amdgcn_s_setprio(3);
    if (tid < 64) poll_flag(go, go_epoch, T.err);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  const int64_t fso = T.fs_off[s];
  if (fso >= 0 && !T.fs_img[s]) {  // batched-leaf parent: the SYRK and k_assemble wrote ld r
    stage_front<PK, SBT>(fscratch + fso, A, r, ld);
  } else if (fso >= 0) {  // assembled by k_assemble as the LDS image (lower part valid): a straight copy
    const double* __restrict__ src = fscratch + fso;
    const int n = PK ? r * (r + 1) / 2 : r * ld;
    for (int base = 0; base < n; base += SBT * 16) {
      double v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int q = base + k * SBT + tid;
        v[k] = (q < n) ? src[q] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int q = base + k * SBT + tid;
        if (q < n) A[q] = v[k];
      }
    }
  } else {  // leaf: original entries only
    const int ntot = PK ? r * (r + 1) / 2 : r * ld;
    for (int q = tid; q < ntot; q += SBT) A[q] = 0.0;
    __syncthreads();
    for (int64_t q = T.asm_ptr[s] + tid; q < T.asm_ptr[s + 1]; q += SBT) {
      const int d = (int)T.asm_dst[q], dj = d / r;  // d < r^2: 32-bit division
      A[fidx<PK>(d - dj * r, dj, r, ld)] = Kx[T.asm_src[q]];
    }
  }
  __syncthreads();
  factor_lds<PK>(T, A, r, w, ld, Dl, MK, cbuf);
  blocked_writeout<PK, false>(A, r, w, ld, Dl, arena + T.l_off[s], arena + T.u_off[s], T.u_ld[s], D, f0, st, tol);
  if (go) {  // released to k_root_solve (go[2 + front]: the epoch); nothing of this kernel follows
    __threadfence();
    __syncthreads();
  }
  if (tid == 0) {
    // lazy inertia: the factorisation's end
    if (stamp) atomicMax(reinterpret_cast<unsigned long long*>(&stamp->t1), (unsigned long long)wall_clock64());
    if (go) __hip_atomic_store(go + 2 + blockIdx.x, go_epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------ leaf folding
// A tree front folds its micro-leaf children (w <= 2, r <= 32; SymbolicPlan::absorb) into its LDS
// front instead of k_micro_factor writing their update blocks to HBM and the gather pre-assembly
// summing them.  Per batch of leaves: (1) thread per leaf row gathers the row's entries of the leaf's
// two columns from the caller's K values; (2) thread per leaf row: the leaf's pivots d0, l10, d1 (from
// its first two rows) and the row's l (and l d) in LDS; (3) the product list: thread t walks its chunk of destination-sorted products
// F(i, j) -= l0(q1) l0(q2) d0 + l1(q1) l1(q2) d1, one partial sum per destination run, so every
// entry of F has one writer and a fixed order (leaf order) — no atomics, balanced by product count
// whatever the row density.
// Latency: every phase is one or two global round trips at most (8 leaf rows per thread in flight;
// product entries 16 per thread in flight, the next group's loads issued before the current group's
// arithmetic, the first group before phase 1).
// k_fact_tree's workgroup: 8 waves (2 per SIMD) — every memory phase of a tree front (the leaf fold,
// the staging copy, the children's pushes, the write-out) is latency-bound, and a second wave per SIMD
// doubles the loads in flight; the in-LDS factorisation deals its tiles over the 8 waves
constexpr int FTN = SymbolicPlan::kFoldThreads;
static_assert(FTN == 512, "k_fact_tree: 512 threads");

// one copy for both storage variants (a static __shared__ inside the template would be allocated twice)
struct FoldBatchTab {
  int64_t j[SymbolicPlan::kFoldMaxBatches + 1], po[SymbolicPlan::kFoldMaxBatches];
  int32_t k[SymbolicPlan::kFoldMaxBatches + 1], pl[SymbolicPlan::kFoldMaxBatches];
};
__device__ __forceinline__ FoldBatchTab& fold_batch_tab() {
  __shared__ FoldBatchTab t;
  return t;
}

#ifndef MADIPM_FOLD_GP
#define MADIPM_FOLD_GP 16  // fold product entries per thread and group (32 spills; variants: tools/build_variant.sh)
#endif
// cval / cdst: per thread, the parked sum and destination of a chunk's first run when it continues
// the left neighbour's run (k_fact_tree's MK / cbuf, idle during the fold)
template <bool PK>
__device__ __forceinline__ void fold_leaves(const FrontTab& T, int s, int r, int ld, double* A, const double* Kx, double* arena,
                                            double* D, LDLStatus* st, double tol, double* ext, double* cval,
                                            int32_t* cdst, int64_t* fdg, const FoldStart& F0, bool with_asm) {
  int64_t tph[4] = {0, 0, 0, 0}, tc = fdg ? wall_clock64() : 0;
  auto lap = [&](int k) {
    if (fdg) {
      const int64_t t2 = wall_clock64();
      tph[k] += t2 - tc;
      tc = t2;
    }
  };
  constexpr int RPT = 8;   // leaf rows per thread and pass
  constexpr int GP = MADIPM_FOLD_GP;  // product entries per thread and group
  const int RM = T.fold_rmax[s], LM = T.fold_lmax[s];
  double2* LQ = reinterpret_cast<double2*>(ext);  // per batch row: K values of columns 0/1, then (l0, l1)
  double2* PQ = LQ + RM;                          // (l0 d0, l1 d1)
  int32_t* pf0 = reinterpret_cast<int32_t*>(PQ + RM);     // per leaf: first pivot (in 3 LM doubles of carve)
  int64_t* ploff = reinterpret_cast<int64_t*>(reinterpret_cast<double*>(pf0) + 3 * LM);
  int32_t* prow0 = reinterpret_cast<int32_t*>(ploff + LM);  // batch-local first row of the leaf
  int32_t* pwrc = prow0 + LM;
  int32_t* kk = pwrc + LM;                                   // per batch row: batch-local leaf
  const int tid = threadIdx.x;
  const int b0 = F0.b0, nb = F0.b1 - F0.b0;  // the front's batches (a helper: its share)
  if (nb > SymbolicPlan::kFoldMaxBatches) {  // the batch table below has room for kFoldMaxBatches
    if (tid == 0) __hip_atomic_fetch_or(T.err, kErrLdsCarve, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // the batch table (first leaf, first row, product offset and length), loaded once into LDS: read
  // from global per batch it cost two dependent round trips at each batch's gather and products
  FoldBatchTab& ft = fold_batch_tab();
  int32_t *tb_k = ft.k, *tb_pl = ft.pl;
  int64_t *tb_j = ft.j, *tb_po = ft.po;
  int32_t rk = 0, rpl = 0;
  int64_t rj = 0, rpo = 0;
  if (tid <= nb) {
    const int bq = b0 + tid, bc = min(bq, b0 + nb - 1);  // the sentinel entry (tid == nb) is the next batch's start
    rk = T.fold_bat[bq];
    rpl = T.fold_plen[bc];
    rj = T.fold_row0[bq];
    rpo = T.fold_poff[bc];
  }
  // product entries (SymbolicPlan::fold_prod): thread t walks chunk t, GP entries per group
  constexpr uint32_t PAD = SymbolicPlan::kFoldPad;
  uint32_t e[GP];
  auto load_group = [&](uint32_t (&g)[GP], const uint32_t* P, int k, int len) {
#pragma unroll
    for (int u = 0; u < GP; ++u) {
      const int kk = k + u;  // uniform: a scalar branch, not a per-lane wait
      g[u] = (kk < len) ? P[(int64_t)kk * FTN] : PAD;
    }
  };
  // the leaf rows' K entries of batch b + 1 are loaded into registers during batch b (indices before
  // its pivots, values before its products) and stored after its products: only batch 0's gather is
  // exposed (r3: every batch's gather, two dependent round trips, lay on the front's critical path).
  // A batch of more than RPT x FTN rows gathers its remaining passes in place.
  int32_t sa[RPT], sb[RPT];
  double va[RPT], vb[RPT];
  auto gather_idx = [&](int64_t j0, int nrow, int q0) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int q = q0 + u * FTN + tid;
      sa[u] = (q < nrow) ? T.ab_src0[j0 + q] : -1;
      sb[u] = (q < nrow) ? T.ab_src1[j0 + q] : -1;
    }
  };
  auto gather_val = [&]() {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      va[u] = (sa[u] >= 0) ? Kx[sa[u]] : 0.0;
      vb[u] = (sb[u] >= 0) ? Kx[sb[u]] : 0.0;
    }
  };
  auto gather_store = [&](int nrow, int q0) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int q = q0 + u * FTN + tid;
      if (q < nrow) LQ[q] = double2{va[u], vb[u]};
    }
  };
  // the leaf tables (first row, w | rc, L offset, first pivot) of batch b + 1 are loaded during batch
  // b's L and product phases (after batch b's pivots consumed them): no exposed round trip in the
  // gather and pivot phases (r5: two per batch, ~3 us of the level-2 fronts' ~13 us per batch)
  int64_t laf[2], llo[2];
  int32_t lwr[2], lf0[2];
  auto leaf_tab = [&](int kb, int nl) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = tid + h * FTN;
      const bool ok = k < nl;
      laf[h] = ok ? T.ab_first[kb + k] : 0;
      lwr[h] = ok ? T.ab_wrc[kb + k] : 0;
      llo[h] = ok ? T.ab_loff[kb + k] : 0;
      lf0[h] = ok ? T.ab_f0[kb + k] : 0;
    }
  };
  // batch 0's leaf tables, first gather pass and first product group (its table entries as uniform
  // loads) and this front's original K entries, all in one round trip; their K values (the leaf rows'
  // and the front's own) in a second — the zero fill of the front beside them
  if (nb > 0) {
    leaf_tab(F0.kq0, F0.kq1 - F0.kq0);
    gather_idx(F0.row0, (int)(F0.row1 - F0.row0), 0);
    load_group(e, T.fold_prod + F0.poff + tid, 0, F0.plen);
  } else {
    gather_idx(0, 0, 0);  // no leaves: no loads
  }
  const int64_t qa = with_asm ? T.asm_ptr[s] + tid : 0, qe = with_asm ? T.asm_ptr[s + 1] : 0;
  const bool a0 = qa < qe;
  const int ad = a0 ? (int)T.asm_dst[qa] : 0;
  const int64_t as = a0 ? T.asm_src[qa] : 0;
  const int ntot = PK ? r * (r + 1) / 2 : r * ld;
  for (int q = tid; q < ntot; q += FTN) A[q] = 0.0;
  const double av = a0 ? Kx[as] : 0.0;
  gather_val();
  if (tid <= nb) {
    tb_k[tid] = rk;
    tb_j[tid] = rj;
    if (tid < nb) tb_po[tid] = rpo, tb_pl[tid] = rpl;
  }
  __syncthreads();  // the zero fill
  if (a0) {
    const int dj = ad / r;  // d < r^2: 32-bit division
    A[fidx<PK>(ad - dj * r, dj, r, ld)] = av;
  }
  for (int64_t q = qa + FTN; q < qe; q += FTN) {
    const int d = (int)T.asm_dst[q], dj = d / r;
    A[fidx<PK>(d - dj * r, dj, r, ld)] = Kx[T.asm_src[q]];
  }
  __syncthreads();  // the batch table and the original entries
  for (int b = 0; b < nb; ++b) {
    const int k0 = tb_k[b], k1 = tb_k[b + 1];
    const int64_t j0 = tb_j[b];
    const int nrow = (int)(tb_j[b + 1] - j0), nleaf = k1 - k0;
    if (nrow > RM || nleaf > LM || nleaf > 2 * FTN) {  // a batch beyond the carve the front was sized by
      if (tid == 0) __hip_atomic_fetch_or(T.err, kErrLdsCarve, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;  // (uniform: the batch table is in LDS)
    }
    // (1) the leaf rows' K entries (the first pass and the leaf tables in registers already)
    gather_store(nrow, 0);
    for (int q0 = RPT * FTN; q0 < nrow; q0 += RPT * FTN) {
      gather_idx(j0, nrow, q0);
      gather_val();
      gather_store(nrow, q0);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = tid + h * FTN;
      if (k < nleaf) {
        const int q0 = (int)(laf[h] - j0), wrc = lwr[h];
        prow0[k] = q0;
        pwrc[k] = wrc;
        ploff[k] = llo[h];
        pf0[k] = lf0[h];
        for (int i = 0; i < (wrc >> 8); ++i) kk[q0 + i] = k;
      }
    }
    __syncthreads();
    lap(0);
    const bool pre = b + 1 < nb;  // prefetch the next batch's first pass and leaf tables
    if (pre) {
      gather_idx(tb_j[b + 1], (int)(tb_j[b + 2] - tb_j[b + 1]), 0);
      leaf_tab(tb_k[b + 1], tb_k[b + 2] - tb_k[b + 1]);
    }
    lap(1);
    // (2) per leaf row: the leaf's pivots from its first two rows (rows i < w, never rewritten here;
    // every row's thread forms them itself: no per-leaf phase and barrier), then its L entries (HBM
    // panel for the solves: d on the diagonal, zero above; LDS: l and l d of the update rows); the
    // first row's thread stores D and checks the pivots
    for (int q = tid; q < nrow; q += FTN) {
      const int k = kk[q];
      const int wrc = pwrc[k], w = wrc & 255, rc = wrc >> 8, jf = prow0[k], i = q - jf;
      const double2 r0 = LQ[jf], r1 = (w == 2) ? LQ[jf + 1] : double2{0.0, 0.0};
      const double d0 = r0.x, f10 = r1.x;
      const double l10 = (w == 2) ? f10 / d0 : 0.0;
      const double d1 = (w == 2) ? r1.y - l10 * f10 : 0.0;
      double* __restrict__ L = arena + ploff[k];
      if (i >= w) {
        const double2 a = LQ[q];
        const double li0 = a.x / d0;
        const double li1 = (w == 2) ? (a.y - li0 * f10) / d1 : 0.0;
        LQ[q] = double2{li0, li1};
        PQ[q] = double2{li0 * d0, li1 * d1};
        L[i] = li0;
        if (w == 2) L[i + rc] = li1;
      } else if (i == 0) {
        L[0] = d0;
        if (w == 2) L[rc] = 0.0;
        const int f0 = pf0[k];
        D[f0] = d0;
        if (bad_pivot(d0, tol)) atomicMin(&st->fail_pivot, f0 + 1);
        if (w == 2) {
          D[f0 + 1] = d1;
          if (bad_pivot(d1, tol)) atomicMin(&st->fail_pivot, f0 + 2);
        }
      } else {  // i == 1, w == 2
        L[1] = l10;
        L[1 + rc] = d1;
      }
    }
    __syncthreads();
    lap(2);
    if (pre) gather_val();
    // (3) this thread's chunk of the destination-sorted products (entry k at FTN k + tid: each load
    // instruction is coalesced)
    const uint32_t* __restrict__ P = T.fold_prod + tb_po[b] + tid;
    const int len = tb_pl[b];
    const uint32_t head = T.fold_chead[(int64_t)(b0 + b) * FTN + tid];
    int d = (int)(head & 0xffffu);              // the running destination
    bool park = (head & SymbolicPlan::kFoldCont) != 0;  // the first run continues the left chunk's
    cdst[tid] = -1;
    double acc = 0.0;  // the negated sum of the open run
    for (int k = 0; k < len; k += GP) {
      uint32_t nx[GP];
      if (k + GP < len) {
        load_group(nx, P, k + GP, len);
      } else if (b + 1 < nb) {  // the next batch's first group
        load_group(nx, T.fold_prod + tb_po[b + 1] + tid, 0, tb_pl[b + 1]);
      }
      // every LDS operand of the group is read before its first update of A (a kFoldPad entry reads
      // row 0 and adds nothing)
      double v[GP];
#pragma unroll
      for (int u = 0; u < GP; ++u) {
        const uint32_t q1 = e[u] & 0xfffu, q2 = (e[u] >> 12) & 0xfffu;
        const bool pad = q1 == PAD;
        const double2 la = LQ[pad ? 0u : q1], pb = PQ[q2];
        v[u] = pad ? 0.0 : fma(la.x, pb.x, la.y * pb.y);
      }
      // a run's sum is subtracted at its last entry with a non-returning LDS atomic — one writer per
      // address (a run split by a chunk cut parks its continuation parts instead), so the result is
      // deterministic, and no wait for the old value.  Selects and one predicated atomic per entry;
      // padding never ends a run, and acc restarts every batch.
#pragma unroll
      for (int u = 0; u < GP; ++u) {
        d += (int)((e[u] >> 24) & 127u);
        const bool end = (int32_t)e[u] < 0;
        const double sum = acc - v[u];
        if (end && park) {
          cval[tid] = sum;
          cdst[tid] = d;
        } else if (end) {
          __hip_atomic_fetch_add(A + d, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        park = park && !end;
        acc = end ? 0.0 : sum;
      }
      if (k + GP < len || b + 1 < nb) {
#pragma unroll
        for (int u = 0; u < GP; ++u) e[u] = nx[u];
      }
    }
    if (len == 0 && b + 1 < nb) load_group(e, T.fold_prod + tb_po[b + 1] + tid, 0, tb_pl[b + 1]);
    __syncthreads();
    // the parked parts, left to right: the first chunk of each continued run adds the run's parts
    if (cdst[tid] >= 0 && (tid == 0 || cdst[tid - 1] != cdst[tid])) {
      const int dd = cdst[tid];
      double t = 0.0;
      for (int u = tid; u < FTN && cdst[u] == dd; ++u) t += cval[u];
      A[dd] += t;
    }
    __syncthreads();
    lap(3);
  }
  if (fdg && threadIdx.x == 0)
    for (int k = 0; k < 4; ++k) fdg[k] = tph[k];
}

// ------------------------------------------------------------------ factorisation tree
// ONE launch factorises every tree front (SymbolicPlan::ftree: phase-1 fronts of <= 192 rows whose
// children are pre-leaves or tree fronts).  Workgroups take fronts in topological order from an
// atomic ticket (no deadlock at any grid size); a front stages its pre-assembled scratch (original
// entries + pre-leaf children, one gather pass before this launch) into LDS, then waits for its tree
// children's flags and adds their update blocks child by child (sc1 loads; the children stored them
// write-through), factorises in LDS and publishes (every wave drains, barrier, one flag store).  The
// last workgroup to finish resets the ticket counters for the next launch.
// Child update block -> parent front in LDS: child columns dealt to waves (NC per wave and round,
// NH 64-row chunks), all of a round's loads (sc1: handed over inside the launch) issued before the
// read-modify-writes; the parent column base is wave-uniform, so a row costs one rels lookup.
// Destinations are distinct within a child, so all LDS reads of a round precede its writes.
#ifndef PUSH_NC2
#define PUSH_NC2 8
#endif
#ifndef PUSH_NC3
#define PUSH_NC3 6
#endif
template <bool PK, int NH, int NC>
__device__ __forceinline__ void push_cols(double* A, int r, int ld, const double* U, int64_t uld, int uc,
                                          const int32_t* rels) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  for (int b0 = NC * wv; b0 < uc; b0 += nw * NC) {
    // every global load of the round first, from clamped addresses (no branches between them)
    double x[NC][NH];
#pragma unroll
    for (int cb = 0; cb < NC; ++cb) {
      const int bc = min(b0 + cb, uc - 1);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int ac = min(b0 + cb + lane + 64 * h, uc - 1);
        x[cb][h] = __hip_atomic_load(U + ac + ucol_off(bc, uc, uld), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // then the destinations (relative indices in LDS) and the read-modify-writes
    int dst[NC][NH];
#pragma unroll
    for (int cb = 0; cb < NC; ++cb) {
      const int b = b0 + cb, j = rels[min(b, uc - 1)];
      const int base = PK ? ((j * (2 * r - j - 1)) >> 1) : j * ld;  // fidx(i, j) = base + i
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int a = b + lane + 64 * h;
        dst[cb][h] = (b < uc && a < uc) ? base + rels[min(a, uc - 1)] : -1;
      }
    }
#pragma unroll
    for (int cb = 0; cb < NC; ++cb)
#pragma unroll
      for (int h = 0; h < NH; ++h) x[cb][h] += A[max(dst[cb][h], 0)];
#pragma unroll
    for (int cb = 0; cb < NC; ++cb)
#pragma unroll
      for (int h = 0; h < NH; ++h)
        if (dst[cb][h] >= 0) A[dst[cb][h]] = x[cb][h];
  }
}

template <bool PK>
__device__ __forceinline__ void fact_tree_front(const FrontTab& T, int s, const int32_t* __restrict__ dep, int q0, int q1,
                                                int32_t* flags, int epoch, const double* Kx, double* arena,
                                                const double* fscratch,
                                                double* D, LDLStatus* st, double tol, int32_t* err, double* A,
                                                double* Dl, double* MK, double* cbuf, int32_t* rels, int64_t* dg) {
  const int tid = threadIdx.x;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int ld = PK ? 0 : (r | 1);
  const FoldStart F0 = T.fstart[s];  // (with the front's other words: no dependent round trip later)
  // the fold helper (if any) and its flag / image, loaded now — after the fold they were two dependent
  // round trips in front of the children's wait
  const int hh = T.absorb[s] ? T.fold_help[s] : -1;
  const int hflag = hh >= 0 ? T.fhelp[hh].flag : 0;
  const int64_t himg = hh >= 0 ? T.fhelp[hh].img : 0, hdofs = hh >= 0 ? T.fhelp[hh].dofs : 0;
  const int hnimg = hh >= 0 ? T.fhelp[hh].nimg : 0;
  {  // the front and its leaf batches must fit the launch's LDS: else a sticky error, never a write
     // past the carve (the symbolic analysis sizes both; this catches a plan that breaks it)
    const int ntot = PK ? r * (r + 1) / 2 : r * ld;
    const int64_t need = 8 * (int64_t)((ntot + 1) & ~1) +
                         (T.absorb[s] ? (int64_t)SymbolicPlan::kFoldRowBytes * T.fold_rmax[s] +
                                            (int64_t)SymbolicPlan::kFoldLeafBytes * T.fold_lmax[s]
                                      : 0);
    if (need > T.lds_cap) {
      if (tid == 0) {
        __hip_atomic_fetch_or(T.err, kErrLdsCarve, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&flags[s], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);  // release the parent
      }
      return;
    }
  }
  if (T.absorb[s]) {  // original entries, then the micro-leaf children folded in LDS
    const int ntot = PK ? r * (r + 1) / 2 : r * ld;
    fold_leaves<PK>(T, s, r, ld, A, Kx, arena, D, st, tol, A + ((ntot + 1) & ~1), cbuf, reinterpret_cast<int32_t*>(MK),
                    dg ? dg + 16 : nullptr, F0, true);  // 16-byte aligned
  } else {  // pre-assembled as the LDS image: a straight copy, 16 loads in flight per thread
    const double* __restrict__ src = fscratch + T.fs_off[s];
    const int n = PK ? r * (r + 1) / 2 : r * ld;
    for (int base = 0; base < n; base += FTN * 16) {
      double v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int q = base + k * FTN + tid;
        v[k] = (q < n) ? src[q] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int q = base + k * FTN + tid;
        if (q < n) A[q] = v[k];
      }
    }
  }
  if (dg) {
    __syncthreads();
    if (tid == 0) dg[1] = wall_clock64();
  }
  if (q1 > q0) {  // the first child's relative indices are symbolic: load them before the wait
    const int c = dep[q0];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    for (int a = tid; a < uc; a += FTN) rels[a] = T.rel[T.rel_ptr[c] + a];
  }
  if (tid < 64) poll_deps(dep, q0, q1, flags, epoch, err);
  if (hh >= 0 && tid == 0) poll_flag(flags + hflag, epoch, err);  // the helper that folded the first batches
  __syncthreads();
  if (dg && tid == 0) dg[2] = wall_clock64();
  if (hh >= 0) {  // its image — the entries its products reached, in LDS order — added entry by entry,
                  // 16 loads in flight per thread (the untouched entries, zero in the image, are skipped)
    const double* __restrict__ img = T.fimg + himg;
    const uint16_t* __restrict__ hd = T.fimg_dst + hdofs;
    for (int base = 0; base < hnimg; base += FTN * 16) {
      double v[16];
      int q[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int e = min(base + k * FTN + tid, hnimg - 1);
        v[k] = ld_sc1(img + e);
        q[k] = hd[e];
      }
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (base + k * FTN + tid < hnimg) A[q[k]] += v[k];
    }
    __syncthreads();
  }
  for (int q = q0; q < q1; ++q) {  // tree children, child order
    const int c = dep[q];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const int64_t uld = T.u_ld[c];
    const double* U = arena + T.u_off[c];
    if (q > q0) {
      for (int a = tid; a < uc; a += FTN) rels[a] = T.rel[T.rel_ptr[c] + a];
      __syncthreads();
    }
    // one memory round trip per round: 8 waves x NC columns
    if (uc <= 64)
      push_cols<PK, 1, 8>(A, r, ld, U, uld, uc, rels);
    else if (uc <= 128)
      push_cols<PK, 2, PUSH_NC2>(A, r, ld, U, uld, uc, rels);
    else
      push_cols<PK, 3, PUSH_NC3>(A, r, ld, U, uld, uc, rels);
    __syncthreads();
  }
  if (dg && tid == 0) dg[3] = wall_clock64();
  factor_lds<PK>(T, A, r, w, ld, Dl, MK, cbuf, dg ? dg + 8 : nullptr);
  if (dg && tid == 0) dg[4] = wall_clock64();
  // the parent reads only U: publish it first, then write L and D (read by later launches)
  writeout_u<PK, true>(A, r, w, ld, arena + T.u_off[s], T.u_ld[s]);
  if (dg) {
    __syncthreads();
    if (tid == 0) dg[14] = wall_clock64();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(&flags[s], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (dg && tid == 0) dg[15] = wall_clock64();
  writeout_ld<PK>(A, r, w, ld, Dl, arena + T.l_off[s], D, f0, st, tol);
  if (dg && tid == 0) {
    dg[5] = wall_clock64();
    dg[6] = s;
    dg[7] = r;
  }
}

// ---- Medium tree fronts (kFactTreeMax < r <= kFactTreeMedMax): the front F (r x r, ld r, big-front
// storage: L = F[:, :w], U = F[w:, w:] in place) stays in HBM — pre-assembled there by the gather pass
// (original entries + pre-leaf children) — and ONE workgroup factorises it panel by panel, right-looking:
//   children: the tree children's update blocks are added into F (read-modify-write, child order);
//   panel k (columns c0 .. c0 + pw, pw <= 64): rows c0 .. r staged into LDS as an (r - c0) x pw front,
//     factorised by the in-LDS schedule without its Schur pass (blocked_factor_pipe, defer 2), written
//     back (L, d on the diagonal, D, pivot check);
//   trailing update in HBM: F[i, j] -= sum_t L(i, t) d_t L(j, t) over the panel's columns, i >= j >= c0 + pw,
//     16 x 16 tiles on f64 MFMA with both operands from the LDS panel (tile rows along the lanes:
//     16 consecutive rows of one column per store, coalesced); the last panel's tiles are the update
//     block U, stored write-through (sc1) for the parent, then the flag.
// (The level path ran each 64-column panel of these fronts as three launches, k_big_diag -> k_big_trsm
// -> k_big_update, per level: ~37 us per panel plus the launch gaps, supportcase10's fronts r ~ 230.)
constexpr int MED_PW = 64;
__device__ __forceinline__ void med_trailing(double* __restrict__ F, int r, int c0, int pw, const double* A, int ld,
                                             const double* Dl, bool last) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  const int rp = r - c0;                // panel rows (LDS row i' = front row c0 + i')
  const int nb = (rp - pw + 15) >> 4;   // 16-row blocks of the trailing matrix
  const int ntile = nb * (nb + 1) / 2;
  const int nks = (pw + 3) >> 2;
  const int kl = lane >> 4, il = lane & 15;
  // tile t -> (I, J), J <= I, row-major over the lower triangle; its C entries (lane: row i0 + il,
  // columns j0 + kl + 4 g), clamped in range — the next tile's C is loaded before this tile's MFMAs
  auto coords = [&](int t, int& i0, int& j0) {
    int I = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    while (I * (I + 1) / 2 > t) --I;
    const int J = t - I * (I + 1) / 2;
    i0 = pw + 16 * I;  // LDS rows of the tile's rows (i) and columns (j)
    j0 = pw + 16 * J;
  };
  auto load_c = [&](int t, double (&c)[4]) {
    int i0, j0;
    coords(min(t, ntile - 1), i0, j0);
    const int ic = min(i0 + il, rp - 1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int jc = min(j0 + kl + 4 * g, rp - 1);
      c[g] = F[(int64_t)(c0 + ic) + (int64_t)(c0 + jc) * r];
    }
  };
  // C of the next TWO tiles in flight while a tile's MFMAs run (one ahead left each wave's C loads
  // exposed: a tile's 16 k-steps take ~0.4 us against a ~1-2 us HBM round trip)
  double c[4], cn[4];
  if (wv < ntile) {
    load_c(wv, c);
    load_c(wv + nw, cn);
  }
  for (int t = wv; t < ntile; t += nw) {
    int i0, j0;
    coords(t, i0, j0);
    double cnn[4];
    load_c(t + 2 * nw, cnn);  // (clamped: the last tile's again when there is no such tile)
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    const int ja = min(j0 + il, rp - 1), ib = min(i0 + il, rp - 1);
    for (int ks = 0; ks < nks; ++ks) {
      const int k = 4 * ks + kl;
      const int kc = min(k, pw - 1);
      const double d = (k < pw) ? Dl[kc] : 0.0;
      const double av = A[ja + kc * ld] * d;   // A operand: (m = il -> column j0 + il, k)
      const double bv = A[ib + kc * ld];       // B operand: (k, n = il -> row i0 + il)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
    // result lane l, element g: (m = kl + 4 g -> column j0 + m, n = il -> row i0 + il)
    const int i = i0 + il;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = j0 + kl + 4 * g;
      if (i < rp && j < rp && i >= j) {
        double* q = F + (int64_t)(c0 + i) + (int64_t)(c0 + j) * r;
        const double v = c[g] - acc[g];
        if (last)
          __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          *q = v;
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      c[g] = cn[g];
      cn[g] = cnn[g];
    }
  }
}

__device__ __forceinline__ void fact_med_front(const FrontTab& T, int s, const int32_t* __restrict__ dep, int q0, int q1,
                                               int32_t* flags, int epoch, double* arena, double* D, LDLStatus* st,
                                               double tol, int32_t* err, double* A, double* Dl, double* MK, double* cbuf,
                                               int64_t* dg) {
  const int tid = threadIdx.x;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  double* __restrict__ F = arena + T.l_off[s];
  if (dg && tid == 0) dg[1] = wall_clock64();  // (no staging: the front lives in HBM)
  if (tid < 64) poll_deps(dep, q0, q1, flags, epoch, err);
  __syncthreads();
  if (dg && tid == 0) dg[2] = wall_clock64();
  // tree children's update blocks (agent-scope loads: written by other workgroups), child order
  for (int q = q0; q < q1; ++q) {
    const int c = dep[q];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const int64_t uld = T.u_ld[c];
    const double* U = arena + T.u_off[c];
    const int32_t* __restrict__ rl = T.rel + T.rel_ptr[c];
    const int ne = uc * uc;
    for (int base = 0; base < ne; base += FTN * 8) {
      double x[8];
      int64_t dst[8];
      int32_t ra[8], rb[8];
      bool ok[8];
      // every load of the round first and unconditional (a, b are in range: e is clamped) — the
      // relative indices loaded under `ok` compiled into a branch with a wait per entry, 8 serial
      // round trips per round (r5: the critical level-3/4 medium fronts of supportcase10 spent 40-60
      // us here)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = min(base + k * FTN + tid, ne - 1);
        const int b = e / uc, a = e - b * uc;
        ok[k] = base + k * FTN + tid < ne && a >= b;
        x[k] = __hip_atomic_load(U + max(a, b) + ucol_off(b, uc, uld), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ra[k] = rl[a];
        rb[k] = rl[b];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(ra[k]), "+v"(rb[k]));
#pragma unroll
      for (int k = 0; k < 8; ++k) dst[k] = ok[k] ? (int64_t)ra[k] + (int64_t)rb[k] * r : -1;
      // the read-modify-writes: every F load of the round first, unconditional from clamped addresses
      // (a masked += compiled into a branch with a wait inside: 8 serial round trips per round)
      double f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = F[max(dst[k], (int64_t)0)];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (dst[k] >= 0) F[dst[k]] = f[k] + x[k];
    }
    __syncthreads();
  }
  if (dg && tid == 0) dg[3] = wall_clock64();
  for (int c0 = 0; c0 < w; c0 += MED_PW) {
    const int pw = min(MED_PW, w - c0), rp = r - c0, ld = rp | 1;
    const bool last = c0 + pw >= w;
    // stage rows c0 .. r of the panel's columns (lower part) into LDS, 16 loads in flight per thread
    const int ne = rp * pw;
    for (int base = 0; base < ne; base += FTN * 16) {
      double v[16];
      int dst[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int e = base + k * FTN + tid;
        const int ec = min(e, ne - 1);
        const int j = ec / rp, i = ec - j * rp;
        v[k] = F[(int64_t)(c0 + i) + (int64_t)(c0 + j) * r];
        dst[k] = (e < ne && i >= j) ? i + j * ld : -1;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (dst[k] >= 0) A[dst[k]] = v[k];
    }
    __syncthreads();
    blocked_factor_pipe<false>(A, rp, pw, ld, Dl, MK, cbuf, 2, nullptr, T.err, 0);
    __syncthreads();
    // write back: L (d on the diagonal), D + pivot check
    for (int base = 0; base < ne; base += FTN * 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = base + k * FTN + tid;
        if (e < ne) {
          const int j = e / rp, i = e - j * rp;
          if (i >= j) F[(int64_t)(c0 + i) + (int64_t)(c0 + j) * r] = (i == j) ? Dl[j] : A[i + j * ld];
        }
      }
    }
    if (tid < pw) {
      const double d = Dl[tid];
      D[f0 + c0 + tid] = d;
      if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + c0 + tid + 1);
    }
    if (rp > pw) med_trailing(F, r, c0, pw, A, ld, Dl, last);
    __syncthreads();  // the next panel's staging reads the updated trailing matrix; A is rewritten
  }
  if (dg && tid == 0) dg[4] = wall_clock64();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(&flags[s], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (dg && tid == 0) {
    dg[5] = wall_clock64();
    dg[6] = s;
    dg[7] = r;
  }
}

// A fold helper: the first batches of a front's micro leaves (FoldHelp [b0, b1)) folded into a zeroed
// LDS image of the front — their L and D written as the front's own — and the image stored
// write-through for the front, which adds it after its own batches and waits (fixed order: bitwise
// reproducible).  The helpers take the first tickets, so the heaviest fronts' folds are split over two
// CUs (ex10: 272 fronts of 35-50 us of folding on 256 CUs made the 16 late level-2 fronts the chain).
template <bool PK>
__device__ __forceinline__ void fold_help_task(const FrontTab& T, int h, int32_t* flags, int epoch, const double* Kx,
                                               double* arena, double* D, LDLStatus* st, double tol, double* A,
                                               double* MK, double* cbuf) {
  const int tid = threadIdx.x;
  const FoldHelp H = T.fhelp[h];
  const int s = H.front, r = T.nrows[s], ld = PK ? 0 : (r | 1);
  const int ntot = PK ? r * (r + 1) / 2 : r * ld;
  const int64_t need = 8 * (int64_t)((ntot + 1) & ~1) + (int64_t)SymbolicPlan::kFoldRowBytes * T.fold_rmax[s] +
                       (int64_t)SymbolicPlan::kFoldLeafBytes * T.fold_lmax[s];
  if (need > T.lds_cap) {  // as the front's own check: a sticky error, never a write past the carve
    if (tid == 0) {
      __hip_atomic_fetch_or(T.err, kErrLdsCarve, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&flags[H.flag], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  fold_leaves<PK>(T, s, r, ld, A, Kx, arena, D, st, tol, A + ((ntot + 1) & ~1), cbuf, reinterpret_cast<int32_t*>(MK),
                  nullptr, H.fs, false);
  __syncthreads();
  double* __restrict__ img = T.fimg + H.img;  // only the entries its products reached (fimg_dst)
  const uint16_t* __restrict__ hd = T.fimg_dst + H.dofs;
  for (int k = tid; k < H.nimg; k += FTN) st_sc1(img + k, A[hd[k]]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(&flags[H.flag], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(FTN) void k_fact_tree(FrontTab T, const int32_t* __restrict__ order, int nt, int nhelp,
                                                  const int32_t* __restrict__ dep_ptr, const int32_t* __restrict__ dep,
                                                  int32_t* counter, int32_t* flags, int epoch,
                                                  const double* __restrict__ Kx, double* arena,
                                                  const double* __restrict__ fscratch, double* D, LDLStatus* st,
                                                  double tol, int32_t* err, int64_t* dbg) {
  extern __shared__ __attribute__((aligned(16))) double A[];
  __shared__ double Dl[192];
  __shared__ double MK[16 * LDM];
  __shared__ __attribute__((aligned(16))) double cbuf[2 * 16 * LDM];
  __shared__ int32_t rels[192];
  __shared__ int s_task;
  if (threadIdx.x == 0) s_task = atomicAdd(counter, 1);
  __syncthreads();
  const int t = s_task;
  if (t >= nt) return;
  if (t < nhelp) {  // fold helper tickets first (no dependencies)
    const int sh = T.fhelp[t].front;
    if (T.nrows[sh] <= 128 && !T.fold_pk[sh])
      fold_help_task<false>(T, t, flags, epoch, Kx, arena, D, st, tol, A, MK, cbuf);
    else
      fold_help_task<true>(T, t, flags, epoch, Kx, arena, D, st, tol, A, MK, cbuf);
  } else {
  const int s = order[t - nhelp];
  int64_t* dg = dbg ? dbg + 24 * t : nullptr;
  if (dg && threadIdx.x == 0) dg[0] = wall_clock64();
  if (T.nrows[s] > SymbolicPlan::kFactTreeMax)
    fact_med_front(T, s, dep, dep_ptr[t], dep_ptr[t + 1], flags, epoch, arena, D, st, tol, err, A, Dl, MK, cbuf, dg);
  else if (T.nrows[s] <= 128 && !T.fold_pk[s])
    fact_tree_front<false>(T, s, dep, dep_ptr[t], dep_ptr[t + 1], flags, epoch, Kx, arena, fscratch, D, st, tol, err, A, Dl,
                           MK, cbuf, rels, dg);
  else
    fact_tree_front<true>(T, s, dep, dep_ptr[t], dep_ptr[t + 1], flags, epoch, Kx, arena, fscratch, D, st, tol, err, A, Dl,
                          MK, cbuf, rels, dg);
  }
  if (threadIdx.x == 0 && atomicAdd(counter + 1, 1) == nt - 1) {  // last one out: reset the tickets
    counter[0] = 0;
    counter[1] = 0;
  }
}

// Diagonal block of 64-column panel `step` (one workgroup per front): load, blocked factorisation,
// write L11 (d on the diagonal), D and the M_K blocks for k_big_trsm.
// The diagonal block of panel `step` of front s, staged in A64 (lower part, identity-padded past kw):
// blocked factorisation, then L11 (d on the diagonal), D and the M_K blocks for k_big_trsm.
// Loads / stores of the big-front panel kernels: plain in their own launches (kernel boundaries order
// them), write-through (sc1) stores and sc1 loads inside k_big_dag, whose tasks hand tiles to each
// other within one launch (every handed-off byte stored sc1 and drained before the flag, every load
// of it sc1: the guide's Guideline 16, R1 without an acquire).
// (global address space explicitly: inside a non-inlined task body a generic pointer compiles to flat_
// loads / stores, which also count on lgkmcnt — every LDS wait then waits for them — and are not the
// global_ sc1 accesses the hand-off protocol requires)
typedef __attribute__((address_space(1))) double gdouble;
template <bool SC>
__device__ __forceinline__ double ldF(const double* p) {
  if constexpr (SC) return __hip_atomic_load((const gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *(const gdouble*)p;
}
template <bool SC>
__device__ __forceinline__ void stF(double* p, double v) {
  if constexpr (SC) __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *(gdouble*)p = v;
}
constexpr int BIG_MSZ = 4 * 16 * LDM;  // doubles of one panel's M_K blocks

// the diagonal block of panel `step`, staged in A64: factorised; L11 (d on the diagonal), D and the
// M_K blocks (to M: the front's slot in Mbuf, or the panel's slot in k_big_dag's Mch) written
template <bool SC = false>
__device__ __forceinline__ void big_diag_tail(const FrontTab& T, int s, int step, double* A64, double* Ms, double* Dl,
                                              double* __restrict__ arena, double* __restrict__ D,
                                              double* __restrict__ M, LDLStatus* st, double tol) {
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int k0 = step * 64, kw = min(64, w - k0);
  double* __restrict__ F = arena + T.l_off[s] + k0 + (int64_t)k0 * r;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  diag64(A64, Dl, Ms, tid);
  for (int j = wv; j < kw; j += 4)
    if (lane >= j && lane < kw) stF<SC>(F + lane + (int64_t)j * r, (lane == j) ? Dl[j] : A64[lane + j * LDA]);
  if (tid < kw) {
    const double d = Dl[tid];
    stF<SC>(D + f0 + k0 + tid, d);
    if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + k0 + tid + 1);
  }
  for (int e = tid; e < BIG_MSZ; e += NT) stF<SC>(M + e, Ms[e]);
}

// Lookahead: the update launch of panel `step` leaves panel step + 1's diagonal tile final in the
// workgroup of its task (0, 0), which factorises it right away (big_diag_tail) while the launch's
// other tiles are still updated — no k_big_diag launch, and its latency off the panel chain, for
// every panel but the first.  Entry (i, j) of the tile (< 64 each) arrives through put(i, j, v).
__device__ __forceinline__ bool big_next_diag(const FrontTab& T, int s, int step) {
  return 64 * (step + 1) < T.first[s + 1] - T.first[s];
}
__device__ __forceinline__ void big_diag_prepare(double* A64, int kw) {
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * 64; e += NT) {
    const int i = e & 63, j = e >> 6;
    A64[i + j * LDA] = (i < kw && j < kw) ? 0.0 : (i == j ? 1.0 : 0.0);
  }
}

// the diagonal block of panel `step`: staged (identity-padded past kw), factorised, written (big_diag_tail)
template <bool SC>
__device__ __forceinline__ void diag_body(const FrontTab& T, int s, int step, double* __restrict__ arena,
                                          double* __restrict__ D, double* __restrict__ M, LDLStatus* st, double tol,
                                          double* sm) {
  double* A64 = sm;
  double* Ms = sm + 64 * LDA;
  double* Dl = Ms + 4 * 16 * LDM;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int k0 = step * 64, kw = min(64, w - k0);
  const double* __restrict__ F = arena + T.l_off[s] + k0 + (int64_t)k0 * r;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  (void)f0;
  {
    // all 16 loads in flight from clamped addresses, masked after (a predicated load compiles into a
    // branch with a wait of its own)
    double v[16];
    const int lc = min(lane, kw - 1);
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = ldF<SC>(F + lc + (int64_t)min(wv + 4 * e, kw - 1) * r);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int j = wv + 4 * e;
      A64[lane + j * LDA] = (lane < kw && j < kw) ? (lane >= j ? v[e] : 0.0) : (lane == j ? 1.0 : 0.0);
    }
  }
  __syncthreads();
  big_diag_tail<SC>(T, s, step, A64, Ms, Dl, arena, D, M, st, tol);
}
constexpr int DIAG_LDS = 64 * LDA + 4 * 16 * LDM + 64;
__global__ __launch_bounds__(NT) void k_big_diag(FrontTab T, const int32_t* __restrict__ list, int step,
                                                 double* __restrict__ arena, double* __restrict__ D,
                                                 double* __restrict__ Mbuf, LDLStatus* st, double tol) {
  __shared__ __attribute__((aligned(16))) double sm[DIAG_LDS];
  int s, item;
  task_of(list, s, item);
  (void)item;
  diag_body<false>(T, s, step, arena, D, Mbuf + (int64_t)T.bigslot[s] * 4096, st, tol, sm);
}

// Rows below the diagonal block of panel `step` (64-row tiles; wave w owns 16 rows): blocked
// forward substitution X_K = A_K - sum_{J<K} (L_J D_J) L_KJ^T, L_K = X_K M_K, all on f64 MFMA.
// LDS of one k_big_trsm task: L11 (64 x LDA), the M_K blocks, the pivots, four 16 x 64 slabs
constexpr int TRSM_LDS = 64 * LDA + BIG_MSZ + 64 + 4 * 17 * 64;
template <bool SC>
__device__ __forceinline__ void trsm_body(const FrontTab& T, int s, int step, int rt, double* __restrict__ arena,
                                          const double* __restrict__ D, const double* __restrict__ M, double* sm) {
  double* L11 = sm;
  double* Ms = sm + 64 * LDA;
  double* Dl = Ms + BIG_MSZ;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int k0 = step * 64, kw = min(64, w - k0);
  const int I0 = k0 + kw + rt * 64;
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double* S = Dl + 64 + wv * (17 * 64);  // this wave's slab: 16 rows x 64 cols, S[m + 17 * j]
  const int row = I0 + 16 * wv + (lane & 15);  // slab row of this lane; 4 columns per pass
  {
    // every operand load in flight at once from clamped addresses, masked at the LDS stores (a
    // predicated load compiles into a branch with a wait of its own)
    double lv[16], sv[16], mv[5], dv;
    const int lc = min(lane, kw - 1), rc = min(row, r - 1);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      lv[e] = ldF<SC>(F + (k0 + lc) + (int64_t)(k0 + min(wv + 4 * e, kw - 1)) * r);
      sv[e] = ldF<SC>(F + rc + (int64_t)(k0 + min((lane >> 4) + 4 * e, kw - 1)) * r);
    }
#pragma unroll
    for (int e = 0; e < 5; ++e) mv[e] = ldF<SC>(M + min(tid + e * NT, BIG_MSZ - 1));
    dv = ldF<SC>(D + f0 + k0 + min(tid, kw - 1));
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int j = wv + 4 * e, jj = (lane >> 4) + 4 * e;
      L11[lane + j * LDA] = (lane < kw && j < kw && lane > j) ? lv[e] : 0.0;
      S[(lane & 15) + jj * 17] = (row < r && jj < kw) ? sv[e] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 5; ++e)
      if (tid + e * NT < BIG_MSZ) Ms[tid + e * NT] = mv[e];
    if (tid < 64) Dl[tid] = (tid < kw) ? dv : 1.0;
  }
  __syncthreads();
  for (int K = 0; K < 4; ++K) {
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int J = 0; J < K; ++J) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 16 * J + 4 * ks + (lane >> 4);
        const double av = S[(lane & 15) + k * 17] * Dl[k];
        const double bv = L11[(16 * K + (lane & 15)) + k * LDA];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) S[((lane >> 4) + 4 * g) + (16 * K + (lane & 15)) * 17] -= acc[g];
    wave_sync();
    dbl4 l = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = 4 * ks + (lane >> 4);
      const double av = S[(lane & 15) + (16 * K + k) * 17];
      const double bv = Ms[K * 16 * LDM + k * LDM + (lane & 15)];
      l = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, l, 0, 0, 0);
    }
    wave_sync();
#pragma unroll
    for (int g = 0; g < 4; ++g) S[((lane >> 4) + 4 * g) + (16 * K + (lane & 15)) * 17] = l[g];
    wave_sync();
  }
  for (int j = lane >> 4; j < kw; j += 4)
    if (row < r) stF<SC>(F + row + (int64_t)(k0 + j) * r, S[(lane & 15) + j * 17]);
}

// Rows below the diagonal block of panel `step` (64-row tiles; wave w owns 16 rows): blocked
// forward substitution X_K = A_K - sum_{J<K} (L_J D_J) L_KJ^T, L_K = X_K M_K, all on f64 MFMA.
__global__ __launch_bounds__(NT) void k_big_trsm(FrontTab T, const int32_t* __restrict__ list, int step,
                                                 double* __restrict__ arena, const double* __restrict__ D,
                                                 const double* __restrict__ Mbuf) {
  __shared__ __attribute__((aligned(16))) double sm[TRSM_LDS];
  int s, rt;
  task_of(list, s, rt);
  trsm_body<false>(T, s, step, rt, arena, D, Mbuf + (int64_t)T.bigslot[s] * 4096, sm);
}

// Trailing update of one 64x64 lower tile: C -= (L_I D) L_J^T, f64 MFMA 16x16x4, over K = the
// columns of up to kpan panels (deferred multi-panel update).  Task tij = ti | tj << 16 | mode << 31:
//   mode 0 (local): K = panel `step` only, tiles relative to the panel's end, columns limited to the
//     end of the panel group (kpan panels from (step / kpan) kpan): the group's later panels only;
//   mode 1 (trailing): K = the panels of the group ending at `step`, tiles relative to the group's
//     end: the rest of the front, ONE load/store of C per group instead of one per panel.
// kpan = 1: every step is a group of one (the r2 right-looking update).  The K chunks of 64 are
// staged through LDS one after another; the next chunk's operands are loaded (from
// clamped addresses) while the current chunk's MFMAs run.
constexpr int UPD_LDT = 80;  // [k][row] layout: conflict-free ds_read_b64 for the 16x4 operand pattern
constexpr int UPD_LDS = 2 * 64 * UPD_LDT;
// Mnext: where the lookahead diagonal block's M_K blocks go (the front's Mbuf slot; k_big_dag: the
// next panel's slot)
template <bool SC>
__device__ __forceinline__ void update_body(const FrontTab& T, int s, int step, int kpan, int tij,
                                            double* __restrict__ arena, double* __restrict__ D,
                                            double* __restrict__ Mnext, LDLStatus* st, double tol, double* WLt) {
  constexpr int LDT = UPD_LDT;
  double* Wt = WLt;
  double* Lt = WLt + 64 * LDT;
  static_assert(64 * LDA <= 64 * LDT && 4 * 16 * LDM + 64 <= 64 * LDT, "lookahead diagonal block aliases Wt / Lt");
  const int ti = tij & 0xffff, tj = (tij >> 16) & 0x7fff;
  const bool trailing = tij < 0;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int g0 = (step / kpan) * kpan;                         // first panel of the group
  const int gend = min(64 * (g0 + kpan), w);                   // first column after the group
  const int kb = trailing ? 64 * g0 : 64 * step;               // K range [kb, ke)
  const int ke = trailing ? gend : min(64 * step + 64, w);
  const int c0 = ke;                                           // tiles relative to the K range's end
  const int jlim = trailing ? r : gend;
  const int I0 = c0 + ti * 64, J0 = c0 + tj * 64;
  const int nch = (ke - kb + 63) >> 6;                         // K chunks of 64 (<= kpan)
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int qr = (wv >> 1) * 32, qc = (wv & 1) * 32;
  const int ri = min(I0 + lane, r - 1), rj = min(J0 + lane, r - 1);
  // operands of chunk ch: columns kb + 64 ch + wv + 4 e (clamped into the K range); one register
  // set, reloaded with the next chunk right after its LDS stores, so those loads run under the
  // current chunk's MFMAs (which read LDS only)
  double wl[16], ll[16], dk[16];
  auto load = [&](int ch) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int kk = min(kb + 64 * ch + wv + 4 * e, ke - 1);
      const int64_t col = (int64_t)kk * r;
      wl[e] = ldF<SC>(F + ri + col);
      ll[e] = ldF<SC>(F + rj + col);
      dk[e] = ldF<SC>(D + f0 + kk);
    }
  };
  load(0);
  // C tile prefetch (its latency overlaps the first chunk)
  double c[2][2][4];
#pragma unroll
  for (int bj = 0; bj < 2; ++bj)
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = min(I0 + qr + bi * 16 + (lane & 15), r - 1);
        const int j = min(J0 + qc + bj * 16 + (lane >> 4) + 4 * g, r - 1);
        c[bj][bi][g] = ldF<SC>(F + i + (int64_t)j * r);  // masked at the store
      }
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  for (int ch = 0; ch < nch; ++ch) {
    const int kc = kb + 64 * ch, kw = min(64, ke - kc);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int kk = wv + 4 * e;
      Wt[kk * LDT + lane] = (kk < kw && I0 + lane < r) ? wl[e] * dk[e] : 0.0;
      Lt[kk * LDT + lane] = (kk < kw && J0 + lane < r) ? ll[e] : 0.0;
    }
    __syncthreads();
    if (ch + 1 < nch) load(ch + 1);  // wave-uniform
    const int nks = (kw + 3) >> 2;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      if (ks < nks) {  // wave-uniform
        const int kk = ks * 4 + (lane >> 4);
        const double a0 = Lt[kk * LDT + qc + (lane & 15)];
        const double a1 = Lt[kk * LDT + qc + 16 + (lane & 15)];
        const double b0 = Wt[kk * LDT + qr + (lane & 15)];
        const double b1 = Wt[kk * LDT + qr + 16 + (lane & 15)];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    if (ch + 1 < nch) __syncthreads();  // the LDS tiles are rewritten by the next chunk
  }
  // D layout: col n = lane&15 (-> row i of F), row m = (lane>>4) + 4g (-> column j of F)
#pragma unroll
  for (int bj = 0; bj < 2; ++bj)
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = I0 + qr + bi * 16 + (lane & 15);
        const int j = J0 + qc + bj * 16 + (lane >> 4) + 4 * g;
        if (i < r && j < jlim && i >= j) stF<SC>(F + i + (int64_t)j * r, c[bj][bi][g] - acc[bj][bi][g]);
      }
  // lookahead: task (0, 0) of a local update holds the next panel's diagonal tile, final now (the
  // panel's last local update; the next panel lies inside the group, below jlim)
  // (trailing mode, k_big_dag's tiles next to the group: only when the group is full, c0 = its end)
  if (ti == 0 && tj == 0 && (!trailing || 64 * (step + 1) == c0) && big_next_diag(T, s, step)) {
    double* A64 = Wt;  // the operand tiles are free: aliased by the diagonal block, M_K and pivots
    double* Ms = Lt;
    double* Dl = Lt + 4 * 16 * LDM;
    const int kw = min(64, w - c0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's C stores land before L11's (same addresses)
    __syncthreads();  // every wave's last MFMA operand read
    big_diag_prepare(A64, kw);
    __syncthreads();
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i = qr + bi * 16 + (lane & 15), j = qc + bj * 16 + (lane >> 4) + 4 * g;
          if (i < kw && j < kw && i >= j) A64[i + j * LDA] = c[bj][bi][g] - acc[bj][bi][g];
        }
    __syncthreads();
    big_diag_tail<SC>(T, s, step + 1, A64, Ms, Dl, arena, D, Mnext, st, tol);
  }
}

__global__ __launch_bounds__(NT) void k_big_update(FrontTab T, const int32_t* __restrict__ list, int step, int kpan,
                                                   double* __restrict__ arena, double* __restrict__ D,
                                                   double* __restrict__ Mbuf, LDLStatus* st, double tol) {
  __shared__ __attribute__((aligned(16))) double WLt[UPD_LDS];
  int s, tij;
  task_of(list, s, tij);
  update_body<false>(T, s, step, kpan, tij, arena, D, Mbuf + (int64_t)T.bigslot[s] * 4096, st, tol, WLt);
}

// (pos, neg, zero) of D over the columns with colmask == want (colmask NULL: all)
__global__ __launch_bounds__(NT) void k_inertia(const double* __restrict__ D, int n, LDLStatus* st, int spd,
                                                const uint8_t* __restrict__ colmask, int want) {
  __shared__ int red[3][NT / 64];
  int pos = 0, neg = 0, zero = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (colmask && colmask[i] != want) continue;
    const double d = D[i];
    pos += d > 0.0;
    neg += d < 0.0;
    zero += !(d > 0.0) && !(d < 0.0);
    if (spd && !(d > 0.0)) atomicMin(&st->fail_pivot, i + 1);
  }
  for (int o = 32; o > 0; o >>= 1) {
    pos += __shfl_down(pos, o, 64);
    neg += __shfl_down(neg, o, 64);
    zero += __shfl_down(zero, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = pos;
    red[1][wv] = neg;
    red[2][wv] = zero;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int v = 0;
    for (int q = 0; q < NT / 64; ++q) v += red[threadIdx.x][q];
    atomicAdd(threadIdx.x == 0 ? &st->npos : (threadIdx.x == 1 ? &st->nneg : &st->nzero), v);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && want != 1) st->t1 = wall_clock64();  // end of the factorisation
}

// LDLSolver::count_inertia (lazily, after a factorisation without k_inertia): clear the counts; then
// k_inertia with want = 1 and no column mask counts every pivot and leaves the t1 stamp alone
__global__ void k_zero_counts(LDLStatus* st) { st->npos = st->nneg = st->nzero = 0; }

// ------------------------------------------------------------------ batched leaf columns (SymbolicPlan::lb)
// A group: n single-column leaf fronts c_j under one parent P, W (m x n, ld m) = their K columns on the
// parent rows gpos, d_j = K(c_j, c_j).  Factor: L(:, c_j) = W(:, j) / d_j, and P absorbs
// F_P[gpos, gpos] -= W D^{-1} W^T (one SYRK instead of n rank-1 fronts).

// W / d from the caller's values: one workgroup per member column (contiguous CSC run)
__global__ __launch_bounds__(NT) void k_lb_build(const SymbolicPlan::LBGroup* __restrict__ G,
                                                 const int32_t* __restrict__ gid, const int32_t* __restrict__ mem,
                                                 const int64_t* __restrict__ cs, const int64_t* __restrict__ ce,
                                                 const int64_t* __restrict__ wbase, const int32_t* __restrict__ wrow,
                                                 const double* __restrict__ Kx, double* __restrict__ W,
                                                 double* __restrict__ dlb, double* __restrict__ dinv,
                                                 double* __restrict__ D, LDLStatus* st, double tol) {
  const int j = blockIdx.x;
  const SymbolicPlan::LBGroup g = G[gid[j]];
  double* __restrict__ Wc = W + g.w_off + (int64_t)(j - g.mem_off) * g.m;
  const int64_t c0 = cs[j], c1 = ce[j];
  const int32_t* __restrict__ wr = wrow + wbase[j] - c0;
  for (int64_t e = c0 + threadIdx.x; e < c1; e += NT) {
    const int k = wr[e];
    const double v = Kx[e];
    if (k >= 0) {
      Wc[k] = v;
    } else {
      dlb[j] = v;
      dinv[j] = 1.0 / v;
      D[mem[j]] = v;
      if (bad_pivot(v, tol)) atomicMin(&st->fail_pivot, mem[j] + 1);
    }
  }
}

// F[gpos[a], gpos[b]] -= sum_{j in [k0, k1)} W[a, j] W[b, j] / d_j for a >= b: 128 x 128 output
// tiles (lower), 4 waves of 64 x 64 (4 x 4 f64 MFMA 16x16x4 blocks each), K staged through LDS
// 16 columns at a time (double-buffered, operands [k][row] with a padded stride).  One launch per
// K-chunk keeps the chunk of W (m x 2048) resident in the Infinity Cache across all tiles.
constexpr int SYT = 128, SYK = 16, SYLD = SYT + 16;
#ifndef SYRK_WAVES
#define SYRK_WAVES 2  // waves per SIMD the register budget is cut for (2: accumulators in VGPRs, 2 WGs per CU)
#endif
__global__ __launch_bounds__(NT, SYRK_WAVES) void k_lb_syrk(const double* __restrict__ W, const double* __restrict__ dinv, int m,
                                                int k0, int k1, const int32_t* __restrict__ gpos,
                                                double* __restrict__ F, int ld) {
  __shared__ __attribute__((aligned(16))) double As[2][SYK * SYLD];  // (W D^{-1})[I rows]
  __shared__ __attribute__((aligned(16))) double Bs[2][SYK * SYLD];  // W[J rows]
  int I = 0, rem = blockIdx.x;
  while (rem > I) {
    rem -= I + 1;
    ++I;
  }
  const int J = rem;
  const int I0 = I * SYT, J0 = J * SYT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;  // wave's 64 x 64 quadrant: I rows wm.., J rows wn..
  const int lr = tid & (SYT - 1), lk = tid >> 7;      // loader: row lr, columns lk + 2q
  dbl4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  // the next chunk's operands: loads from clamped addresses, issued together and consumed (masked,
  // scaled) only at the LDS store after the current chunk's MFMAs — a predicated load compiled into a
  // branch with a wait inside, exposing 8 memory latencies per chunk (SQ_WAIT_ANY 55 % of wave cycles)
  double ra[8], rb[8], rd[8];
  auto gload = [&](int kb) {
    const int ri = min(I0 + lr, m - 1), rj = min(J0 + lr, m - 1);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kc = min(kb + lk + 2 * q, k1 - 1);
      const int64_t col = (int64_t)kc * m;
      ra[q] = W[ri + col];
      rb[q] = W[rj + col];
      rd[q] = dinv[kc];
    }
  };
  auto sstore = [&](int kb, int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool ok = kb + lk + 2 * q < k1;
      As[buf][(lk + 2 * q) * SYLD + lr] = (ok && I0 + lr < m) ? ra[q] * rd[q] : 0.0;
      Bs[buf][(lk + 2 * q) * SYLD + lr] = (ok && J0 + lr < m) ? rb[q] : 0.0;
    }
  };
  gload(k0);
  sstore(k0, 0);
  __syncthreads();
  int buf = 0;
  for (int kb = k0; kb < k1; kb += SYK) {
    const bool more = kb + SYK < k1;
    if (more) gload(kb + SYK);
#pragma unroll
    for (int k4 = 0; k4 < SYK / 4; ++k4) {
      const int kk = 4 * k4 + (lane >> 4);
      double fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        fa[t] = Bs[buf][kk * SYLD + wn + 16 * t + (lane & 15)];  // A operand: W_J rows (m)
        fb[t] = As[buf][kk * SYLD + wm + 16 * t + (lane & 15)];  // B operand: (W D^-1)_I rows (n)
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    if (more) {
      sstore(kb + SYK, buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  // acc[a][b][g]: row i = I0 + wm + 16 b + (lane & 15), column j = J0 + wn + 16 a + (lane >> 4) + 4 g.
  // F read-modify-written 16 entries at a time: the reads from clamped addresses, all in flight
  // together, the writes masked (a masked read-modify-write per entry compiled into a branch with a
  // wait inside: 64 serial memory latencies per lane)
  int gi[4], gj[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b) gi[b] = gpos[min(I0 + wm + 16 * b + (lane & 15), m - 1)];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int g = 0; g < 4; ++g) gj[a][g] = gpos[min(J0 + wn + 16 * a + (lane >> 4) + 4 * g, m - 1)];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    double fv[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) fv[b][g] = F[gi[b] + (int64_t)gj[a][g] * ld];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = I0 + wm + 16 * b + (lane & 15), j = J0 + wn + 16 * a + (lane >> 4) + 4 * g;
        if (i < m && j <= i) F[gi[b] + (int64_t)gj[a][g] * ld] = fv[b][g] - acc[a][b][g];
      }
  }
}

// Trailing update of a big front's panel group on 128 x 128 lower tiles (the group's K = 64 kpan columns,
// tiles relative to the group's end c0): C -= (L_I D) L_J^T, four waves x 64 x 64 quadrants of f64 MFMA
// 16x16x4, K-chunks of 16 double-buffered through LDS (k_lb_syrk's engine on the front's own columns).
// A 128-tile reads 2 x 128 K doubles per 2 x 128^2 K flops — twice k_big_update's 64-tile arithmetic
// intensity, on the update that carries ~90 % of neos' factorisation flops.
// Split K (nsplit > 1, launches of few tiles: one workgroup per CU ran each tile's K chain with its
// loads exposed, ~67 us per tile whatever the launch size on neos): workgroup blockIdx.x takes part
// blockIdx.x % nsplit of tile blockIdx.x / nsplit's K range (16-column chunks), stores its partial
// product write-through (psum), and the last part to take the tile's ticket sums the partials in part
// order (fixed: bitwise reproducible), then runs the epilogue (and the lookahead of tile (0, 0)).
constexpr int UPD_PART = 4 * 4 * 4 * NT;  // partial product doubles of one part (acc of every thread)
constexpr int U128_LDS = 4 * SYK * SYLD;   // As[2] then Bs[2]
// acc[a][b] += sum_{k in [k0, k1)} (L D)[I0 + rows, k] L[J0 + cols, k] on a 128 x 128 tile of front F (ld r):
// four waves x 64 x 64 quadrants of f64 MFMA 16x16x4, K-chunks of 16 double-buffered through LDS (AB)
template <bool SC>
__device__ __forceinline__ void upd128_gemm(const double* __restrict__ F, const double* __restrict__ D, int f0, int r,
                                            int I0, int J0, int k0, int k1, double* AB, dbl4 (&acc)[4][4]) {
  double (*As)[SYK * SYLD] = reinterpret_cast<double (*)[SYK * SYLD]>(AB);           // (L D)[I rows]
  double (*Bs)[SYK * SYLD] = reinterpret_cast<double (*)[SYK * SYLD]>(AB + 2 * SYK * SYLD);  // L[J rows]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
  const int lr = tid & (SYT - 1), lk = tid >> 7;
  double ra[8], rb[8], rd[8];
  const int ri = min(I0 + lr, r - 1), rj = min(J0 + lr, r - 1);
  auto gload = [&](int kb) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kc = min(kb + lk + 2 * q, k1 - 1);
      const int64_t col = (int64_t)kc * r;
      ra[q] = ldF<SC>(F + ri + col);
      rb[q] = ldF<SC>(F + rj + col);
      rd[q] = ldF<SC>(D + f0 + kc);
    }
  };
  auto sstore = [&](int kb, int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool ok = kb + lk + 2 * q < k1;
      As[buf][(lk + 2 * q) * SYLD + lr] = (ok && I0 + lr < r) ? ra[q] * rd[q] : 0.0;
      Bs[buf][(lk + 2 * q) * SYLD + lr] = (ok && J0 + lr < r) ? rb[q] : 0.0;
    }
  };
  if (k0 >= k1) return;  // (a split part past the group's K has nothing to multiply)
  gload(k0);
  sstore(k0, 0);
  __syncthreads();
  int buf = 0;
  for (int kb = k0; kb < k1; kb += SYK) {
    const bool more = kb + SYK < k1;
    if (more) gload(kb + SYK);
#pragma unroll
    for (int k4 = 0; k4 < SYK / 4; ++k4) {
      const int kk = 4 * k4 + (lane >> 4);
      double fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        fa[t] = Bs[buf][kk * SYLD + wn + 16 * t + (lane & 15)];
        fb[t] = As[buf][kk * SYLD + wm + 16 * t + (lane & 15)];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    if (more) {
      sstore(kb + SYK, buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
}

__global__ __launch_bounds__(NT, 2) void k_big_upd128(FrontTab T, const int32_t* __restrict__ list, int step, int kpan,
                                                     double* __restrict__ arena, double* __restrict__ D,
                                                     double* __restrict__ Mbuf, LDLStatus* st, double tol,
                                                     int nsplit, double* __restrict__ psum, int32_t* ptick) {
  // one buffer: As[2] then Bs[2]; after the MFMAs task (0, 0) reuses it for the lookahead diagonal block
  __shared__ __attribute__((aligned(16))) double AB[U128_LDS];
  __shared__ int s_last;
  static_assert(64 * LDA + 4 * 16 * LDM + 64 <= U128_LDS, "lookahead diagonal block aliases As / Bs");
  const int tile = blockIdx.x / nsplit, part = blockIdx.x - tile * nsplit;
  const int2 task = reinterpret_cast<const int2*>(list)[tile];
  const int s = task.x, tij = task.y;
  const int ti = tij & 0xffff, tj = (tij >> 16) & 0x7fff;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int g0 = (step / kpan) * kpan;
  const int kg0 = 64 * g0, k1g = min(64 * (g0 + kpan), w);  // K range = the group's columns
  const int c0 = k1g;
  const int kps = ((k1g - kg0 + nsplit - 1) / nsplit + SYK - 1) / SYK * SYK;  // this part's K columns
  const int k0 = min(kg0 + part * kps, k1g), k1 = min(k0 + kps, k1g);
  const int I0 = c0 + ti * SYT, J0 = c0 + tj * SYT;
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
  dbl4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  upd128_gemm<false>(F, D, f0, r, I0, J0, k0, k1, AB, acc);
  if (nsplit > 1) {  // the tile's parts: partials write-through, the last part sums them in part order
    double* __restrict__ mine = psum + ((int64_t)tile * nsplit + part) * UPD_PART;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) st_sc1(mine + ((a * 4 + b) * 4 + g) * NT + tid, acc[a][b][g]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      s_last = __hip_atomic_fetch_add(ptick + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) ptick[tile] = 0;  // every part has taken its ticket: ready for the next launch
    // the sum in part order, every part (this one's too) read back: 8 values of every part per round,
    // all 32 loads in flight (unconditional, the part index clamped; a load per value in a runtime
    // loop compiled to one memory round trip per load)
    const double* __restrict__ all = psum + (int64_t)tile * nsplit * UPD_PART;
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      double pv[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double* pq = all + (int64_t)min(q, nsplit - 1) * UPD_PART + tid;
#pragma unroll
        for (int u = 0; u < 8; ++u) pv[q][u] = ld_sc1(pq + (h * 8 + u) * NT);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = h * 8 + u, a = e >> 4, b = (e >> 2) & 3, g = e & 3;
        double v = pv[0][u];
#pragma unroll
        for (int q = 1; q < 4; ++q) v = (q < nsplit) ? v + pv[q][u] : v;
        acc[a][b][g] = v;
      }
    }
  }
  // acc[a][b][g]: row i = I0 + wm + 16 b + (lane & 15), column j = J0 + wn + 16 a + (lane >> 4) + 4 g;
  // the C reads of a column block from clamped addresses, all in flight, the writes masked
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    double fv[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = min(I0 + wm + 16 * b + (lane & 15), r - 1), j = min(J0 + wn + 16 * a + (lane >> 4) + 4 * g, r - 1);
        fv[b][g] = F[i + (int64_t)j * r];
      }
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = I0 + wm + 16 * b + (lane & 15), j = J0 + wn + 16 * a + (lane >> 4) + 4 * g;
        if (i < r && j <= i) F[i + (int64_t)j * r] = fv[b][g] - acc[a][b][g];
        acc[a][b][g] = fv[b][g] - acc[a][b][g];  // kept for the lookahead diagonal block below
      }
  }
  // lookahead: task (0, 0) holds the next panel's diagonal tile (rows / columns [c0, c0 + 64): wave 0's
  // quadrant), final now — the group's trailing update is its last before that panel
  if (ti == 0 && tj == 0 && 64 * (step + 1) == c0 && big_next_diag(T, s, step)) {
    double* A64 = AB;
    double* Ms = AB + 64 * LDA;
    double* Dl = Ms + 4 * 16 * LDM;
    const int kw = min(64, w - c0);
    __syncthreads();  // every wave's last MFMA operand read
    big_diag_prepare(A64, kw);
    __syncthreads();
    if (wv == 0) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int i = 16 * b + (lane & 15), j = 16 * a + (lane >> 4) + 4 * g;
            if (i < kw && j < kw && i >= j) A64[i + j * LDA] = acc[a][b][g];
          }
    }
    __syncthreads();
    big_diag_tail(T, s, step + 1, A64, Ms, Dl, arena, D, Mbuf + (int64_t)T.bigslot[s] * 4096, st, tol);
  }
}

// All big fronts of a level in ONE launch (r6): their 64-column panels' diagonal blocks, trsm tiles,
// local updates and trailing updates as tasks of a dependency-driven persistent kernel, instead of a
// k_big_diag / k_big_trsm / k_big_update / k_big_upd128 launch per panel step and kind (neos: ~400
// launches per factorisation, each boundary a ~4.6 us gap, and the panel chain diag -> trsm -> update
// serialised by them).  Per panel group G (kpan panels, columns [64 g0, gend)):
//   chain(G):  trsm tiles (kind 0) and local updates inside the group (kind 1, as k_big_update mode 0;
//              task (0, 0) factorises the next panel's diagonal block);
//   feed(G):   the trailing update of the next group's columns [gend, gend + 64 kpan), 64 x 64 tiles with
//              K = the group (kind 1, k_big_update's trailing mode; tile (0, 0) factorises the next
//              group's first diagonal block);
//   bulk(G):   the rest of the trailing matrix, 128 x 128 tiles (kind 2, k_big_upd128's engine, K unsplit).
// Tickets run chain(0) feed(0) chain(1) bulk(0) feed(1) chain(2) bulk(1) ... : the next group's panel
// chain only needs the feed tiles, so it runs while the previous group's bulk update occupies the chip.
// A task's dependencies (host-built, LDLSolver::build_schedules) are the last earlier writers of every
// 64 x 64 block of the front it reads or read-modify-writes: all earlier tickets (a workgroup waits only
// for tickets taken by running workgroups: no deadlock whatever the residency).  Every handed-off value
// is stored write-through (sc1) and drained before the task's flag, every load of one is sc1; each
// panel's M_K blocks go to a slot of their own (Mch, per front and panel).  Same operands and MFMA order
// as the per-step kernels with K unsplit (MADIPM_UPD_SPLIT=0): the same factor bit for bit.
// the task bodies as calls (one register allocation per body, not the union of four inlined ones)
__device__ __attribute__((noinline)) void dag_trsm(const FrontTab& T, int s, int step, int rt, double* arena,
                                                   const double* D, const double* M, double* sm) {
  trsm_body<true>(T, s, step, rt, arena, D, M, sm);
}
__device__ __attribute__((noinline)) void dag_update(const FrontTab& T, int s, int step, int kpan, int tij, double* arena,
                                                     double* D, double* Mnext, LDLStatus* st, double tol, double* sm) {
  update_body<true>(T, s, step, kpan, tij, arena, D, Mnext, st, tol, sm);
}
__device__ __attribute__((noinline)) void dag_diag(const FrontTab& T, int s, double* arena, double* D, double* M,
                                                   LDLStatus* st, double tol, double* sm) {
  diag_body<true>(T, s, 0, arena, D, M, st, tol, sm);
}
__device__ __attribute__((noinline)) void dag_bulk(const FrontTab& T, int s, int step, int kpan, int item, double* arena,
                                                   const double* D, double* sm) {
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int g0 = (step / kpan) * kpan, gend = min(64 * (g0 + kpan), w), cb = gend + 64 * kpan;
  const int I0 = cb + 128 * (item & 0xffff), J0 = cb + 128 * ((item >> 16) & 0x7fff);
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63;
  dbl4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  upd128_gemm<true>(F, D, f0, r, I0, J0, 64 * g0, gend, sm, acc);
  const int wv = tid >> 6, wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    double fv[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = min(I0 + wm + 16 * b + (lane & 15), r - 1), j = min(J0 + wn + 16 * a + (lane >> 4) + 4 * g, r - 1);
        fv[b][g] = ldF<true>(F + i + (int64_t)j * r);
      }
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = I0 + wm + 16 * b + (lane & 15), j = J0 + wn + 16 * a + (lane >> 4) + 4 * g;
        if (i < r && j <= i) stF<true>(F + i + (int64_t)j * r, fv[b][g] - acc[a][b][g]);
      }
  }
}

struct DagTask {
  int32_t s, step, item, kind;  // 0 trsm (item: row tile), 1 64-tile update (ti | tj << 16, bit 31: trailing),
                                // 2 128-tile trailing update (I | J << 16), 3 first diagonal block
};
constexpr int DAG_LDS = UPD_LDS > TRSM_LDS ? (UPD_LDS > U128_LDS ? UPD_LDS : U128_LDS) : (TRSM_LDS > U128_LDS ? TRSM_LDS : U128_LDS);
static_assert(DAG_LDS * 8 <= 80 * 1024 && DIAG_LDS <= DAG_LDS, "two k_big_dag workgroups per CU");
__global__ __launch_bounds__(NT, 2) void k_big_dag(FrontTab T, const DagTask* __restrict__ tasks, const int32_t* __restrict__ dptr,
                                                   const int32_t* __restrict__ dlist, int ntask, int32_t* flags, int epoch,
                                                   int32_t* counter, int kpan, double* __restrict__ arena,
                                                   double* __restrict__ D, double* __restrict__ Mch,
                                                   const int64_t* __restrict__ mslot, LDLStatus* st, double tol,
                                                   int32_t* err, int64_t* dbg) {
  // 80 KB: two workgroups per CU (the ticket word borrows the first double: read before any task uses it)
  __shared__ __attribute__((aligned(16))) double sm[DAG_LDS];
  int* s_t = reinterpret_cast<int*>(sm);
  const int tid = threadIdx.x, lane = tid & 63;
  for (;;) {
    __syncthreads();  // the previous task's LDS reads
    if (tid == 0) *s_t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int t = *s_t;
    __syncthreads();  // every wave has the ticket before a task overwrites the word
    if (t >= ntask) break;
    const DagTask tk = tasks[t];
    if (dbg && tid == 0) dbg[4 * t] = wall_clock64();
    if (tid < 64) {  // wave 0 polls the dependencies' flags, 64 at a time
      const int q0 = dptr[t], q1 = dptr[t + 1];
      for (int q = q0; q < q1; q += 64) {
        const int d = q + lane < q1 ? dlist[q + lane] : -1;
        int spins = 0;
        for (;;) {
          const bool ok = d < 0 || __hip_atomic_load(flags + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          ++spins;
          // bounded: a lost hand-off raises the sticky error, and once raised no later wait spins
          // (the launch drains in milliseconds, the factor is reported invalid)
          if (spins > (1 << 25) ||
              ((spins & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            if (lane == 0) atomicOr(err, kErrHandoff);
            break;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only (sc1 loads follow)
    }
    __syncthreads();
    if (dbg && tid == 0) dbg[4 * t + 1] = wall_clock64();
    double* Mp = Mch + mslot[tk.s] * BIG_MSZ;  // the front's per-panel M_K slots
    // the panel chain's tasks (latency-bound, on the critical path) issue ahead of a co-resident 128-tile
    // update's waves (MFMA-bound, off it)
    if (tk.kind == 2)
      __builtin_amdgcn_s_setprio(0);
    else
      __builtin_amdgcn_s_setprio(2);
    if (tk.kind == 0)
      dag_trsm(T, tk.s, tk.step, tk.item, arena, D, Mp + (int64_t)tk.step * BIG_MSZ, sm);
    else if (tk.kind == 1)
      dag_update(T, tk.s, tk.step, kpan, tk.item, arena, D, Mp + (int64_t)(tk.step + 1) * BIG_MSZ, st, tol, sm);
    else if (tk.kind == 3)
      dag_diag(T, tk.s, arena, D, Mp, st, tol, sm);
    else  // 128 x 128 trailing tile, columns past the feed tiles: rows / columns cb + 128 (I, J)
      dag_bulk(T, tk.s, tk.step, kpan, tk.item, arena, D, sm);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's sc1 stores drained
    __syncthreads();
    if (tid == 0) __hip_atomic_store(flags + t, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dbg && tid == 0) {
      dbg[4 * t + 2] = wall_clock64();
      dbg[4 * t + 3] = blockIdx.x;
    }
  }
  if (tid == 0 && atomicAdd(counter + 1, 1) == (int)gridDim.x - 1) {  // last one out: reset the tickets
    counter[0] = 0;
    counter[1] = 0;
  }
}

// forward: s_j = b(c_j) / d_j, t = W s (two passes: column chunks of LBF_COLS -> partials, then the
// chunks summed in order), the group's update vector = -t; the members' forward values are b(c_j)
constexpr int LBF_COLS = 256;
constexpr int LB_KCHUNK = 2048;  // members per SYRK launch (m x 2048 doubles of W stay cache-resident)
__global__ __launch_bounds__(NT) void k_lb_fwd1(const double* __restrict__ W, const double* __restrict__ dlb,
                                                const int32_t* __restrict__ mem, const int32_t* __restrict__ perm,
                                                int m, int n, int64_t mem0, const double* __restrict__ b,
                                                double* __restrict__ xi, double* __restrict__ part) {
  __shared__ double sj[LBF_COLS];
  const int c0 = blockIdx.y * LBF_COLS;
  const int nc = min(LBF_COLS, n - c0);
  if (threadIdx.x < nc) {
    const int j = c0 + threadIdx.x;
    const int col = mem[mem0 + j];
    const double bj = b[perm[col]];
    sj[threadIdx.x] = bj / dlb[mem0 + j];
    if (blockIdx.x == 0) xi[col] = bj;
  }
  __syncthreads();
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= m) return;
  const double* __restrict__ Wc = W + (int64_t)c0 * m + i;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int j = 0;
  for (; j + 3 < nc; j += 4) {
    a0 = fma(Wc[(int64_t)j * m], sj[j], a0);
    a1 = fma(Wc[(int64_t)(j + 1) * m], sj[j + 1], a1);
    a2 = fma(Wc[(int64_t)(j + 2) * m], sj[j + 2], a2);
    a3 = fma(Wc[(int64_t)(j + 3) * m], sj[j + 3], a3);
  }
  for (; j < nc; ++j) a0 = fma(Wc[(int64_t)j * m], sj[j], a0);
  part[(int64_t)blockIdx.y * m + i] = (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(NT) void k_lb_fwd2(const double* __restrict__ part, int m, int nchunk,
                                                double* __restrict__ uv) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= m) return;
  double v = 0.0;
  for (int c = 0; c < nchunk; ++c) v += part[(int64_t)c * m + i];
  uv[i] = -v;
}

// backward: x_j = (y_j - W(:, j)^T x_P(gpos)) / d_j, one wave per member column
__global__ __launch_bounds__(NT) void k_lb_bwd(const double* __restrict__ W, const double* __restrict__ dlb,
                                               const int32_t* __restrict__ mem, const int32_t* __restrict__ perm,
                                               const int32_t* __restrict__ xrow, int m, int n, int64_t mem0,
                                               double* __restrict__ xi, double* __restrict__ out) {
  const int j = blockIdx.x * (NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= n) return;
  const double* __restrict__ Wc = W + (int64_t)j * m;
  double a = 0.0;
  for (int k = lane; k < m; k += 64) a = fma(Wc[k], xi[xrow[k]], a);
  a = wave_sum(a);
  if (lane == 0) {
    const int col = mem[mem0 + j];
    const double x = (xi[col] - a) / dlb[mem0 + j];
    xi[col] = x;
    out[perm[col]] = x;
  }
}

// ------------------------------------------------------------------ solves
// Multifrontal forward solve per front:  v = [b(own cols); 0] + extend-add of the children's update
// vectors;  v[0:w] <- L11^{-1} v[0:w];  v[w:] -= L21 v[0:w];  own part -> xi, rest -> update vector.
// Backward:  v[0:w] = D^{-1} xi(own) - L21^T x(below rows);  x_own = L11^{-T} v[0:w].
//  * fronts with r <= 128: one WAVE per front (wave-synchronous, v in LDS), 4 fronts per workgroup;
//  * bigger fronts: dependency-driven persistent kernels.  Tasks = 64-row blocks (forward) or 64-column
//    panels (backward), dequeued in dependency order from one atomic counter; block i waits for the
//    published x of panels < i (release/acquire flags tagged with a per-solve epoch), so the whole
//    level is ONE launch and the panel GEMVs of different blocks overlap.
constexpr int SW = 4;  // waves (= small fronts) per workgroup


// Small-front solves (32 < r <= 128): one WORKGROUP per front.  The whole workgroup first copies the
// r x w L panel into LDS with every load in flight at once (the panel is contiguous in HBM, ld r; in
// LDS ld = r | 1 so that column-strided lane accesses of the backward solve are conflict-free), then
// wave 0 runs the substitution from LDS: lane l holds rows (forward) or pivot columns (backward) l and
// l + 64 in registers, the value of row/column t is broadcast with readlane.  Turning the panel read
// from a latency chain into one bandwidth burst is what bounds these levels.
__device__ __forceinline__ double bcast3(const double (&v)[3], int t) {
  return (t < 64) ? readlane_f64(v[0], t) : ((t < 128) ? readlane_f64(v[1], t - 64) : readlane_f64(v[2], t - 128));
}

// Blocked substitutions of ONE wave on a panel staged in LDS (col-major, ld rl), rows / columns
// i = lane + 64 h (h < 3) held in v[h].  Pivots are taken 16 at a time: the block's L entries of
// every row are loaded into registers up front (one LDS latency per block), then the 16-step
// dependency chain touches only v[HB] (readlane broadcast + one fma per step), and the rows of the
// other thirds get the block's contribution as 16 independent fmas.  HB (the third holding the
// block) is a template parameter so every register index is static.
template <int HB>
__device__ __forceinline__ void fwd_block16(double (&v)[3], const double* Ls, int rl, int r, int t0, int kb, int lane) {
  double lb[3][16];
#pragma unroll
  for (int h = HB; h < 3; ++h) {
    const int i = lane + 64 * h;
    const int ic = min(i, r - 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) lb[h][k] = (k < kb && i > t0 + k && i < r) ? Ls[ic + (t0 + k) * rl] : 0.0;
  }
  double xs[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    xs[k] = 0.0;
    if (k < kb) {  // wave-uniform
      xs[k] = readlane_f64(v[HB], (t0 & 63) + k);
      v[HB] = fma(-lb[HB][k], xs[k], v[HB]);
    }
  }
#pragma unroll
  for (int h = HB + 1; h < 3; ++h)
#pragma unroll
    for (int k = 0; k < 16; ++k) v[h] = fma(-lb[h][k], xs[k], v[h]);
}

// forward: v[i] -= L(i, t) v[t] for i > t, t < w
__device__ __forceinline__ void fwd_subst16(double (&v)[3], const double* Ls, int rl, int r, int w, int lane) {
  for (int t0 = 0; t0 < w; t0 += 16) {
    const int kb = min(16, w - t0);
    if (t0 < 64)
      fwd_block16<0>(v, Ls, rl, r, t0, kb, lane);
    else if (t0 < 128)
      fwd_block16<1>(v, Ls, rl, r, t0, kb, lane);
    else
      fwd_block16<2>(v, Ls, rl, r, t0, kb, lane);
  }
}

template <int HB>
__device__ __forceinline__ void bwd_block16(double (&v)[3], const double* Ls, int rl, int w, int t0, int kb, int lane) {
  double lb[HB + 1][16];
#pragma unroll
  for (int h = 0; h <= HB; ++h) {
    const int j = lane + 64 * h;
    const int jc = min(j, w - 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) lb[h][k] = (k < kb && j < t0 + k) ? Ls[(t0 + k) + jc * rl] : 0.0;
  }
  double xs[16];
#pragma unroll
  for (int k = 15; k >= 0; --k) {
    xs[k] = 0.0;
    if (k < kb) {  // wave-uniform
      xs[k] = readlane_f64(v[HB], (t0 & 63) + k);
      v[HB] = fma(-lb[HB][k], xs[k], v[HB]);
    }
  }
#pragma unroll
  for (int h = 0; h < HB; ++h)
#pragma unroll
    for (int k = 0; k < 16; ++k) v[h] = fma(-lb[h][k], xs[k], v[h]);
}

// backward (transposed): v[j] -= L(t, j) v[t] for j < t, t = w-1 .. 1
__device__ __forceinline__ void bwd_subst16(double (&v)[3], const double* Ls, int rl, int w, int lane) {
  for (int t0 = ((w - 1) >> 4) << 4; t0 >= 0; t0 -= 16) {
    const int kb = min(16, w - t0);
    if (t0 < 64)
      bwd_block16<0>(v, Ls, rl, w, t0, kb, lane);
    else if (t0 < 128)
      bwd_block16<1>(v, Ls, rl, w, t0, kb, lane);
    else
      bwd_block16<2>(v, Ls, rl, w, t0, kb, lane);
  }
}

// r <= SMALL_SOLVE_MAX rows (3 per lane of wave 0), panel r x w staged in LDS (ld r | 1)
constexpr int SMALL_SOLVE_MAX = 192;

__global__ __launch_bounds__(NT) void k_fwd_small(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                  const double* __restrict__ arena, const double* __restrict__ b,
                                                  double* __restrict__ xi, double* __restrict__ uvec) {
  extern __shared__ __attribute__((aligned(16))) double Ls[];
  __shared__ double v0s[SMALL_SOLVE_MAX];
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int rl = r | 1;
  stage_panel(arena + T.l_off[s], Ls, r, w, rl);
  const int lane = threadIdx.x & 63;
  // initial vector (own b + children's update vectors): all 256 threads, rows strided, each row's
  // gather list walked with 4 loads in flight
  for (int i = threadIdx.x; i < r; i += NT) {
    const int64_t e = T.row_ptr[s] + i;
    const int64_t p1 = T.sv_ptr[e + 1];
    int64_t p = T.sv_ptr[e];
    double vi = 0.0;
    for (; p + 3 < p1; p += 4) {
      const int64_t q0 = T.sv_src[p], q1 = T.sv_src[p + 1], q2 = T.sv_src[p + 2], q3 = T.sv_src[p + 3];
      vi += (uvec[q0] + uvec[q1]) + (uvec[q2] + uvec[q3]);
    }
    for (; p < p1; ++p) vi += uvec[T.sv_src[p]];
    v0s[i] = vi + fwd_init(T, s, i, w, f0, b);
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  double v[3];
  int ci[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int i = lane + 64 * h;
    v[h] = (i < r) ? v0s[i] : 0.0;
    ci[h] = min(i, r - 1);
  }
  fwd_subst16(v, Ls, rl, r, w, lane);  // v[i] -= L(i, t) v[t] for i > t, t < w
  (void)ci;
  double* __restrict__ uo = uvec + T.uvec_off[s];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int i = lane + 64 * h;
    if (i < w)
      xi[f0 + i] = v[h];
    else if (i < r)
      uo[i - w] = v[h];
  }
}

__global__ __launch_bounds__(NT) void k_bwd_small(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                  const double* __restrict__ arena, const double* __restrict__ D,
                                                  double* __restrict__ xi, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double Ls[];
  __shared__ double xbs[SMALL_SOLVE_MAX];
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int rl = r | 1;
  stage_panel(arena + T.l_off[s], Ls, r, w, rl);
  const int lane = threadIdx.x & 63;
  const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
  const int nb = r - w;
  // x of the rows below the pivot block (ancestors: final), all threads
  for (int k = threadIdx.x; k < nb; k += NT) xbs[k] = xi[rows[w + k]];
  double own[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int j = lane + 64 * h;
    own[h] = (threadIdx.x < 64 && j < w) ? xi[f0 + j] / D[f0 + j] : 0.0;
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  int cj[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) cj[h] = min(lane + 64 * h, w - 1);
  // v[j] = x_j / d_j - sum_{i >= w} L(i, j) x_i
  double acc[3] = {0.0, 0.0, 0.0};
  for (int k8 = 0; k8 < nb; k8 += 8) {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = k8 + kk;
      if (k < nb) {
        const double x = xbs[k];
#pragma unroll
        for (int h = 0; h < 3; ++h) acc[h] = fma(Ls[(w + k) + cj[h] * rl], x, acc[h]);
      }
    }
  }
  double v[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) v[h] = (lane + 64 * h < w) ? own[h] - acc[h] : 0.0;
  bwd_subst16(v, Ls, rl, w, lane);  // for t = w-1 .. 1: v[j] -= L(t, j) v[t] for j < t
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int j = lane + 64 * h;
    if (j < w) {
      xi[f0 + j] = v[h];
      if (T.wout[s]) out[T.perm[f0 + j]] = v[h];
    }
  }
}

// Fronts with r <= 32 (the leaf level has ~10^5): HALF a wave per front, 8 fronts per workgroup;
// lane l & 31 holds row / pivot column l & 31, values exchanged with 32-wide shuffles.
__global__ __launch_bounds__(NT) void k_fwd_tiny(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                 const double* __restrict__ arena, const double* __restrict__ b,
                                                 double* __restrict__ xi, double* __restrict__ uvec) {
  const int lane = threadIdx.x & 63, lr = lane & 31;
  const int q = (blockIdx.x * SW + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool live = q < nf;
  const int s = fronts[live ? q : nf - 1];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const double* __restrict__ L = arena + T.l_off[s];
  double v = 0.0;
  if (lr < r) {
    v = fwd_init(T, s, lr, w, f0, b);
    const int64_t e = T.row_ptr[s] + lr;
    const int64_t p1 = T.sv_ptr[e + 1];
    for (int64_t p = T.sv_ptr[e]; p < p1; ++p) v += uvec[T.sv_src[p]];
  }
  const int wmax = max(__builtin_amdgcn_readlane(w, 0), __builtin_amdgcn_readlane(w, 32));
  const int cl = min(lr, r - 1);
  for (int t4 = 0; t4 < wmax; t4 += 4) {
    double c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = L[cl + (int64_t)min(t4 + k, w - 1) * r];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = t4 + k;
      const double xt = __shfl(v, t & 31, 32);
      v = fma((t < w && lr > t) ? -c[k] : 0.0, xt, v);
    }
  }
  if (live && lr < r) {
    if (lr < w)
      xi[f0 + lr] = v;
    else
      *uvec_dst(T, s, lr - w, uvec) = v;
  }
}

__global__ __launch_bounds__(NT) void k_bwd_tiny(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                 const double* __restrict__ arena, const double* __restrict__ D,
                                                 double* __restrict__ xi, double* __restrict__ out) {
  const int lane = threadIdx.x & 63, lr = lane & 31;
  const int q = (blockIdx.x * SW + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool live = q < nf;
  const int s = fronts[live ? q : nf - 1];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const double* __restrict__ L = arena + T.l_off[s];
  const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
  const int nb = r - w;
  const double xb = (lr < nb) ? xi[rows[w + lr]] : 0.0;  // x of below row w + lr (final)
  const int cj = min(lr, w - 1);
  const int nbmax = max(__builtin_amdgcn_readlane(nb, 0), __builtin_amdgcn_readlane(nb, 32));
  double acc = 0.0;
  for (int k4 = 0; k4 < nbmax; k4 += 4) {
    double c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = L[min(w + k4 + k, r - 1) + (int64_t)cj * r];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double x = __shfl(xb, (k4 + k) & 31, 32);
      acc = fma((k4 + k < nb) ? c[k] : 0.0, x, acc);
    }
  }
  double v = (lr < w) ? xi[f0 + lr] / D[f0 + lr] - acc : 0.0;
  const int wmax = max(__builtin_amdgcn_readlane(w, 0), __builtin_amdgcn_readlane(w, 32));
  for (int t4 = wmax - 1; t4 > 0; t4 -= 4) {
    double c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = L[min(max(t4 - k, 0), w - 1) + (int64_t)cj * r];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = t4 - k;
      const double xt = __shfl(v, max(t, 0) & 31, 32);
      v = fma((t > 0 && t < w && lr < t) ? -c[k] : 0.0, xt, v);
    }
  }
  if (live && lr < w) {
    xi[f0 + lr] = v;
    if (T.wout[s]) out[T.perm[f0 + lr]] = v;
  }
}

// initial forward vector of a big front (own b entries + children's update vectors), in HBM;
// task = (front, chunk of GAT_ROWS rows), GAT_G lanes per row stride the row's gather list (children
// in list order per lane, lanes combined by a fixed butterfly: deterministic)
constexpr int GAT_G = 8, GAT_ROWS = NT / GAT_G;
__global__ __launch_bounds__(NT) void k_fwd_gather(FrontTab T, const int32_t* __restrict__ list,
                                                   const double* __restrict__ b, const double* __restrict__ uvec,
                                                   double* __restrict__ vwork) {
  int s, chunk;
  task_of(list, s, chunk);
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int i = chunk * GAT_ROWS + threadIdx.x / GAT_G, gl = threadIdx.x & (GAT_G - 1);
  if (i >= r) return;  // whole groups leave together
  const int64_t e = T.row_ptr[s] + i;
  const int64_t p1 = T.sv_ptr[e + 1];
  double vi = 0.0;
  for (int64_t p = T.sv_ptr[e] + gl; p < p1; p += GAT_G) vi += uvec[T.sv_src[p]];
#pragma unroll
  for (int o = GAT_G / 2; o > 0; o >>= 1) vi += __shfl_xor(vi, o, GAT_G);
  if (gl == 0) vwork[e] = vi + fwd_init(T, s, i, w, f0, b);
}

__device__ __forceinline__ bool wait_flag(int32_t* f, int epoch, int32_t* err) {
  int spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 25)) {
      atomicOr(err, kErrHandoff);
      return false;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

__device__ __forceinline__ void publish_flag(int32_t* f, int epoch) {
  // every storing wave drained, then ONE release + relaxed flag store (Guideline 16 R1)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Triangular solves of a 64-pivot diagonal block by one wave, 16 pivots per batch: the batch's L
// entries are loaded first, then each pivot's value is broadcast by v_readlane (an SGPR, a few cycles)
// — a __shfl (ds_bpermute) per pivot put an LDS round trip on the chain: ~5 us per 64-pivot block.
// forward: a[lane] -= L(lane, t) a[t] for t < lane, t < kw; L(i, t) at Ld[t * 65 + i]
__device__ __forceinline__ double tri_fwd64(double a, const double* Ld, int kw, int lane) {
  for (int t0 = 0; t0 < kw; t0 += 16) {
    double lb[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) lb[k] = Ld[min(t0 + k, 63) * 65 + lane];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int tt = t0 + k;
      const double xt = readlane_f64(a, min(tt, 63));
      const double na = a - lb[k] * xt;
      a = (lane > tt && tt < kw) ? na : a;
    }
  }
  return a;
}
// backward (transposed): a[lane] -= L(t, lane) a[t] for t > lane, t < kw, from t = kw - 1 down;
// L(t, j) at Ld[t * 65 + j]
__device__ __forceinline__ double tri_bwd64(double a, const double* Ld, int kw, int lane) {
  for (int t1 = kw - 1; t1 > 0; t1 -= 16) {
    double lb[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) lb[k] = Ld[max(t1 - k, 0) * 65 + lane];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int tt = t1 - k;
      const double xt = readlane_f64(a, max(tt, 0));
      const double na = a - lb[k] * xt;
      a = (lane < tt && tt > 0) ? na : a;
    }
  }
  return a;
}

// Panel solutions handed between the big-front solve tasks as self-validating 8-byte words (the LL
// idea): value halves each stored with the solve's epoch in the upper 32 bits by single-copy-atomic
// 8-byte stores, so a consumer lane polls its two words until both carry the epoch — the data is the
// flag: no release fence and drain before a flag store, no acquire and second round trip after it.
__device__ __forceinline__ void ll_put(uint64_t* w, double v, int epoch) {
  const uint64_t tag = (uint64_t)(uint32_t)epoch << 32;
  __hip_atomic_store(w, tag | (uint32_t)__double2loint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(w + 1, tag | (uint32_t)__double2hiint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ll_get(const uint64_t* w, int epoch, int32_t* err) {
  uint64_t a, b;
  int spins = 0;
  for (;;) {
    a = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(a >> 32) == (uint32_t)epoch && (uint32_t)(b >> 32) == (uint32_t)epoch) break;
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 25)) {
      atomicOr(err, kErrHandoff);
      break;
    }
  }
  return __hiloint2double((int)(uint32_t)b, (int)(uint32_t)a);
}

// Forward, big fronts: task = (front, 64-row block i).  acc(rows) = v(rows) - sum_{panels p < i} L(rows,p) x_p,
// then (pivot block) x_i = L_ii^{-1} acc, handed to the later row blocks through T.xll (ll_put / ll_get).
__global__ __launch_bounds__(NT) void k_fwd_big(FrontTab T, const SolveTask* __restrict__ tasks, int ntasks,
                                                int32_t* counter, int32_t* flags, const int32_t* __restrict__ flag_off,
                                                int epoch, const double* __restrict__ arena,
                                                const double* __restrict__ vwork, double* __restrict__ xi,
                                                double* __restrict__ uvec, int32_t* err) {
  __shared__ int s_task;
  __shared__ double xs[64];
  __shared__ double part[4][64];
  __shared__ double Ld[64 * 65];
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  for (;;) {
    if (tid == 0) s_task = atomicAdd(counter, 1);
    __syncthreads();
    const int t = s_task;
    __syncthreads();
    if (t >= ntasks) return;
    const int s = tasks[t].front, i = tasks[t].blk;
    const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
    const double* __restrict__ L = arena + T.l_off[s];
    const int row0 = i * 64, nrow = min(64, r - row0);
    const int npan = (w + 63) >> 6;
    const int np = min(i, npan);
    const int row = row0 + lane;
    const bool pivot_blk = row0 < w;
    const int kw = pivot_blk ? min(64, w - row0) : 0;
    // every load below is issued unconditionally from a clamped address and masked after: a
    // predicated load compiles into a branch with a wait of its own (16 serial round trips per batch)
    const int rowc = row0 + min(lane, nrow - 1);
    // prefetch the diagonal block (columns row0 .. row0+kw-1 of this row block) into LDS
    if (kw > 0) {
      double v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = L[rowc + (int64_t)(row0 + min(g + 4 * e, kw - 1)) * r];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (g + 4 * e < kw) Ld[(g + 4 * e) * 65 + lane] = (lane < nrow) ? v[e] : 0.0;
    }
    double acc = 0.0;
    // the panel pieces are final (factorisation): panel p + 1's loads are issued before panel p's flag
    // wait and x loads, so one L round trip per task is exposed instead of one per panel
    double lv[16], ln[16];
    auto load_panel = [&](double (&dst)[16], int p) {
      const int cb = p * 64 + g * 16;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) dst[cc] = L[rowc + (int64_t)min(cb + cc, w - 1) * r];
    };
    if (np > 0) load_panel(lv, 0);
    for (int p = 0; p < np; ++p) {
      if (p + 1 < np) load_panel(ln, p + 1);  // wave-uniform
      const int cb = p * 64 + g * 16;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) lv[cc] = (lane < nrow && cb + cc < w) ? lv[cc] : 0.0;
      if (tid < 64) {
        const double xv = ll_get(T.xll + ((int64_t)flag_off[s] + p) * 128 + 2 * tid, epoch, err);
        xs[tid] = (p * 64 + tid < w) ? xv : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) acc += lv[cc] * xs[g * 16 + cc];
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) lv[cc] = ln[cc];
      __syncthreads();
    }
    part[g][lane] = acc;
    __syncthreads();
    if (g == 0) {
      double a = (lane < nrow) ? vwork[T.row_ptr[s] + row] - ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]))
                               : 0.0;
      a = tri_fwd64(a, Ld, kw, lane);
      if (pivot_blk) ll_put(T.xll + ((int64_t)flag_off[s] + i) * 128 + 2 * lane, a, epoch);  // every lane: 0 past nrow
      if (lane < nrow) {
        if (row < w)
          xi[f0 + row] = a;
        else
          uvec[T.uvec_off[s] + row - w] = a;
      }
    }
    __syncthreads();
  }
}

// Backward, big fronts, rows below the pivot block (independent of the panel chain): task =
// (front, panel p, 256-row chunk); writes bpart[(bp_off[front] + p * nchunk + chunk) * 64 + col] =
// sum over the chunk's rows of L(row, col) x(row).  The chain kernel sums the chunks in order.
constexpr int BWD_CHUNK = 256;
__global__ __launch_bounds__(NT) void k_bwd_below(FrontTab T, const int32_t* __restrict__ list,
                                                  const int32_t* __restrict__ bp_off, const double* __restrict__ arena,
                                                  const double* __restrict__ xi, double* __restrict__ bpart) {
  __shared__ double tile[64 * 65];
  __shared__ double xr[64];
  __shared__ double part[4][64];
  int s, pc;
  task_of(list, s, pc);
  const int p = pc & 0xffff, chunk = pc >> 16;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  (void)f0;
  const double* __restrict__ L = arena + T.l_off[s];
  const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
  const int c0 = p * 64, kw = min(64, w - c0);
  const int nch = (r - w + BWD_CHUNK - 1) / BWD_CHUNK;
  const int R0 = w + chunk * BWD_CHUNK, R1 = min(r, R0 + BWD_CHUNK);
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  double acc = 0.0;
  // unconditional loads from clamped addresses, masked at the LDS stores; the next row block's loads
  // are issued before this block's products (one round trip exposed per task, not per block)
  double v[16], vn[16], xv = 0.0, xvn = 0.0;
  auto load_blk = [&](double (&dst)[16], double& x, int rb) {
    const int nr = min(64, R1 - rb);
    const int rc = rb + min(lane, nr - 1);
#pragma unroll
    for (int e = 0; e < 16; ++e) dst[e] = L[rc + (int64_t)(c0 + min(g + 4 * e, kw - 1)) * r];
    x = (tid < 64) ? xi[rows[rb + min(tid, nr - 1)]] : 0.0;
  };
  if (R0 < R1) load_blk(v, xv, R0);
  for (int rb = R0; rb < R1; rb += 64) {
    const int nr = min(64, R1 - rb);
#pragma unroll
    for (int e = 0; e < 16; ++e) tile[lane * 65 + g + 4 * e] = (lane < nr && g + 4 * e < kw) ? v[e] : 0.0;
    if (tid < 64) xr[tid] = (tid < nr) ? xv : 0.0;
    __syncthreads();
    if (rb + 64 < R1) load_blk(vn, xvn, rb + 64);  // block-uniform
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) acc += tile[(g * 16 + rr) * 65 + lane] * xr[g * 16 + rr];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = vn[e];
    xv = xvn;
    __syncthreads();
  }
  part[g][lane] = acc;
  __syncthreads();
  if (g == 0)
    bpart[((int64_t)bp_off[s] + (int64_t)p * nch + chunk) * 64 + lane] =
        (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

// Backward, big fronts: task = (front, 64-column pivot panel p), processed from the last panel down.
// acc(cols) = D^{-1} y(cols) - L(below,cols)^T x(below) - sum_{q > p} L(q-block,cols)^T x_q; x_p = L_pp^{-T} acc.
__global__ __launch_bounds__(NT) void k_bwd_big(FrontTab T, const SolveTask* __restrict__ tasks, int ntasks,
                                                int32_t* counter, int32_t* flags, const int32_t* __restrict__ flag_off,
                                                int epoch, const double* __restrict__ arena,
                                                const double* __restrict__ D, double* __restrict__ xi,
                                                double* __restrict__ out, const int32_t* __restrict__ bp_off,
                                                const double* __restrict__ bpart, int32_t* err) {
  __shared__ int s_task;
  __shared__ double tile[64 * 65];
  __shared__ double xr[64];
  __shared__ double part[4][64];
  __shared__ double Ld[64 * 65];
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  for (;;) {
    if (tid == 0) s_task = atomicAdd(counter, 1);
    __syncthreads();
    const int t = s_task;
    __syncthreads();
    if (t >= ntasks) return;
    const int s = tasks[t].front, p = tasks[t].blk;
    const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
    const double* __restrict__ L = arena + T.l_off[s];
    const int c0 = p * 64, kw = min(64, w - c0);
    const int npan = (w + 63) >> 6;
    // diagonal block L(c0+i, c0+j) -> Ld[i*65+j] (unconditional clamped loads, masked at the store)
    {
      double v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = L[(c0 + min(lane, kw - 1)) + (int64_t)(c0 + min(g + 4 * e, kw - 1)) * r];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (g + 4 * e < kw) Ld[lane * 65 + g + 4 * e] = (lane < kw) ? v[e] : 0.0;
    }
    double acc = 0.0;  // partial for column c0+lane over this wave's rows of each tile
    // pivot panels q = npan-1 .. p+1 (wait for each); the rows below come from k_bwd_below.  A tile's
    // L values are final: they are loaded before the wait for its x (the next tile's during this
    // tile's products), only the x values wait for the flag
    const int nq = npan - 1 - p;
    double v[16], vn[16];
    auto load_tile = [&](double (&dst)[16], int q) {
      const int rb = q * 64, nr = min(64, w - rb);
      const int rc = rb + min(lane, nr - 1);
#pragma unroll
      for (int e = 0; e < 16; ++e) dst[e] = L[rc + (int64_t)(c0 + min(g + 4 * e, kw - 1)) * r];
    };
    if (nq > 0) load_tile(v, npan - 1);
    for (int k = 0; k < nq; ++k) {
      const int q = npan - 1 - k;
      const int rb = q * 64, nr = min(64, w - rb);
      // stage the 64 x 64 tile L(rb.., c0..) (coalesced over rows) and the x values of its rows (the
      // panel's solution words, ll_get: they are the hand-off)
      {
        const double xv = (tid < 64) ? ll_get(T.xll + ((int64_t)flag_off[s] + q) * 128 + 2 * tid, epoch, err) : 0.0;
#pragma unroll
        for (int e = 0; e < 16; ++e)
          if (g + 4 * e < kw) tile[lane * 65 + g + 4 * e] = (lane < nr) ? v[e] : 0.0;
        if (tid < 64) xr[tid] = (tid < nr) ? xv : 0.0;
      }
      __syncthreads();
      if (k + 1 < nq) load_tile(vn, q - 1);  // block-uniform
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) acc += tile[(g * 16 + rr) * 65 + lane] * xr[g * 16 + rr];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = vn[e];
      __syncthreads();
    }
    if (g == 0 && r > w) {
      const int nch = (r - w + BWD_CHUNK - 1) / BWD_CHUNK;
      const double* __restrict__ bp = bpart + ((int64_t)bp_off[s] + (int64_t)p * nch) * 64 + lane;
      double below = 0.0;
      for (int c = 0; c < nch; ++c) below += bp[c * 64];
      acc += below;
    }
    part[g][lane] = acc;
    __syncthreads();
    if (g == 0) {
      double a = 0.0;
      if (lane < kw) {
        const int c = f0 + c0 + lane;
        a = xi[c] / D[c] - ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]));
      }
      a = tri_bwd64(a, Ld, kw, lane);
      ll_put(T.xll + ((int64_t)flag_off[s] + p) * 128 + 2 * lane, a, epoch);  // every lane (masked by the readers)
      if (lane < kw) {
        const int c = f0 + c0 + lane;
        xi[c] = a;
        if (T.wout[s]) out[T.perm[c]] = a;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ tree solves (dependency-driven)
// ONE launch per direction covers every "tree" front (LDLSolver ctor: phase-1 fronts whose L panel
// fits LDS and whose children are leaves of <= 32 rows — done by the level-0 launches — or tree
// fronts).  A workgroup takes the next front in topological order from an atomic ticket (every
// front it waits on holds an earlier ticket, taken by a running workgroup: no deadlock at any grid
// size or residency), stages its L panel into LDS BEFORE waiting, then polls its dependencies'
// flags (forward: tree children; backward: the tree parent), substitutes and publishes.  Hand-off
// (MI355X_MICROARCH.md "inter-workgroup visibility", form R1): the payload (xi, uvec) is stored
// write-through (sc1) by the ONE publishing wave, which drains it (vmcnt 0) before its lane 0 stores
// the flag; every consumer load of handed-off bytes is an sc1 load behind the poll and a workgroup
// barrier — no agent-scope fences on the dependency chain.

// Tree-solve substitutions, one wave, 16 pivots per block, mask-free: the panels are staged with the
// upper triangle + diagonal zeroed and the pivot columns zero-padded to a multiple of 16, so every
// block loads its L entries unconditionally (16-byte LDS reads, immediate offsets) and the
// dependency chain is one readlane + one fma per pivot.
// dynamic LDS of the tree solves (+ ~2 KB static): two 256-thread workgroups per CU
constexpr int TREE_ROOT_LDS = 150 * 1024;  // the big etree roots' own forward launch (LDSolver: nroot_task_)
constexpr int TREE_SOLVE_LDS = 76 * 1024;
__device__ __forceinline__ int tree_ldt(int w) { return ((w + 15) & ~15) + 2; }  // forward: row-major ld
__device__ __forceinline__ int tree_ldc(int r) { return ((r + 31) & ~31) + 2; }  // backward: col-major ld

// forward staging: LT[i * ldt + t] = L(i, t) for t < min(i, w), else 0 (t < w16)
template <int NTH = NT>
__device__ __forceinline__ void stage_rowmajor(const double* __restrict__ L, double* LT, int r, int w, int ldt) {
  const int w16 = (w + 15) & ~15;
  const int nel = r * w16;
  ColWalk wk(threadIdx.x, r, NTH);
  for (int base = 0; base < nel; base += NTH * 16) {
    double v[16];
    int dst[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = base + k * NTH + threadIdx.x;
      v[k] = (q < nel && wk.j < w && wk.i > wk.j) ? L[q] : 0.0;
      dst[k] = (q < nel) ? wk.i * ldt + wk.j : -1;
      wk.next();
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (dst[k] >= 0) LT[dst[k]] = v[k];
  }
}

// backward staging: LC[j * ldc + t] = L(t, j) for t > j, else 0 (j < w, t < r)
__device__ __forceinline__ void stage_colmajor(const double* __restrict__ L, double* LC, int r, int w, int ldc) {
  const int nel = r * w;
  ColWalk wk(threadIdx.x, r);
  for (int base = 0; base < nel; base += NT * 16) {
    double v[16];
    int dst[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = base + k * NT + threadIdx.x;
      v[k] = (q < nel && wk.i > wk.j) ? L[q] : 0.0;
      dst[k] = (q < nel) ? wk.j * ldc + wk.i : -1;
      wk.next();
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (dst[k] >= 0) LC[dst[k]] = v[k];
  }
  const int pad = ((w + 15) & ~15) - r;  // the last pivot block may reach past row r - 1: zero rows
  for (int q = threadIdx.x; q < w * pad; q += NT) LC[(q / pad) * ldc + r + q % pad] = 0.0;
}

template <int HB>
__device__ __forceinline__ void fwd_block_t(double (&v)[3], const double* LT, int ldt, int r, int t0, int lane) {
  double lb[3][16];
#pragma unroll
  for (int h = HB; h < 3; ++h) {
    const double2* rp = reinterpret_cast<const double2*>(LT + min(lane + 64 * h, r - 1) * ldt + t0);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const double2 q = rp[m];
      lb[h][2 * m] = q.x;
      lb[h][2 * m + 1] = q.y;
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double xt = readlane_f64(v[HB], (t0 & 63) + k);
#pragma unroll
    for (int h = HB; h < 3; ++h) v[h] = fma(-lb[h][k], xt, v[h]);
  }
}

// forward: v[i] -= L(i, t) v[t] for i > t, t < w (columns >= w are zero)
__device__ __forceinline__ void fwd_subst_t(double (&v)[3], const double* LT, int ldt, int r, int w, int lane) {
  for (int t0 = 0; t0 < w; t0 += 16) {
    if (t0 < 64)
      fwd_block_t<0>(v, LT, ldt, r, t0, lane);
    else if (t0 < 128)
      fwd_block_t<1>(v, LT, ldt, r, t0, lane);
    else
      fwd_block_t<2>(v, LT, ldt, r, t0, lane);
  }
}

template <int HB>
__device__ __forceinline__ void bwd_block_c(double (&v)[3], const double* LC, int ldc, int w, int t0, int lane) {
  double lb[HB + 1][16];
#pragma unroll
  for (int h = 0; h <= HB; ++h) {
    const double2* cp = reinterpret_cast<const double2*>(LC + min(lane + 64 * h, w - 1) * ldc + t0);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const double2 q = cp[m];
      lb[h][2 * m] = q.x;
      lb[h][2 * m + 1] = q.y;
    }
  }
#pragma unroll
  for (int k = 15; k >= 0; --k) {  // lanes >= w hold 0 and stay 0 until k < kb
    const double xt = readlane_f64(v[HB], (t0 & 63) + k);
#pragma unroll
    for (int h = 0; h <= HB; ++h) v[h] = fma(-lb[h][k], xt, v[h]);
  }
}

// backward (transposed): v[j] -= L(t, j) v[t] for j < t, t = w-1 .. 1
__device__ __forceinline__ void bwd_subst_c(double (&v)[3], const double* LC, int ldc, int w, int lane) {
  for (int t0 = ((w - 1) >> 4) << 4; t0 >= 0; t0 -= 16) {
    if (t0 < 64)
      bwd_block_c<0>(v, LC, ldc, w, t0, lane);
    else if (t0 < 128)
      bwd_block_c<1>(v, LC, ldc, w, t0, lane);
    else
      bwd_block_c<2>(v, LC, ldc, w, t0, lane);
  }
}

// backward (transposed) on the forward's row-major panel: v[j] -= L(t, j) v[t] for j < t, t = w-1 .. 0,
// L(t, j) = LT[t ldt + j] — the same fma sequence as bwd_subst_c (bitwise the same x).  Used by the
// forward kernel for an elimination-tree root (r == w) whose panel it already holds in LDS.
template <int HB>
__device__ __forceinline__ void bwd_block_t(double (&v)[3], const double* LT, int ldt, int w, int t0, int lane) {
  double lb[HB + 1][16];
#pragma unroll
  for (int h = 0; h <= HB; ++h) {
    const int j = min(lane + 64 * h, w - 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) lb[h][k] = LT[min(t0 + k, w - 1) * ldt + j];
  }
#pragma unroll
  for (int k = 15; k >= 0; --k) {
    const double xt = readlane_f64(v[HB], (t0 & 63) + k);
#pragma unroll
    for (int h = 0; h <= HB; ++h) v[h] = fma(-lb[h][k], xt, v[h]);
  }
}
__device__ __forceinline__ void bwd_subst_t(double (&v)[3], const double* LT, int ldt, int w, int lane) {
  for (int t0 = ((w - 1) >> 4) << 4; t0 >= 0; t0 -= 16) {
    if (t0 < 64)
      bwd_block_t<0>(v, LT, ldt, w, t0, lane);
    else if (t0 < 128)
      bwd_block_t<1>(v, LT, ldt, w, t0, lane);
    else
      bwd_block_t<2>(v, LT, ldt, w, t0, lane);
  }
}

// ---- Chunked tree-solve fronts: medium fronts (SMALL_SOLVE_MAX < r <= kFactTreeMedMax) and every
// front whose whole panel would not fit the tree solves' LDS budget (TREE_SOLVE_LDS: two workgroups per
// CU, so the 272 level-1/2 fronts of ex10 all start at once — with one per CU, 16 of them waited for
// a level-1 front to retire).  The L panel is streamed in 16-column chunks, double-buffered: wave 0
// substitutes chunk c while waves 1..3 stage chunk c +- 1.  v (forward) / x (backward) stay in wave 0's
// registers, 4 rows per lane.
constexpr int MED_SOLVE_MAX = SymbolicPlan::kFactTreeMedMax;
constexpr int MCW = 16, MLDT = MCW + 2;           // forward chunk: pivot columns, row-major ld
constexpr int MFBUF = MED_SOLVE_MAX * MLDT;       // doubles per forward chunk buffer
constexpr int MLDC = MED_SOLVE_MAX + 2;           // backward chunk: col-major ld
constexpr int MBBUF = MCW * MLDC;                 // doubles per backward chunk buffer
constexpr int MED_FWD_LDS = 2 * MFBUF, MED_BWD_LDS = 2 * MBBUF + 2 * MED_SOLVE_MAX;  // doubles
static_assert(8 * MED_FWD_LDS <= TREE_SOLVE_LDS && 8 * MED_BWD_LDS <= TREE_SOLVE_LDS,
              "chunked tree-solve buffers fit the tree launches' LDS");

// rows [ra, r) x columns [c0, c0 + MCW) of L (ld r) -> LT[(i - ra) MLDT + (t - c0)] = L(i, t) for
// t < w and i > t, else 0; threads lt = 0 .. nthr - 1 of the caller's group
__device__ __forceinline__ void stage_fwd_chunk(const double* __restrict__ L, double* LT, int r, int w, int ra, int c0,
                                                int lt, int nthr) {
  const int nrow = r - ra, nel = nrow * MCW;
  ColWalk wk(lt, nrow, nthr);
  for (int base = 0; base < nel; base += nthr * 8) {
    double v[8];
    int dst[8];
    bool ok[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = base + k * nthr + lt, i = ra + wk.i, t = c0 + wk.j;
      ok[k] = t < w && i > t;
      v[k] = L[min(i, r - 1) + (int64_t)min(t, w - 1) * r];  // clamped, in range: masked below
      dst[k] = q < nel ? wk.i * MLDT + wk.j : -1;
      wk.next();
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (dst[k] >= 0) LT[dst[k]] = ok[k] ? v[k] : 0.0;
  }
}

template <int HB>
__device__ __forceinline__ void fwd_block_m(double (&v)[4], const double* LT, int r, int ra, int tc, int t0, int lane) {
  double lb[4][16];
#pragma unroll
  for (int h = HB; h < 4; ++h) {
    const double2* rp = reinterpret_cast<const double2*>(LT + (min(lane + 64 * h, r - 1) - ra) * MLDT + tc);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const double2 q = rp[m];
      lb[h][2 * m] = q.x;
      lb[h][2 * m + 1] = q.y;
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double xt = readlane_f64(v[HB], (t0 & 63) + k);
#pragma unroll
    for (int h = HB; h < 4; ++h) v[h] = fma(-lb[h][k], xt, v[h]);
  }
}

// column chunk [c0, c0 + MCW) of L (ld r), rows [c0, r) -> LC[(j - c0) MLDC + (t - c0)] = L(t, j) for
// j < w and t > j, else 0
__device__ __forceinline__ void stage_bwd_chunk(const double* __restrict__ L, double* LC, int r, int w, int c0, int lt,
                                                int nthr) {
  const int nrow = r - c0, nel = nrow * MCW;
  ColWalk wk(lt, nrow, nthr);
  for (int base = 0; base < nel; base += nthr * 8) {
    double v[8];
    int dst[8];
    bool ok[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = base + k * nthr + lt, t = c0 + wk.i, j = c0 + wk.j;
      ok[k] = j < w && t > j;
      v[k] = L[min(t, r - 1) + (int64_t)min(j, w - 1) * r];
      dst[k] = q < nel ? wk.j * MLDC + wk.i : -1;
      wk.next();
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (dst[k] >= 0) LC[dst[k]] = ok[k] ? v[k] : 0.0;
  }
}

// forward solve of a medium tree front (all NT threads; v0: the gathered initial values of its rows)
__device__ __forceinline__ void fwd_med_front(const FrontTab& T, int s, const double* __restrict__ arena, double* Ls,
                                              const double* v0, double* xi, double* uvec, int32_t* tflags, int epoch) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const double* __restrict__ L = arena + T.l_off[s];
  const int nch = (((w + 15) & ~15) + MCW - 1) / MCW;
  double* buf[2] = {Ls, Ls + MFBUF};
  stage_fwd_chunk(L, buf[0], r, w, 0, 0, tid, NT);
  double v[4];
  double* dst[4];
  uvec_dsts<4>(T, s, w, r, f0, wv == 0, lane, uvec, xi, dst);
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const int i = lane + 64 * h;
    v[h] = (i < r) ? v0[i] : 0.0;
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int c0 = c * MCW;
    if (wv == 0) {
      const int ra = (c0 >> 6) << 6;
      const double* LT = buf[c & 1];
      const int tend = min(c0 + MCW, (w + 15) & ~15);
      for (int t0 = c0; t0 < tend; t0 += 16) {
        const int tc = t0 - c0;
        switch (t0 >> 6) {
          case 0: fwd_block_m<0>(v, LT, r, ra, tc, t0, lane); break;
          case 1: fwd_block_m<1>(v, LT, r, ra, tc, t0, lane); break;
          case 2: fwd_block_m<2>(v, LT, r, ra, tc, t0, lane); break;
          default: fwd_block_m<3>(v, LT, r, ra, tc, t0, lane); break;
        }
      }
    } else if (c + 1 < nch) {
      const int c1 = c0 + MCW;
      stage_fwd_chunk(L, buf[(c + 1) & 1], r, w, (c1 >> 6) << 6, c1, tid - 64, NT - 64);
    }
    __syncthreads();
  }
  if (wv == 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
      if (lane + 64 * h < r) st_sc1(dst[h], v[h]);
    publish_sc1(&tflags[s], epoch);
  }
  __syncthreads();
}

// backward solve of a medium tree front (all NT threads): chunks from the last to the first; xall holds
// the final x of every row below the current chunk (the ancestors' rows, then this front's later pivots)
__device__ __forceinline__ void bwd_med_front(const FrontTab& T, int s, const double* __restrict__ arena,
                                              const double* __restrict__ D, double* Ls, double* xi, double* out,
                                              const int32_t* __restrict__ pdep, int t, int32_t* tflags, int epoch,
                                              int32_t* err) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s], nb = r - w;
  const double* __restrict__ L = arena + T.l_off[s];
  double* buf[2] = {Ls, Ls + MBBUF};
  double* xall = Ls + 2 * MBBUF;            // r doubles
  double* ownv = xall + MED_SOLVE_MAX;      // w doubles: the forward values / d
  const int nch = (w + MCW - 1) / MCW;
  // symbolic / previous-launch data before the wait: the rows below, the own values, the last chunk
  const int rk = (tid < nb) ? T.rows[T.row_ptr[s] + w + tid] : 0;
  if (tid < w) ownv[tid] = xi[f0 + tid] / D[f0 + tid];
  stage_bwd_chunk(L, buf[(nch - 1) & 1], r, w, (nch - 1) * MCW, tid, NT);
  if (tid < 64 && pdep[t] >= 0) poll_deps(pdep, t, t + 1, tflags, epoch, err);
  __syncthreads();
  if (tid < nb) xall[w + tid] = ld_sc1(xi + rk);
  __syncthreads();
  const bool wo = T.wout[s];
  constexpr int NG = 64 / MCW;  // lane groups of the wave: group g sums the rows t = c1 + g (mod NG)
  const int jl = lane % MCW, grp = lane / MCW;
  for (int c = nch - 1; c >= 0; --c) {
    const int c0 = c * MCW, c1 = min(c0 + MCW, w), j = c0 + jl;
    if (wv == 0) {
      const double* LC = buf[c & 1] + jl * MLDC;
      // rows below the chunk (NG lane groups, interleaved rows), then the chunk's own triangle
      double a0 = 0.0, a1 = 0.0;
      int q = c1 + grp;
      for (; q + NG < r; q += 2 * NG) {
        a0 = fma(LC[q - c0], xall[q], a0);
        a1 = fma(LC[q + NG - c0], xall[q + NG], a1);
      }
      for (; q < r; q += NG) a0 = fma(LC[q - c0], xall[q], a0);
      const double part = a0 + a1;
      double p[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) p[g] = __shfl(part, jl + MCW * g, 64);
      static_assert(NG == 4, "bwd_med_front: four lane groups");
      const double acc = (p[0] + p[1]) + (p[2] + p[3]);  // the same fixed order in every lane group
      double x = (j < w) ? ownv[min(j, w - 1)] - acc : 0.0;
      for (int tt = c1 - 1; tt > c0; --tt) {  // x_j -= L(tt, j) x_tt, j < tt
        const double xt = readlane_f64(x, tt - c0);
        x = fma(-LC[tt - c0], xt, x);
      }
      if (grp == 0 && j < w) {
        xall[j] = x;
        st_sc1(xi + f0 + j, x);
        if (wo) out[T.perm[f0 + j]] = x;
      }
    } else if (c > 0) {
      stage_bwd_chunk(L, buf[(c - 1) & 1], r, w, (c - 1) * MCW, tid - 64, NT - 64);
    }
    __syncthreads();
  }
  if (tid < 64) publish_sc1(&tflags[s], epoch);
  __syncthreads();
}

// The micro leaves under tree fronts as flat launches: LPL lanes per leaf, each lane forms
// x0, x1 itself (the same loads) and takes rows a = j, j + LPL, ...; the leaf record carries every
// index, so a lane's loads are one dependent level deep (record -> b, L, row table).  Forward before
// k_fwd_tree (it gathers the update entries from gbuf), backward after k_bwd_tree (final ancestors).
constexpr int LPL = 4, LROWS = (32 + LPL - 1) / LPL;
__global__ __launch_bounds__(NT) void k_fwd_leaves(const SolveLeaf* __restrict__ lv, int nleaf,
                                                   const int2* __restrict__ lrow, const double* __restrict__ arena,
                                                   const double* __restrict__ b, double* __restrict__ xi,
                                                   double* __restrict__ gbuf) {
  const int gid = blockIdx.x * NT + threadIdx.x;
  const int k = gid / LPL, j = gid % LPL;
  if (k >= nleaf) return;
  const SolveLeaf L = lv[k];
  const int r = L.rw & 255, w = L.rw >> 8, u = r - w;
  const double* __restrict__ P = arena + L.loff;
  // unconditional loads from clamped in-range addresses (a leaf with no update rows reads its own
  // pivot entry; the row table is padded by one record), masked at the use
  double p[LROWS], q[LROWS];
  int d[LROWS];
#pragma unroll
  for (int m = 0; m < LROWS; ++m) {
    const int a = max(min(j + LPL * m, u - 1), 0);
    p[m] = P[min(w + a, r - 1)];
    q[m] = P[(w == 2) ? min(w + a, r - 1) + r : 0];
    d[m] = lrow[L.roff + a].x;
  }
  const double b0 = b[L.p0], b1r = b[(w == 2) ? L.p1 : L.p0], l10r = P[1 < r ? 1 : 0];
  const double b1 = (w == 2) ? b1r : 0.0, l10 = (w == 2) ? l10r : 0.0;
  const double x0 = b0, x1 = (w == 2) ? b1 - l10 * x0 : 0.0;
  if (j == 0) {
    xi[L.f0] = x0;
    if (w == 2) xi[L.f0 + 1] = x1;
  }
#pragma unroll
  for (int m = 0; m < LROWS; ++m)
    if (j + LPL * m < u) gbuf[d[m]] = (0.0 - p[m] * x0) - (w == 2 ? q[m] : 0.0) * x1;
}

__global__ __launch_bounds__(NT) void k_bwd_leaves(const SolveLeaf* __restrict__ lv, int nleaf,
                                                   const int2* __restrict__ lrow, const double* __restrict__ arena,
                                                   const double* __restrict__ D, double* __restrict__ xi,
                                                   double* __restrict__ out) {
  const int gid = blockIdx.x * NT + threadIdx.x;
  const int k = gid / LPL, j = gid % LPL;
  if (k >= nleaf) return;  // whole leaves only: the LPL lanes of a leaf exit together
  const SolveLeaf L = lv[k];
  const int r = L.rw & 255, w = L.rw >> 8, u = r - w;
  const double* __restrict__ P = arena + L.loff;
  // unconditional loads from clamped in-range addresses, masked at the use (as k_fwd_leaves)
  int src[LROWS];
#pragma unroll
  for (int m = 0; m < LROWS; ++m) src[m] = lrow[L.roff + max(min(j + LPL * m, u - 1), 0)].y;
  double p[LROWS], q[LROWS], x[LROWS];
#pragma unroll
  for (int m = 0; m < LROWS; ++m) {
    const int a = max(min(j + LPL * m, u - 1), 0);
    p[m] = P[min(w + a, r - 1)];
    q[m] = P[(w == 2) ? min(w + a, r - 1) + r : 0];
    x[m] = xi[src[m]];  // the tree fronts' final x (previous launch)
  }
  // the pivots' own entries, for lane 0's tail (loaded with the rest)
  const int f1 = L.f0 + (w == 2 ? 1 : 0);
  const double l10r = P[1 < r ? 1 : 0], xf0 = xi[L.f0], df0 = D[L.f0], xf1 = xi[f1], df1 = D[f1];
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int m = 0; m < LROWS; ++m)
    if (j + LPL * m < u) {
      a0 = fma(p[m], x[m], a0);
      a1 = fma(q[m], x[m], a1);
    }
  // ((lane 0 + lane 1) + (lane 2 + lane 3)): a fixed order
  a0 += __shfl_xor(a0, 1, LPL);
  a1 += __shfl_xor(a1, 1, LPL);
  a0 += __shfl_xor(a0, 2, LPL);
  a1 += __shfl_xor(a1, 2, LPL);
  if (j != 0) return;
  const double l10 = (w == 2) ? l10r : 0.0;
  const double v1 = (w == 2) ? xf1 / df1 - a1 : 0.0;
  const double v0 = xf0 / df0 - a0 - l10 * v1;
  xi[L.f0] = v0;
  out[L.p0] = v0;
  if (w == 2) {
    xi[L.f0 + 1] = v1;
    out[L.p1] = v1;
  }
}

// Tree solves over CHAIN tasks: a task is a maximal chain of tree fronts in which every front is the
// only tree child of the next (LDLSolver ctor), solved back to back by one workgroup (forward deepest
// first, backward top first) together with the folded micro leaves of its fronts: inside a chain no
// flag hand-off, no second workgroup start, and the leaves need no launch of their own.  Only the
// chain's ends talk to other workgroups (forward: the tree children of its deepest front, poll; its top
// publishes.  Backward: the top polls its tree parent; every front publishes for the tasks below).
// Inside the chain a front's stores (update entries, x) are drained (vmcnt 0) before the barrier that
// precedes the next front's sc1 loads of them.
// Dynamic LDS of the tree solve kernels: L panel | gather staging.
__global__ __launch_bounds__(NT) void k_fwd_tree(FrontTab T, const int32_t* __restrict__ cptr, const int32_t* __restrict__ clist,
                                                 int nt, const int32_t* __restrict__ dep_ptr, const int32_t* __restrict__ dep,
                                                 int32_t* counter, int32_t* tflags, int epoch, int lds_doubles,
                                                 const double* __restrict__ arena, const double* __restrict__ b,
                                                 double* xi, double* uvec, int32_t* err, int64_t* dbg,
                                                 const uint8_t* __restrict__ rootbwd, const double* __restrict__ Dg,
                                                 const uint8_t* __restrict__ tchunk, const uint8_t* __restrict__ tside,
                                                 const int32_t* rdone, int nrd, int repoch) {
  extern __shared__ __attribute__((aligned(16))) double Ls[];
  __shared__ double v0s[MED_SOLVE_MAX];
  __shared__ int s_task;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_task = atomicAdd(counter, 1);
    if (s_task == nt - 1) atomicExch(counter, 0);  // every ticket taken: ready for the next launch
  }
  __syncthreads();
  const int t = s_task;
  if (t >= nt) return;
  int64_t* dg = dbg ? dbg + 8 * t : nullptr;
  if (dg && tid == 0) dg[0] = wall_clock64();
  const int q0 = cptr[t], q1 = cptr[t + 1];
  if (dg) {
    __syncthreads();
    if (tid == 0) dg[1] = wall_clock64();
  }
  for (int q = q0; q < q1; ++q) {
    const int s = clist[q];
    const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
    const bool med = tchunk[s];  // chunked front: panel streamed after the gather
    const int ldt = tree_ldt(w);
    double* stg = med ? Ls : Ls + r * ldt;
    const int cap = med ? (lds_doubles / NT) * NT : ((lds_doubles - r * ldt) / NT) * NT;
    // a root factorised on the side stream (LDLSolver::root_async_, first solve after the
    // factorisation): its panel and pivots only after the tail's done flags
    const bool sw = nrd > 0 && tside[t] && q == q1 - 1;
    if (!med && !sw) stage_rowmajor(arena + T.l_off[s], Ls, r, w, ldt);
    // everything that does not depend on the children is loaded before the wait: the gather range
    // (symbolic) and this front's own right-hand side entries (the input b)
    const int64_t e0 = T.row_ptr[s];
    const int64_t P0 = T.sv_ptr[e0], P1 = T.sv_ptr[e0 + r];
    const int64_t pr0 = (tid < r) ? T.sv_ptr[e0 + tid] : 0, pr1 = (tid < r) ? T.sv_ptr[e0 + tid + 1] : 0;
    const double init = (tid < r) ? fwd_init(T, s, tid, w, f0, b) : 0.0;
    double* udst[3];  // wave 0: where its rows' results go (x for pivots, the parent's gather slot below)
    uvec_dsts<3>(T, s, w, r, f0, tid < 64, tid & 63, uvec, xi, udst);
    // an elimination-tree root (r == w) also runs its backward substitution here:
    // its pivots and the caller's positions are loaded before the wait
    const bool rb = q == q1 - 1 && rootbwd[t];
    double dpiv[3];
    int pj[3];
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int j = min((tid & 63) + 64 * h, max(w - 1, 0));
      dpiv[h] = (rb && tid < 64) ? Dg[f0 + j] : 1.0;
      pj[h] = (rb && tid < 64) ? T.perm[f0 + j] : 0;
    }
    // initial vector: the children scattered their update entries into this front's contiguous range
    // gbuf[P0, P1) in row order, each row's entries from childless children (the leaves, solved by an
    // earlier launch) first and from its tree children (this launch) last (sv_nt, LDLSolver ctor).  The
    // leaf part is summed BEFORE the wait: staged through LDS (16 coalesced loads in flight per
    // thread), thread i sums row i's leaf entries in order (4 partial sums); after the wait only the
    // tree children's few entries per row are loaded (one round trip)
    const int ntr = (tid < r) ? (int)T.sv_nt[e0 + tid] : 0;
    const int64_t pl1 = pr1 - ntr;  // the row's leaf part: [pr0, pl1)
    double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
    for (int64_t base = P0; base < P1; base += cap) {
      const int n = (int)min((int64_t)cap, P1 - base);
      for (int g0 = 0; g0 < n; g0 += NT * 16) {
        double tmp[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int g = g0 + k * NT + tid;
          tmp[k] = (g < n) ? ld_sc1(T.gbuf + base + g) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int g = g0 + k * NT + tid;
          if (g < n) stg[g] = tmp[k];
        }
      }
      __syncthreads();
      const int lo = (int)(max(pr0, base) - base), hi = (int)(min(pl1, base + n) - base);
      int p = lo;
      for (; p + 3 < hi; p += 4) {
        c0 += stg[p];
        c1 += stg[p + 1];
        c2 += stg[p + 2];
        c3 += stg[p + 3];
      }
      for (; p < hi; ++p) c0 += stg[p];
      __syncthreads();
    }
    if (q == q0 && tid < 64) poll_deps(dep, dep_ptr[t], dep_ptr[t + 1], tflags, epoch, err);
    __syncthreads();  // + the previous front's / the leaves' drained stores (vmcnt 0 before it)
    if (sw) {
      if (tid < 64) {
        const int lane = tid;
        int spins = 0;
        for (;;) {
          const bool ok = lane >= nrd ||
                          __hip_atomic_load(rdone + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == repoch;
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1 << 25)) {
            if (lane == 0) atomicOr(err, kErrHandoff);
            break;
          }
        }
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (!med) stage_rowmajor(arena + T.l_off[s], Ls, r, w, ldt);
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int j = min((tid & 63) + 64 * h, max(w - 1, 0));
        dpiv[h] = (rb && tid < 64) ? Dg[f0 + j] : 1.0;
      }
      __syncthreads();
    }
    if (dg && tid == 0 && q == q0) dg[2] = wall_clock64();
    double ct = 0.0;  // the tree children's entries of this row, in order
    for (int k = 0; k < ntr; ++k) ct += ld_sc1(T.gbuf + pl1 + k);
    if (tid < r) v0s[tid] = (((c0 + c1) + (c2 + c3)) + ct) + init;
    __syncthreads();
    if (med) {
      fwd_med_front(T, s, arena, Ls, v0s, xi, uvec, tflags, epoch);
      continue;
    }
    if (dg && tid == 0 && q == q1 - 1) dg[3] = wall_clock64();
    if (tid < 64) {
      const int lane = tid;
      double v[3];
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int i = lane + 64 * h;
        v[h] = (i < r) ? v0s[i] : 0.0;
      }
      fwd_subst_t(v, Ls, ldt, r, w, lane);
      if (dg && tid == 0 && q == q1 - 1) dg[4] = wall_clock64();
      if (rb) {  // k_bwd_tree's work for this root: x = L^-T (D^-1 y), published with the backward epoch
#pragma unroll
        for (int h = 0; h < 3; ++h) v[h] = (lane + 64 * h < w) ? v[h] / dpiv[h] : 0.0;
        bwd_subst_t(v, Ls, ldt, w, lane);
        double* out = const_cast<double*>(b);  // the caller's vector: x at this root's pivots (read by no other task)
#pragma unroll
        for (int h = 0; h < 3; ++h) {
          const int j = lane + 64 * h;
          if (j < w) {
            st_sc1(xi + f0 + j, v[h]);
            if (T.wout[s]) out[pj[h]] = v[h];
          }
        }
        publish_sc1(&tflags[s], epoch + 1);
      } else {
#pragma unroll
        for (int h = 0; h < 3; ++h) {
          const int i = lane + 64 * h;
          if (i < r) st_sc1(udst[h], v[h]);
        }
        if (q == q1 - 1)
          publish_sc1(&tflags[s], epoch);  // the chain's top: its tree parent is another task's
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();  // wave 0 is done with Ls; its stores are drained
  }
  if (dg && tid == 0) {
    dg[5] = wall_clock64();
    dg[6] = clist[q1 - 1];
    dg[7] = T.nrows[clist[q1 - 1]];
  }
}

// The big elimination-tree roots of the tree solves (LDLSolver::nroot_task_: r == w, panel beyond the
// tree launches' 76 KB; ex10's 120-column coupling root), one 1024-thread workgroup each, after the
// forward tree launch (every child has scattered its update entries): the panel staged row-major in
// one round of loads, each row's gather segment summed by four threads (strided, all loads in
// flight), then the forward and backward substitutions on the staged panel (k_fwd_tree's root-backward
// path: the same fma sequences).  In k_fwd_tree the root's single 256-thread workgroup staged 125 KB
// of panel and its ~20k gather entries through the LDS left beside the panel: 26-34 us per solve.
constexpr int RSN = 1024;
__global__ __launch_bounds__(RSN) void k_root_solve(FrontTab T, const int32_t* __restrict__ fronts,
                                                    const double* __restrict__ arena, double* b, double* xi,
                                                    const double* __restrict__ Dg, int32_t* tflags, int epoch,
                                                    const int32_t* rdone, int nrd, int repoch, int64_t* dbg,
                                                    RootArgs RA) {
  extern __shared__ __attribute__((aligned(16))) double Ls[];
  __shared__ double part[4 * SMALL_SOLVE_MAX], inits[SMALL_SOLVE_MAX];
  int64_t* dg = dbg ? dbg + 8 * blockIdx.x : nullptr;  // MADIPM_TREE_DEBUG: phase stamps
  if (dg && threadIdx.x == 0) dg[0] = wall_clock64();
  const int q = blockIdx.x;
  const bool ra = q < RA.n;  // (the shapes in the launch arguments; beyond kRootArgs, from the tables)
  const int s = ra ? RA.s[q] : fronts[q];
  const int f0 = ra ? RA.f0[q] : T.first[s], w = ra ? RA.w[q] : T.first[s + 1] - f0, r = ra ? RA.r[q] : T.nrows[s];
  const int64_t loff = ra ? RA.loff[q] : T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63;
  const int ldt = tree_ldt(w);
  // gather: row i = tid >> 2 summed by threads k = tid & 3 over the entries lo + 4 m + k of its segment
  // (the tail past the last full group of 4 by k = 0, in order: k_fwd_tree's summation)
  const int i = tid >> 2, k = tid & 3;
  const int64_t e0 = ra ? RA.e0[q] : T.row_ptr[s];
  int64_t lo = 0, len = 0;
  if (i < r) {
    lo = T.sv_ptr[e0 + i];
    len = T.sv_ptr[e0 + i + 1] - lo;
  }
  const double init = (i < r && k == 0) ? fwd_init(T, s, i, w, f0, b) : 0.0;
  // wave 0's pivots and the caller's positions, and the panel: loaded with everything else, except
  // right after a factorisation whose root tail ran on the side stream (nrd > 0: after the gather,
  // the tail's done flags and the acquire)
  double dpiv[3];
  int pj[3];
  auto factor_loads = [&]() {
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int j = min(lane + 64 * h, max(w - 1, 0));
      dpiv[h] = (tid < 64) ? Dg[f0 + j] : 1.0;
      pj[h] = (tid < 64) ? T.perm[f0 + j] : 0;
    }
    stage_rowmajor<RSN>(arena + loff, Ls, r, w, ldt);
  };
  if (nrd == 0) factor_loads();
  double c = 0.0;
  const int64_t q4 = len >> 2;
  for (int64_t m0 = 0; m0 < q4; m0 += 16) {  // 16 loads in flight (ex10's root rows: ~14 per thread)
    double x[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) x[u] = T.gbuf[lo + 4 * min(m0 + u, max(q4 - 1, (int64_t)0)) + k];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (m0 + u < q4) c += x[u];
  }
  if (k == 0)
    for (int64_t p = 4 * q4; p < len; ++p) c += T.gbuf[lo + p];
  if (i < r) {
    part[4 * i + k] = c;
    if (k == 0) inits[i] = init;
  }
  if (dg && tid == 0) dg[1] = wall_clock64();
  if (nrd > 0) {  // the root tail on the side stream (LDLSolver::root_async_): every root factorised
    if (tid < 64) {
      int spins = 0;
      for (;;) {
        const bool ok = lane >= nrd ||
                        __hip_atomic_load(rdone + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == repoch;
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 25)) {
          if (lane == 0) atomicOr(T.err, kErrHandoff);
          break;
        }
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (dg && tid == 0) dg[2] = wall_clock64();
    factor_loads();
  }
  __syncthreads();  // the panel and the partial sums
  if (dg && tid == 0) {
    if (nrd == 0) dg[2] = dg[1];
    dg[3] = wall_clock64();
  }
  if (tid < 64) {
    double v[3];
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int ii = lane + 64 * h;
      v[h] = (ii < r) ? ((part[4 * ii] + part[4 * ii + 1]) + (part[4 * ii + 2] + part[4 * ii + 3])) + inits[ii] : 0.0;
    }
    fwd_subst_t(v, Ls, ldt, r, w, lane);
    if (dg && tid == 0) dg[4] = wall_clock64();
#pragma unroll
    for (int h = 0; h < 3; ++h) v[h] = (lane + 64 * h < w) ? v[h] / dpiv[h] : 0.0;
    bwd_subst_t(v, Ls, ldt, w, lane);
    if (dg && tid == 0) dg[5] = wall_clock64();
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int j = lane + 64 * h;
      if (j < w) {
        st_sc1(xi + f0 + j, v[h]);
        if (T.wout[s]) b[pj[h]] = v[h];
      }
    }
    publish_sc1(&tflags[s], epoch + 1);  // the backward epoch: k_bwd_tree's children of the root wait on it
    if (dg && tid == 0) dg[6] = wall_clock64();
  }
}

__global__ __launch_bounds__(NT) void k_bwd_tree(FrontTab T, const int32_t* __restrict__ cptr, const int32_t* __restrict__ clist,
                                                 int nt, const int32_t* __restrict__ pdep, int32_t* counter, int32_t* tflags,
                                                 int epoch, const double* __restrict__ arena,
                                                 const double* __restrict__ D, double* xi, double* __restrict__ out,
                                                 int32_t* err, const uint8_t* __restrict__ rootbwd,
                                                 const uint8_t* __restrict__ tchunk) {
  extern __shared__ __attribute__((aligned(16))) double Ls[];
  __shared__ double xbs[SMALL_SOLVE_MAX];
  __shared__ double bpart[3][64];  // waves 1..3: their share of the update rows' products (w <= 64)
  __shared__ int s_task;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_task = atomicAdd(counter, 1);
    if (s_task == nt - 1) atomicExch(counter, 0);  // every ticket taken: ready for the next launch
  }
  __syncthreads();
  const int t = s_task;  // backward ticket t = forward task nt - 1 - t (reverse topological order)
  if (t >= nt) return;
  const int tf = nt - 1 - t;
  if (rootbwd[tf]) return;  // solved and published by k_fwd_tree
  const int q0 = cptr[tf], q1 = cptr[tf + 1];
  const int lane = tid & 63;
  for (int q = q1 - 1; q >= q0; --q) {  // top first
    const int s = clist[q];
    const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
    if (tchunk[s]) {  // chunked front: panel streamed, double-buffered
      bwd_med_front(T, s, arena, D, Ls, xi, out, pdep, t, tflags, epoch, err);
      continue;
    }
    const int ldc = tree_ldc(r);
    stage_colmajor(arena + T.l_off[s], Ls, r, w, ldc);
    const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
    const int nb = r - w;
    double own[3];  // this front's forward values (previous launch): plain loads, unconditional from
                    // clamped rows (loads under the mask compiled into a wait each), masked after
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int jc = min(lane + 64 * h, max(w - 1, 0));
      own[h] = xi[f0 + jc] / D[f0 + jc];
    }
#pragma unroll
    for (int h = 0; h < 3; ++h) own[h] = (tid < 64 && lane + 64 * h < w) ? own[h] : 0.0;
    static_assert(SMALL_SOLVE_MAX < NT, "k_bwd_tree: one update row per thread");
    const int rk = (tid < nb) ? rows[w + tid] : 0;  // symbolic: loaded before the wait
    int pj[3];  // wave 0: the caller's positions of its pivots
#pragma unroll
    for (int h = 0; h < 3; ++h) pj[h] = (tid < 64 && lane + 64 * h < w) ? T.perm[f0 + lane + 64 * h] : 0;
    const bool wo = T.wout[s];
    if (q == q1 - 1 && tid < 64 && pdep[t] >= 0) poll_deps(pdep, t, t + 1, tflags, epoch, err);
    __syncthreads();  // + the previous (parent) front's drained x stores
    if (tid < nb) xbs[tid] = ld_sc1(xi + rk);
    __syncthreads();
    // the update rows' products L(w + k, j) x_k: for a front of <= 64 pivots and >= 64 update rows the
    // four waves each take a quarter of the rows (ex10's level 1-3 fronts: 70-128 rows, one column per
    // lane) and wave 0 adds the parts in wave order; else wave 0 alone, three columns per lane
    const bool split = w <= 64 && nb >= 64;  // uniform
    double part = 0.0;
    if (split) {
      const int wv = tid >> 6, kb0 = (nb * wv) >> 2, kb1 = (nb * (wv + 1)) >> 2;
      const int cj = min(lane, w - 1);
      double a0 = 0.0, a1 = 0.0;
      int k = kb0;
      for (; k + 1 < kb1; k += 2) {
        a0 = fma(Ls[(w + k) + cj * ldc], xbs[k], a0);
        a1 = fma(Ls[(w + k + 1) + cj * ldc], xbs[k + 1], a1);
      }
      if (k < kb1) a0 = fma(Ls[(w + k) + cj * ldc], xbs[k], a0);
      part = a0 + a1;
      if (wv > 0) bpart[wv - 1][lane] = part;
      __syncthreads();
    }
    if (tid < 64) {
      int cj[3];
#pragma unroll
      for (int h = 0; h < 3; ++h) cj[h] = min(lane + 64 * h, w - 1);
      double acc[3][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
      if (split) {
        acc[0][0] = ((part + bpart[0][lane]) + bpart[1][lane]) + bpart[2][lane];
      } else {
        for (int k8 = 0; k8 < nb; k8 += 8) {
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const int k = k8 + kk;
            if (k < nb) {
              const double x = xbs[k];
#pragma unroll
              for (int h = 0; h < 3; ++h) acc[h][kk & 1] = fma(Ls[(w + k) + cj[h] * ldc], x, acc[h][kk & 1]);
            }
          }
        }
      }
      double v[3];
#pragma unroll
      for (int h = 0; h < 3; ++h) v[h] = (lane + 64 * h < w) ? own[h] - (acc[h][0] + acc[h][1]) : 0.0;
      bwd_subst_c(v, Ls, ldc, w, lane);
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int j = lane + 64 * h;
        if (j < w) {
          st_sc1(xi + f0 + j, v[h]);
          if (wo) out[pj[h]] = v[h];
        }
      }
      publish_sc1(&tflags[s], epoch);  // tasks whose top hangs below s poll it
    }
    __syncthreads();  // wave 0 is done with Ls; its stores are drained
  }
}

// ------------------------------------------------------------------ sharding (SURVEY §8 e)
// External forward contribution of the top fronts: task = (top front, 256-row chunk); xch[xoff + i] =
// (shard 0: own right-hand side entry) + this shard's subtree-root update vectors, child order.
__global__ __launch_bounds__(NT) void k_ext_gather(FrontTab T, const int32_t* __restrict__ list, int shard0,
                                                   const int64_t* __restrict__ sx_ptr, const int64_t* __restrict__ sx_src,
                                                   const double* __restrict__ b, const double* __restrict__ uvec,
                                                   double* __restrict__ xch) {
  int s, chunk;
  task_of(list, s, chunk);
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int i = chunk * NT + threadIdx.x;
  if (i >= r) return;
  const int64_t e = T.xoff[s] + i;
  double v = (shard0 && i < w) ? b[T.perm[f0 + i]] : 0.0;
  for (int64_t p = sx_ptr[e]; p < sx_ptr[e + 1]; ++p) v += uvec[sx_src[p]];
  xch[e] = v;
}

// status of this shard's subtrees -> its slot (other slots 0), all-reduced with the top fronts
__global__ void k_pack_status(const LDLStatus* st, double* slots, int shard, int nshards) {
  const int q = threadIdx.x;
  if (q >= nshards) return;
  const bool me = q == shard;
  slots[4 * q + 0] = me ? (double)st->fail_pivot : 0.0;
  slots[4 * q + 1] = me ? (double)st->npos : 0.0;
  slots[4 * q + 2] = me ? (double)st->nneg : 0.0;
  slots[4 * q + 3] = me ? (double)st->nzero : 0.0;
}

// Top-front exchange buffer (sharded factorisation): only the lower triangles of the top fronts
// (plus the status slots) travel through the all-reduce — half the bytes of the full r x r blocks.
// One workgroup per top-front column: col[3 c] = arena offset of F(c, c), col[3 c + 1] = packed
// offset, col[3 c + 2] = length r - c.
__global__ __launch_bounds__(NT) void k_tri_pack(const int64_t* __restrict__ col, const double* __restrict__ arena,
                                                 double* __restrict__ xp, int dir) {
  const int64_t a = col[3 * blockIdx.x], p = col[3 * blockIdx.x + 1], n = col[3 * blockIdx.x + 2];
  for (int64_t i = threadIdx.x; i < n; i += NT) {
    if (dir == 0)
      xp[p + i] = arena[a + i];
    else
      const_cast<double*>(arena)[a + i] = xp[p + i];
  }
}

__global__ void k_unpack_status(LDLStatus* st, const double* slots, int nshards) {
  double f = (double)INT_MAX, p = 0, ng = 0, z = 0;
  for (int q = 0; q < nshards; ++q) {
    f = fmin(f, slots[4 * q]);
    p += slots[4 * q + 1];
    ng += slots[4 * q + 2];
    z += slots[4 * q + 3];
  }
  st->fail_pivot = (int)f;
  st->npos = (int)p;
  st->nneg = (int)ng;
  st->nzero = (int)z;
}

struct BufList {
  double* p[16];
};
__global__ __launch_bounds__(NT) void k_local_allreduce(BufList B, int nbuf, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    double v = 0.0;
    for (int q = 0; q < nbuf; ++q) v += B.p[q][i];
    for (int q = 0; q < nbuf; ++q) B.p[q][i] = v;
  }
}

// Sharded solve, solution exchange: slice `me` of g <- this shard's subtree x (caller positions
// gidx), every other slice <- 0 (so that a sum all-reduce can stand in for the all-gather) ...
__global__ __launch_bounds__(NT) void k_gather_pack(const int32_t* gidx, int64_t n, int64_t per, int me,
                                                    const double* b, double* g) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int32_t p = gidx[i];
    g[i] = (i / per == me && p >= 0) ? b[p] : 0.0;
  }
}
// ... and after the gather, the other shards' x into the caller's vector
__global__ __launch_bounds__(NT) void k_gather_scatter(const int32_t* gidx, int64_t n, int64_t per, int me,
                                                       const double* g, double* b) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int32_t p = gidx[i];
    if (i / per != me && p >= 0) b[p] = g[i];
  }
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace

LDLSolver::LDLSolver(int n, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& sopt,
                     double ptol, const int32_t* user_perm, Comm* comm)
    : pivot_tol(ptol), comm_(comm) {
  PhaseClock clk("LDLSolver");
  symbolic_analyze(n, colptr, rowval, sopt, user_perm, S_);
  clk("symbolic_analyze");
  const SymbolicPlan& S = S_;
  MADIPM_REQUIRE(S.nshards == 1 || comm == nullptr || (comm->size == S.nshards && comm->rank == S.shard),
                 "communicator does not match the shard layout");
  first_.upload(S.first);
  nrows_.upload(S.nrows);
  row_ptr_.upload(S.row_ptr);
  rows_.upload(S.rows);
  l_off_.upload(S.l_off);
  u_off_.upload(S.u_off);
  {  // a small tree front whose parent is a tree front stores its update block packed lower
     // (u (u + 1) / 2, column-major; u_ld 0 on the device): written by k_fact_tree's write-out and read
     // only by its tree parent's push (or a medium parent's add) — about half the square block's lines
    std::vector<int32_t> uld(S.u_ld);
    for (int f = 0; f < S.nsuper; ++f) {
      const int p = S.parent[f];
      if (!S.ftree.empty() && S.ftree[f] && S.nrows[f] <= SymbolicPlan::kFactTreeMax && p >= 0 && S.ftree[p] &&
          S.nrows[f] > S.first[f + 1] - S.first[f])
        uld[f] = 0;
    }
    u_ld_.upload(uld);
  }
  uvec_off_.upload(S.uvec_off);
  asm_ptr_.upload(S.asm_ptr);
  asm_src_.upload(S.asm_src);
  asm_dst64_.upload(S.asm_dst);
  child_ptr_.upload(S.child_ptr);
  child_list_.upload(S.child_list);
  rel_ptr_.upload(S.rel_ptr);
  rel_.upload(S.rel);
  perm_.upload(S.perm);
  T_.first = first_;
  {
    const char* ek = std::getenv("MADIPM_BIG_KPAN");  // panels per deferred big-front update group
    big_kpan_ = ek ? std::max(1, std::min(8, std::atoi(ek))) : 4;
    const char* es = std::getenv("MADIPM_UPD_SPLIT");  // A/B: 0 = one workgroup per k_big_upd128 tile
    upd_split_ = !(es && es[0] == '0');
    const char* ec = std::getenv("MADIPM_BIG_DAG");  // A/B: 0 = one launch per panel step and kind
    big_dag_ = !(ec && ec[0] == '0');
    // persistent workgroups of the big-front solve kernels (2 per CU; MADIPM_BIG_SOLVE_WG for A/B)
    if (const char* eg = std::getenv("MADIPM_BIG_SOLVE_WG")) big_solve_wg_ = std::max(64, std::atoi(eg));
    // pipelined in-LDS factorisation schedule (1, default); 0 = the barrier schedule, bitwise the same
    // factor (test_ldl_fact_pipe_bitwise)
    const char* ep = std::getenv("MADIPM_FACT_PIPE");
    T_.fpipe = (ep && ep[0] == '0') ? 0 : 1;
    const char* ef = std::getenv("MADIPM_DEBUG_PIPE_FAULT");  // tests: drop one hand-off (sticky error)
    T_.pipe_fault = (ef && ef[0] == '1') ? 1 : 0;
    // the assembly's device-side source-count check (MADIPM_DEBUG_ASM_SRC_CAP=<n>, tests only: a
    // smaller bound, so the check fires)
    T_.asm_src_cap = kAsmLdsSrc * kAsmLdsWinMax;
    if (const char* e = std::getenv("MADIPM_DEBUG_ASM_SRC_CAP")) T_.asm_src_cap = std::atoi(e);
  }
  T_.nrows = nrows_;
  T_.row_ptr = row_ptr_;
  T_.rows = rows_;
  T_.l_off = l_off_;
  T_.u_off = u_off_;
  T_.u_ld = u_ld_;
  T_.uvec_off = uvec_off_;
  T_.asm_ptr = asm_ptr_;
  T_.asm_src = asm_src_;
  T_.asm_dst = asm_dst64_;
  T_.child_ptr = child_ptr_;
  T_.child_list = child_list_;
  T_.rel_ptr = rel_ptr_;
  T_.rel = rel_;
  T_.perm = perm_;
  fs_off_.upload(S.fs_off);
  sv_ptr_.upload(S.sv_ptr);
  sv_src_.upload(S.sv_src);
  sv_nt_.alloc(std::max<int64_t>(S.row_ptr[S.nsuper], 1));  // the tree solve's split (set with its tables)
  sv_nt_.zero();
  // g_ptr_, atiles_: with the big-child records below (bt renumbered, source-path tiles)
  {
    // int32 sources when every arena / K index fits (leaf update blocks stay materialised: forming
    // them from the leaves' L panels in the gather was measured slower, r1 — 6 scattered loads per
    // source instead of 1)
    // (the check and the narrowing on the analysis threads: ~170 M sources on neos)
    const int64_t ns = (int64_t)S.g_src.size();
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(analysis_threads(), ns / 4000000));
    hvec<int32_t> g32(ns);
    std::atomic<bool> fits{ns > 0};
    {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
          const int64_t q0 = ns * t / T, q1 = ns * (t + 1) / T;
          bool ok = true;
          for (int64_t q = q0; q < q1; ++q) {
            const int64_t v = S.g_src[q];
            ok = ok && v >= INT32_MIN && v < (1LL << 30);
            g32[q] = (int32_t)v;
          }
          if (!ok) fits = false;
        });
      for (auto& x : th) x.join();
    }
    if (fits) {
      g_src32_.upload(g32);
    } else {
      g_src_.upload(S.g_src);
    }
  }
  g_chunk_.upload(S.g_chunk);
  gpart_.alloc(std::max<size_t>(S.g_chunk.size(), 1));
  std::vector<int64_t> asm_cid_off;  // per assembly group: its chunk-path chunks' range in chunk_ids_
  {  // big-child records of the assembly tiles (BigChildRec): a bt entry's block, split into column
     // ranges of <= kBigRecEntries entries; the tiles' bt0 / bt1 renumbered to the records
    const int64_t nb = (int64_t)S.bt.size() / 5;
    std::vector<int64_t> rptr(nb + 1, 0);
    for (int64_t k = 0; k < nb; ++k) {
      const int32_t* e = &S.bt[5 * k];
      const int na = e[4] - e[3], nbt = e[2] - e[1], cpr = kBigRecEntries / na;
      MADIPM_REQUIRE(na >= 1 && na <= 64 && nbt >= 1 && nbt <= 64, "assembly: big-child block outside its tile");
      rptr[k + 1] = rptr[k] + (nbt + cpr - 1) / cpr;
    }
    MADIPM_REQUIRE(rptr[nb] < INT32_MAX, "assembly: too many big-child records");
    std::vector<BigChildRec> br(std::max<int64_t>(rptr[nb], 1));
    const int T = (int)std::min<int64_t>(analysis_threads(), std::max<int64_t>(1, nb / 4096));
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        for (int64_t k = t; k < nb; k += T) {
          const int32_t* e = &S.bt[5 * k];
          const int c = e[0], b0 = e[1], b1 = e[2], a0 = e[3], a1 = e[4];
          const int32_t* rel = S.rel.data() + S.rel_ptr[c];
          const int I0 = rel[a0] & ~63, J0 = rel[b0] & ~63;
          const int na = a1 - a0, cpr = kBigRecEntries / na;
          for (int64_t q = rptr[k]; q < rptr[k + 1]; ++q) {
            BigChildRec& R = br[q];
            R = BigChildRec{};
            R.u_off = S.u_off[c];
            R.u_ld = S.u_ld[c];
            R.a0 = a0;
            R.b0 = b0 + (int)(q - rptr[k]) * cpr;
            R.na = (uint16_t)na;
            R.nb = (uint16_t)std::min(cpr, b1 - R.b0);
            R.na_inv = (65536u + na - 1) / na;
            for (int i = 0; i < na; ++i) R.rows[i] = (uint8_t)(rel[a0 + i] - I0);
            for (int j = 0; j < R.nb; ++j) R.cols[j] = (uint8_t)(rel[R.b0 + j] - J0);
          }
        }
      });
    for (auto& x : th) x.join();
    brec_.upload(br);
    std::vector<SymbolicPlan::AsmTile> at(S.atiles);
    for (auto& a : at) {
      a.bt0 = (int32_t)rptr[a.bt0];
      a.bt1 = (int32_t)rptr[a.bt1];
      // the tile's nonempty-entry count rides in gptr's top 16 bits (asm_chunks_lds: no load of it)
      MADIPM_REQUIRE(a.gptr < ((int64_t)1 << 47), "assembly: entry list offset past 2^47");
      if (a.gptr >= 0) a.gptr |= (int64_t)S.g_ptr[a.gptr] << 48;
    }
    // Tiles of <= kAsmLdsWin windows of sources sum them from LDS (asm_chunks_lds): their entry lists point at
    // sources (pos | first source << 12, then the count << 12), gptr bit 47 set, gchk = the first
    // source | the count << 48; the chunk pass keeps only the other tiles' chunks (chunk_ids_, per
    // assembly group).  MADIPM_ASM_LDS_SRC=0: every tile through the chunk pass (A/B).
    const char* el = std::getenv("MADIPM_ASM_LDS_SRC");
    const bool lds_src = !(el && el[0] == '0');
    int force_win = 0;  // tests: every tile of <= n windows on the LDS source path (no launch-size rule)
    if (const char* ew = std::getenv("MADIPM_ASM_LDS_WIN")) force_win = std::max(0, std::min(kAsmLdsWinMax, std::atoi(ew)));
    std::vector<int32_t> gp2(S.g_ptr);
    std::vector<int64_t> cids;
    int64_t st_lds = 0, st_multi = 0, st_straddle = 0, st_chunk = 0, st_nsmax = 0;  // MADIPM_ASM_STATS
    asm_cid_off.assign(S.atile_lev.size(), 0);
    for (size_t g = 0; g + 1 < S.atile_lev.size(); ++g) {
      asm_cid_off[g] = (int64_t)cids.size();
      for (int32_t t = S.atile_lev[g]; t < S.atile_lev[g + 1]; ++t) {
        const SymbolicPlan::AsmTile& a0 = S.atiles[t];
        if (a0.gptr < 0) continue;
        const int32_t ne = S.g_ptr[a0.gptr];
        const int64_t nchk = S.g_ptr[a0.gptr + ne + 1] >> 12, cb = a0.gchk;
        const int64_t sb = S.g_chunk[cb], ns = S.g_chunk[cb + nchk] - sb;
        // one window in k_assemble's launches of < 256 tiles (LDLSolver::run_fact's one-tile-per-CU
        // instance), kAsmLdsWin elsewhere (k_asm_update: the tiles past the group's fused-front mark)
        const int32_t aend = (int)g < S.nlevels ? S.atile_fz1[g] : S.atile_lev[g + 1];
        const int64_t nwin = force_win ? force_win : (t < aend && aend - S.atile_lev[g] < 256) ? 1 : kAsmLdsWin;
        if (lds_src && ns <= kAsmLdsSrc * nwin && sb < ((int64_t)1 << 48)) {
          for (int32_t k = 0; k < ne; ++k) {
            const int32_t e = S.g_ptr[a0.gptr + 1 + k];
            gp2[a0.gptr + 1 + k] = (e & 4095) | (int32_t)((S.g_chunk[cb + (e >> 12)] - sb) << 12);
          }
          gp2[a0.gptr + ne + 1] = (int32_t)(ns << 12);
          at[t].gptr |= (int64_t)1 << 47;
          at[t].gchk = sb | (ns << 48);
          ++st_lds;
          st_multi += ns > kAsmLdsSrc;
          st_nsmax = std::max(st_nsmax, ns);
          for (int32_t k = 0; k < ne; ++k) {  // entries whose sources cross a window boundary
            const int64_t a = gp2[a0.gptr + 1 + k] >> 12, b = gp2[a0.gptr + 2 + k] >> 12;
            st_straddle += b > a && a / kAsmLdsSrc != (b - 1) / kAsmLdsSrc;
          }
        } else {
          for (int64_t c = cb; c < cb + nchk; ++c) cids.push_back(c);
          ++st_chunk;
        }
      }
    }
    asm_cid_off.back() = (int64_t)cids.size();
    if (std::getenv("MADIPM_ASM_STATS"))
      fprintf(stderr, "asm lds-src: tiles %lld (multi-window %lld, straddling entries %lld, max sources %lld)  chunk-path tiles %lld\n",
              (long long)st_lds, (long long)st_multi, (long long)st_straddle, (long long)st_nsmax, (long long)st_chunk);
    g_ptr_.upload(gp2);
    chunk_ids_.upload(cids);
    atiles_.upload(at);
  }
  fscratch_.alloc(std::max<int64_t>(S.fs_size, 1));
  T_.fs_off = fs_off_;
  {
    // fronts staged into LDS by k_fact_tree (all sizes) and k_small_blocked (r > 32, not big, not a
    // batched-leaf parent, whose SYRK writes ld r) are pre-assembled as their LDS image
    std::vector<uint8_t> img(std::max<size_t>(S.nrows.size(), 1), 0);
    std::vector<uint8_t> lbpar(S.nrows.size(), 0);
    for (const auto& G : S.lb) lbpar[G.parent] = 1;
    for (size_t f = 0; f < S.nrows.size(); ++f)
      img[f] = (S.fs_off[f] >= 0 &&
                (S.ftree[f] ? !S.absorb[f] : (!S.is_big[f] && !lbpar[f] && S.nrows[f] > 32))) ? 1 : 0;
    fs_img_.upload(img);
    T_.fs_img = fs_img_;
  }
  T_.sv_ptr = sv_ptr_;
  T_.sv_src = sv_src_;
  T_.sv_nt = sv_nt_;
  const int ns = S.nsuper, NL = S.nlevels;
  {
    std::vector<int32_t> slot(std::max(ns, 1), -1);
    int nslot = 0;
    for (int s = 0; s < ns; ++s)
      if (S.is_big[s]) slot[s] = nslot++;
    bigslot_.upload(slot);
    minv_.alloc((int64_t)std::max(nslot, 1) * 4096);
    T_.bigslot = bigslot_;
  }
  // sharding tables (unsharded: xoff = -1, every x written, every column counted)
  {
    std::vector<int64_t> xo(std::max(ns, 1), -1);
    std::vector<uint8_t> wo(std::max(ns, 1), 1), cm(std::max(S.N, 1), 1);
    // solution exchange: every shard writes the top x it computes redundantly; the subtree x are
    // all-gathered by shard slices (the partition is shard-independent, so every shard knows them all)
    std::vector<int32_t> gi;
    if (S.nshards > 1) {
      std::vector<std::vector<int32_t>> own(S.nshards);
      for (int s = 0; s < ns; ++s) {
        xo[s] = S.xoff[s];
        for (int j = S.first[s]; j < S.first[s + 1]; ++j) {
          cm[j] = S.top(s) ? 2 : (S.mine(s) ? 1 : 0);
          if (!S.top(s)) own[S.owner[s]].push_back(S.perm[j]);
        }
      }
      for (const auto& o : own) gper_ = std::max<int64_t>(gper_, (int64_t)o.size());
      gper_ = std::max<int64_t>(gper_, 1);
      gi.assign((size_t)(S.nshards * gper_), -1);
      for (int q = 0; q < S.nshards; ++q) std::copy(own[q].begin(), own[q].end(), gi.begin() + q * gper_);
    }
    gidx_.upload(gi.empty() ? std::vector<int32_t>{-1} : gi);
    gsol_.alloc(std::max<int64_t>(S.nshards * gper_, 1));
    xoff_.upload(xo);
    wout_.upload(wo);
    colmask_.upload(cm);
    xch_.alloc(std::max<int64_t>(S.xlen, 1));
    sx_ptr_.upload(S.sx_ptr.empty() ? std::vector<int64_t>{0} : S.sx_ptr);
    sx_src_.upload(S.sx_src.empty() ? std::vector<int64_t>{0} : S.sx_src);
    T_.xoff = xoff_;
    T_.xch = xch_;
    T_.wout = wout_;
  }
  auto lb_member = [&](int s) { return !S.lb_of.empty() && S.lb_of[s] >= 0; };
  // solve classes: fronts up to SMALL_SOLVE_MAX rows whose L panel fits in LDS take the one-launch
  // workgroup-per-front kernels; larger ones the dependency-driven big-front kernels
  auto solve_small = [&](int s) {
    const int r = S.nrows[s], w = S.first[s + 1] - S.first[s];
    return r <= SMALL_SOLVE_MAX && 8 * (r | 1) * w <= 150 * 1024;
  };
  auto in_phase = [&](int s, int phase) {
    if (lb_member(s)) return false;  // batched leaves: W build + the parent's SYRK + GEMV solves
    return phase == 1 ? (!S.top(s) && S.mine(s)) : S.top(s);
  };
  auto tree_panel_doubles = [&](int s) {  // max(forward row-major, backward col-major) staged panel
    const int r = S.nrows[s], w = S.first[s + 1] - S.first[s];
    const int ldt = ((w + 15) & ~15) + 2, ldc = ((r + 31) & ~31) + 2;
    return std::max<int64_t>((int64_t)r * ldt, (int64_t)w * ldc);
  };
  // tree solve set (k_fwd_tree / k_bwd_tree); MADIPM_TREE_SOLVE=0 disables it (A/B measurements)
  std::vector<char> in_tree(std::max(ns, 1), 0);
  {
    const char* ev = std::getenv("MADIPM_TREE_SOLVE");
    const bool on = !(ev && ev[0] == '0');
    std::vector<char> lbpar(std::max(ns, 1), 0);
    for (const auto& G : S.lb) lbpar[G.parent] = 1;
    auto preleaf = [&](int c) { return S.child_ptr[c] == S.child_ptr[c + 1] && S.nrows[c] <= 32; };
    // fronts whose whole panel (+ 8 KB of gather staging) does not fit TREE_SOLVE_LDS, medium fronts
    // (SMALL_SOLVE_MAX < r <= MED_SOLVE_MAX) included, join with their panel streamed in chunks
    for (int s = 0; on && s < ns; ++s) {  // postorder: children first
      if (!in_phase(s, 1) || preleaf(s) || lbpar[s] || S.nrows[s] > MED_SOLVE_MAX) continue;
      bool ok = true;
      for (int q = S.child_ptr[s]; q < S.child_ptr[s + 1] && ok; ++q) {
        const int c = S.child_list[q];
        ok = in_tree[c] || (preleaf(c) && in_phase(c, 1));
      }
      in_tree[s] = ok;
    }
  }
  // micro leaves (w <= 2, r <= 32, no children) under tree fronts, solved from precomputed leaf records
  // (SolveLeaf) by the flat k_fwd_leaves / k_bwd_leaves launches (r3: solving them inside the tree tasks,
  // or their backward only, measured slower: 1478 vs 1534 iters/s)
  std::vector<char> sleaf(std::max(ns, 1), 0);
  {
    for (int c = 0; c < ns; ++c) {
      const int p = S.parent[c];
      sleaf[c] = p >= 0 && in_tree[p] && in_phase(c, 1) && S.child_ptr[c] == S.child_ptr[c + 1] && S.nrows[c] <= 32 &&
                 S.first[c + 1] - S.first[c] <= 2;
    }
  }
  // ---- batched leaf columns
  lb_at_level_.assign(std::max(NL, 1), {});
  if (!S.lb.empty()) {
    lbg_.upload(S.lb);
    lbmem_.upload(S.lb_mem);
    std::vector<int32_t> gid(S.lb_mem.size()), xrow;
    std::vector<int64_t> poff;
    int64_t np = 0;
    for (size_t g = 0; g < S.lb.size(); ++g) {
      const auto& G = S.lb[g];
      for (int j = 0; j < G.n; ++j) gid[G.mem_off + j] = (int32_t)g;
      for (int k = 0; k < G.m; ++k) xrow.push_back(S.rows[S.row_ptr[G.parent] + S.lb_gpos[G.gpos_off + k]]);
      poff.push_back(np);
      np += (int64_t)cdiv(G.n, LBF_COLS) * G.m;
      lb_at_level_[S.level[G.parent]].push_back((int)g);
    }
    lbgid_.upload(gid);
    lbxrow_.upload(xrow);
    lbpoff_.upload(poff);
    lbcs_.upload(S.lb_cs);
    lbce_.upload(S.lb_ce);
    lbwbase_.upload(S.lb_wbase);
    lbwrow_.upload(S.lb_wrow);
    lbgpos_.upload(S.lb_gpos);
    lbW_.alloc(std::max<int64_t>(S.lb_wsize, 1));
    lbW_.zero();  // the pattern is fixed: entries outside it stay 0
    lbd_.alloc(2 * S.lb_mem.size());
    lbpart_.alloc(std::max<int64_t>(np, 1));
  }

  clk("tables + uploads");
  // ---- factorisation tree tables (k_fact_tree)
  {
    std::vector<int32_t> ord(S.ft_order), dptr{0}, dl;  // ticket order (SymbolicPlan::ft_order)
    nftree_ = (int)ord.size();
    for (int s : ord) {
      for (int q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q)
        if (S.ftree[S.child_list[q]]) dl.push_back(S.child_list[q]);
      dptr.push_back((int32_t)dl.size());
      const int r = S.nrows[s], w = S.first[s + 1] - S.first[s], u = r - w;
      const bool sq = r <= 128 && !S.fold_pk[s];
      if (r > SymbolicPlan::kFactTreeMax)  // medium front: one panel (r | 1) x min(64, w) in LDS
        ftree_lds_ = std::max<int>(ftree_lds_, 8 * (((r | 1) * std::min(64, w) + 1) & ~1));
      else
      ftree_lds_ = std::max<int>(ftree_lds_, (sq ? 8 * ((r * (r | 1) + 1) & ~1) : 8 * ((r * (r + 1) / 2 + 1) & ~1)) +
                                                 (S.absorb[s] ? SymbolicPlan::kFoldRowBytes * S.fold_rmax[s] +
                                                                    SymbolicPlan::kFoldLeafBytes * S.fold_lmax[s]
                                                              : 0));
      // folded leaves: their K entries read, their L entries written
      for (int k = S.absorb[s] ? S.mc_ptr[s] : 0; k < (S.absorb[s] ? S.mc_ptr[s + 1] : 0); ++k) {
        const int c = S.mc_list[k];
        const double rc = S.nrows[c], wc = S.first[c + 1] - S.first[c];
        ftree_bytes_ += 12.0 * (S.asm_ptr[c + 1] - S.asm_ptr[c]) + 8.0 * (rc * wc - wc * (wc - 1) / 2.0);
        ftree_alg_ += fact_alg(c);
        for (int t = 0; t < (int)wc; ++t) ftree_flops_ += (rc - t - 1) * (rc - t);
      }
      // staging model: the stored lower trapezoid of the panel written and the front's scatter list
      // read (ftree_bytes_); SURVEY 8(d)'s algorithmic bytes (B_fact = 8 nnzL + 12 nnzK of the
      // front's columns, exact column counts) in ftree_alg_
      (void)u;
      ftree_bytes_ += 8.0 * (r * (double)w - w * (w - 1) / 2.0) + 12.0 * (double)(S.asm_ptr[s + 1] - S.asm_ptr[s]);
      ftree_alg_ += fact_alg(s);
      for (int t = 0; t < w; ++t) ftree_flops_ += (double)(r - t - 1) * (r - t);
    }
    if (const char* ev = std::getenv("MADIPM_TREE_DEBUG"); ev && ev[0] == '1') {  // per-level front shapes
      std::map<int, std::array<double, 7>> lv;  // count, sum r, max r, sum w, sum lds, max lds, sum leaves
      for (int s : ord) {
        const int r = S.nrows[s], w = S.first[s + 1] - S.first[s];
        const bool sq = r <= 128 && !S.fold_pk[s];
        const double lds = (sq ? 8.0 * r * (r | 1) : 4.0 * r * (r + 1)) +
                           (S.absorb[s] ? SymbolicPlan::kFoldRowBytes * S.fold_rmax[s] + SymbolicPlan::kFoldLeafBytes * S.fold_lmax[s] : 0);
        auto& a = lv[S.level[s]];
        a[0] += 1, a[1] += r, a[2] = std::max<double>(a[2], r), a[3] += w, a[4] += lds, a[5] = std::max(a[5], lds);
        a[6] += S.absorb[s] ? S.mc_ptr[s + 1] - S.mc_ptr[s] : 0;
      }
      for (auto& [l, a] : lv)
        fprintf(stderr, "tree level %d: %4.0f fronts  r avg %.0f max %.0f  w avg %.1f  LDS avg %.0f max %.0f KB  leaves avg %.0f\n", l,
                a[0], a[1] / a[0], a[2], a[3] / a[0], a[4] / a[0] / 1024, a[5] / 1024, a[6] / a[0]);
    }
    // the device-side carve check compares against this (MADIPM_DEBUG_LDS_SHRINK=<bytes>, tests only:
    // pretend the launch has that much less, so the check fires)
    T_.lds_cap = ftree_lds_;
    if (const char* e = std::getenv("MADIPM_DEBUG_LDS_SHRINK")) T_.lds_cap -= std::atoi(e);
    auto up = [](DBuf<int32_t>& d, const std::vector<int32_t>& v) { d.upload(v.empty() ? std::vector<int32_t>{0} : v); };
    clk("  tree tables");
    // fold helpers: a front with two or more leaf batches hands the first half of them to a helper
    // ticket (before every front's; the helpers with the most batches first), folds the rest itself
    // and adds the helper's image after its waits (MADIPM_FOLD_HELP=0: no helpers)
    {
      const char* eh = std::getenv("MADIPM_FOLD_HELP");
      const bool on = !(eh && eh[0] == '0');
      int min_nb = 3;  // fronts of at least this many batches get a helper (MADIPM_FOLD_HELP_MIN: A/B)
      if (const char* em = std::getenv("MADIPM_FOLD_HELP_MIN")) min_nb = std::max(2, std::atoi(em));
      int share4 = 2;  // the helper's share of the batches, in quarters (MADIPM_FOLD_HELP_SHARE: A/B)
      if (const char* es = std::getenv("MADIPM_FOLD_HELP_SHARE")) share4 = std::max(1, std::min(3, std::atoi(es)));
      std::vector<int32_t> help(std::max(ns, 1), -1);
      std::vector<FoldStart> fst(std::max(ns, 1), FoldStart{0, 0, 0, 0, 0, 0, 0, 0, 0});
      auto start = [&](int b0, int b1) {  // batches [b0, b1) and the first one's table entries
        FoldStart F{b0, b1, 0, 0, 0, 0, 0, 0, 0};
        if (b1 > b0) {
          F.kq0 = S.fold_bat[b0];
          F.kq1 = S.fold_bat[b0 + 1];
          F.row0 = S.fold_row0[b0];
          F.row1 = S.fold_row0[b0 + 1];
          F.poff = S.fold_poff[b0];
          F.plen = S.fold_plen[b0];
        }
        return F;
      };
      std::vector<FoldHelp> hv;
      std::vector<uint16_t> hdst;  // per helper: the sorted LDS destinations its batches' products reach
      int64_t img = 0;
      // the run-end entries of a batch's product chunks name every destination it writes (a parked
      // continuation ends at its run's destination too): the image holds exactly those, ascending.
      // Helpers are independent: their lists are built on threads (marks over the 16-bit LDS space,
      // then the distinct ones sorted), then appended in ticket order.
      auto dests = [&](int b0, int b1, std::vector<uint8_t>& mark, std::vector<uint16_t>& out) {
        for (int b = b0; b < b1; ++b) {
          const int64_t po = S.fold_poff[b];
          const int len = S.fold_plen[b];
          for (int t = 0; t < SymbolicPlan::kFoldThreads; ++t) {
            int d = (int)(S.fold_chead[(int64_t)b * SymbolicPlan::kFoldThreads + t] & 0xffffu);
            for (int k = 0; k < len; ++k) {
              const uint32_t e = S.fold_prod[po + (int64_t)SymbolicPlan::kFoldThreads * k + t];
              d += (int)((e >> 24) & 127u);
              if ((int32_t)e < 0) {
                MADIPM_REQUIRE(d >= 0 && d < 65536, "fold helper: LDS destination beyond 16 bits");
                if (!mark[d]) {
                  mark[d] = 1;
                  out.push_back((uint16_t)d);
                }
              }
            }
          }
        }
        std::sort(out.begin(), out.end());
        for (uint16_t x : out) mark[x] = 0;
      };
      if (!S.fold_bptr.empty())
        for (int f = 0; f < ns; ++f) fst[f] = start(S.fold_bptr[f], S.fold_bptr[f + 1]);
      std::vector<std::array<int, 3>> cand;  // (front, first batch, end of the helper's batches), ticket order
      for (int f : ord) {
        if (!on || !S.absorb[f]) continue;
        const int b0 = S.fold_bptr[f], nb = S.fold_bptr[f + 1] - b0;
        if (nb < min_nb) continue;
        cand.push_back({f, b0, b0 + std::max(1, std::min(nb - 1, nb * share4 / 4))});
      }
      std::vector<std::vector<uint16_t>> cd(cand.size());
      {
        std::atomic<size_t> next{0};
        auto work = [&] {
          std::vector<uint8_t> mark(65536, 0);
          for (size_t k; (k = next.fetch_add(1)) < cand.size();) dests(cand[k][1], cand[k][2], mark, cd[k]);
        };
        const int nt = std::max(1, std::min<int>(analysis_threads(), (int)(cand.size() / 8)));
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
      }
      for (size_t k = 0; k < cand.size(); ++k) {
        const int64_t dofs = (int64_t)hdst.size();
        const int32_t nimg = (int32_t)cd[k].size();
        hdst.insert(hdst.end(), cd[k].begin(), cd[k].end());
        hv.push_back(FoldHelp{cand[k][0], 0, img, dofs, nimg, 0, start(cand[k][1], cand[k][2])});
        img += (nimg + 1) & ~1LL;
      }
      std::stable_sort(hv.begin(), hv.end(),
                       [](const FoldHelp& a, const FoldHelp& b) { return a.fs.b1 - a.fs.b0 > b.fs.b1 - b.fs.b0; });
      nfhelp_ = (int)hv.size();
      for (int h = 0; h < nfhelp_; ++h) {
        hv[h].flag = ns + h;
        help[hv[h].front] = h;
        fst[hv[h].front] = start(hv[h].fs.b1, S.fold_bptr[hv[h].front + 1]);  // the front keeps the rest
      }
      fstart_.upload(fst);
      fold_help_.upload(help);
      fhelp_.upload(hv.empty() ? std::vector<FoldHelp>{FoldHelp{0, 0, 0, 0, 0, 0, FoldStart{0, 0, 0, 0, 0, 0, 0, 0, 0}}} : hv);
      fimg_.alloc((size_t)std::max<int64_t>(img, 2));
      fimg_dst_.upload(hdst.empty() ? std::vector<uint16_t>{0} : hdst);
      T_.fimg_dst = fimg_dst_;
      if (std::getenv("MADIPM_TREE_DEBUG"))
        fprintf(stderr, "fold helpers: %d, image entries %lld (%.1f MB per factorisation, stored + read)\n", nfhelp_,
                (long long)hdst.size(), 16e-6 * (double)hdst.size());
      T_.fstart = fstart_;
      T_.fold_help = fold_help_;
      T_.fhelp = fhelp_;
      T_.fimg = fimg_;
      dptr.insert(dptr.begin(), (size_t)nfhelp_, 0);  // dep_ptr by ticket: the helpers' ranges are empty
    }
    clk("  fold helpers");
    up(ft_order_, ord);
    up(ft_dptr_, dptr);
    up(ft_dep_, dl);
    fflags_.alloc(std::max(ns + nfhelp_, 1));
    fflags_.zero();
    {
      auto up8 = [](DBuf<uint8_t>& d, const std::vector<uint8_t>& v) { d.upload(v.empty() ? std::vector<uint8_t>{0} : v); };
      auto up32 = [](DBuf<int32_t>& d, const std::vector<int32_t>& v) { d.upload(v.empty() ? std::vector<int32_t>{0} : v); };
      auto up64 = [](DBuf<int64_t>& d, const std::vector<int64_t>& v) { d.upload(v.empty() ? std::vector<int64_t>{0} : v); };
      up8(absorb_, S.absorb);
      up8(fold_pk_, S.fold_pk);
      up32(mc_ptr_, S.mc_ptr);
      up64(ab_first_, S.ab_first);
      up32(ab_src0_, S.ab_src0);
      up32(ab_src1_, S.ab_src1);
      up32(ab_k_, S.ab_k);
      up32(ab_f0_, S.ab_f0);
      up32(ab_wrc_, S.ab_wrc);
      {
        std::vector<int64_t> lo(S.mc_list.size() + 1, 0);
        for (size_t k = 0; k < S.mc_list.size(); ++k) lo[k] = S.l_off[S.mc_list[k]];
        ab_loff_.upload(lo);
      }
      up32(fold_bptr_, S.fold_bptr);
      up32(fold_bat_, S.fold_bat);
      up64(fold_row0_, S.fold_row0);
      up64(fold_poff_, S.fold_poff);
      up32(fold_plen_, S.fold_plen);
      up32(fold_rmax_, S.fold_rmax);
      up32(fold_lmax_, S.fold_lmax);
      fold_prod_.upload(S.fold_prod.empty() ? std::vector<uint32_t>{SymbolicPlan::kFoldPad} : S.fold_prod);
      fold_chead_.upload(S.fold_chead.empty() ? std::vector<uint32_t>{0u} : S.fold_chead);
      T_.absorb = absorb_;
      T_.fold_pk = fold_pk_;
      T_.mc_ptr = mc_ptr_;
      T_.ab_first = ab_first_;
      T_.ab_src0 = ab_src0_;
      T_.ab_src1 = ab_src1_;
      T_.ab_k = ab_k_;
      T_.ab_f0 = ab_f0_;
      T_.ab_wrc = ab_wrc_;
      T_.ab_loff = ab_loff_;
      T_.fold_bptr = fold_bptr_;
      T_.fold_bat = fold_bat_;
      T_.fold_row0 = fold_row0_;
      T_.fold_poff = fold_poff_;
      T_.fold_plen = fold_plen_;
      T_.fold_rmax = fold_rmax_;
      T_.fold_lmax = fold_lmax_;
      T_.fold_prod = fold_prod_.p;
      T_.fold_chead = fold_chead_.p;
    }
    fcnt_.alloc(4);
    fcnt_.zero();
    const char* dv = std::getenv("MADIPM_TREE_DEBUG");
    if (dv && dv[0] == '1' && nftree_) {
      fdbg_.alloc((int64_t)24 * (nftree_ + nfhelp_));
      fdbg_.zero();
    }
  }

  // ---- factorisation launch schedules (phase 1: this shard's subtrees; phase 2: the top fronts)
  clk("  fold table uploads");
  std::vector<int32_t> sched;
  auto align2 = [&]() {
    if (sched.size() & 1) sched.push_back(0);
  };
  // phase-1 level groups: the fused fronts' tiles past their column block 0 wait for k_asm_update
  auto asm_end = [&](int g) { return g < NL ? S.atile_fz1[g] : S.atile_lev[g + 1]; };
  auto asm_launch = [&](int g, std::vector<Launch>& out) {
    if (asm_end(g) <= S.atile_lev[g]) return;
    Launch L{ASSEMBLE, 0, S.atile_lev[g], 0, asm_end(g) - S.atile_lev[g], asm_cid_off[g],
             asm_cid_off[g + 1] - asm_cid_off[g]};  // the chunks of the group's chunk-path tiles
    // algorithmic traffic: chunk pass reads (index, value) per source, writes one partial per chunk;
    // the tile pass reads the entry offsets + partials (+ big-children blocks), writes the lower tile
    const int64_t nsrc = S.g_chunk[S.chunk_lev[g + 1]] - S.g_chunk[S.chunk_lev[g]];
    L.bytes2 = 16.0 * nsrc + 16.0 * L.nchunk;
    L.flops2 = (double)nsrc;
    for (int32_t t = S.atile_lev[g]; t < asm_end(g); ++t) {
      const SymbolicPlan::AsmTile& at = S.atiles[t];
      const int r = S.nrows[at.front], ti = at.tij & 0xffff, tj = (at.tij >> 16) & 0x7fff;
      const double nr = std::min(64, r - 64 * ti), nc = std::min(64, r - 64 * tj);
      L.bytes += 8.0 * (ti == tj ? nr * (nr + 1) / 2 : nr * nc) * (at.tij < 0 ? 2.0 : 1.0) +
                 (at.gptr >= 0 ? 4.0 * (S.g_ptr[at.gptr] + 2) : 0.0);
      for (int k = at.bt0; k < at.bt1; ++k) {
        const int32_t* e = &S.bt[5 * k];
        for (int b = e[1]; b < e[2]; ++b) L.bytes += 8.0 * std::max(0, e[4] - std::max(b, e[3]));
      }
    }
    L.bytes += 8.0 * L.nchunk;
    out.push_back(L);
  };
  auto lb_syrk_launch = [&](int g, std::vector<Launch>& out) {
    const auto& G = S.lb[g];
    Launch L{LB_SYRK, 0, g, 0, 0};
    L.flops = (double)G.m * (G.m + 1) * (double)G.n;
    // W once + the parent's lower triangle read-modify-written once per K-chunk
    L.bytes = 8.0 * (double)G.m * G.n + 16.0 * (double)G.m * (G.m + 1) / 2.0 * cdiv(G.n, LB_KCHUNK);
    out.push_back(L);
  };
  // The big fronts of a level in one k_big_dag launch: tasks in ticket order DIAG(0) | chain(0) feed(0) |
  // chain(1) bulk(0) feed(1) | chain(2) bulk(1) feed(2) | ... | bulk(last) (k_big_dag's comment), every
  // front of the level interleaved; each task's dependencies are the last earlier writers of the 64 x 64
  // blocks of its front that it reads or read-modify-writes (every writer also reads what it writes, so
  // the last writer stands for all earlier ones).  Then the fused fronts' k_asm_update.  The same tiles,
  // operands and order of sums as the per-step launches with K unsplit.
  std::vector<int32_t> dtask, ddptr{0}, ddlist;  // DagTask words, CSR of dependencies (launch-local tickets)
  std::vector<int64_t> mslot(std::max(S.nsuper, 1), 0);
  int64_t nmslot = 0;
  for (int f = 0; f < S.nsuper; ++f)
    if (S.is_big[f]) {
      mslot[f] = nmslot;
      nmslot += cdiv(S.first[f + 1] - S.first[f], 64) + 1;
    }
  auto dag_level = [&](const std::vector<int32_t>& big, int lev, int phase, std::vector<Launch>& out) {
    const int kp = big_kpan_;
    Launch L{BIG_DAG, 0, (int64_t)(dtask.size() / 4), 0, 0};
    // per front, the live written rectangles bucketed by the 64 x 64 blocks they touch: a task depends on
    // every live rectangle its reads or read-modify-writes intersect; a write drops the rectangles (per
    // block) it covers — it depends on them, so it stands for them — and adds its own
    struct Ent {
      int r0, r1, c0, c1, w;
    };
    std::map<int, std::vector<std::vector<Ent>>> live;
    std::vector<int32_t> deps;
    std::vector<Ent> wr;
    std::vector<int> wrs;
    auto region = [&](int s, int r0, int r1, int c0, int c1, bool write) {
      const int nb = (int)cdiv(S.nrows[s], 64);
      auto& g = live[s];
      if (g.empty()) g.resize((size_t)nb * nb);
      r1 = std::min(r1, S.nrows[s]);
      c1 = std::min(c1, S.nrows[s]);
      if (r0 >= r1 || c0 >= c1) return;
      for (int R = r0 >> 6; R <= (r1 - 1) >> 6; ++R)
        for (int C = c0 >> 6; C <= std::min((c1 - 1) >> 6, R); ++C)
          for (const Ent& e : g[(size_t)R * nb + C])
            if (e.r0 < r1 && r0 < e.r1 && e.c0 < c1 && c0 < e.c1) deps.push_back(e.w);
      if (write) {
        wr.push_back(Ent{r0, r1, c0, c1, -1});
        wrs.push_back(s);
      }
    };
    auto emit = [&](int s, int step, int item, int kind) {
      const int t = (int)L.items++;
      std::sort(deps.begin(), deps.end());
      deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
      for (int d : deps) ddlist.push_back(d);
      ddptr.push_back((int32_t)ddlist.size());
      for (size_t k = 0; k < wr.size(); ++k) {
        const Ent q{wr[k].r0, wr[k].r1, wr[k].c0, wr[k].c1, t};
        const int f = wrs[k], nb = (int)cdiv(S.nrows[f], 64);
        auto& g = live[f];
        for (int R = q.r0 >> 6; R <= (q.r1 - 1) >> 6; ++R)
          for (int C = q.c0 >> 6; C <= std::min((q.c1 - 1) >> 6, R); ++C) {
            auto& cell = g[(size_t)R * nb + C];
            const int br0 = R * 64, br1 = br0 + 64, bc0 = C * 64, bc1 = bc0 + 64;
            cell.erase(std::remove_if(cell.begin(), cell.end(), [&](const Ent& e) {
                         const int a0 = std::max(e.r0, br0), a1 = std::min(e.r1, br1);
                         const int b0 = std::max(e.c0, bc0), b1 = std::min(e.c1, bc1);
                         return a0 >= q.r0 && a1 <= q.r1 && b0 >= q.c0 && b1 <= q.c1;  // covered here
                       }),
                       cell.end());
            cell.push_back(q);
          }
      }
      deps.clear();
      wr.clear();
      wrs.clear();
      dtask.insert(dtask.end(), {s, step, item, kind});
    };
    int maxsteps = 0;
    for (int s : big) maxsteps = std::max<int>(maxsteps, (int)cdiv(S.first[s + 1] - S.first[s], 64));
    // first diagonal blocks
    for (int s : big) {
      const int w = S.first[s + 1] - S.first[s], kw = std::min(64, w);
      region(s, 0, kw, 0, kw, true);
      emit(s, 0, 0, 3);
      L.bytes += 8.0 * (kw * (kw + 1.0) + 4 * 16 * 17);
      L.flops += (double)kw * kw * kw / 3.0;
    }
    for (int s : big) L.alg += fact_alg(s);  // every column of the level's big fronts
    auto bulk = [&](int g0) {  // 128 x 128 trailing tiles of group [g0, g0 + kp), columns past the feed tiles
      for (int s : big) {
        const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
        if ((int)cdiv(w, 64) <= g0 || S.fused[s]) continue;
        const int gend = std::min(64 * (g0 + kp), w), cb = gend + 64 * kp;
        if (cb >= r) continue;
        const int nt = (int)cdiv(r - cb, 128);
        const double K = gend - 64 * g0, nbt = r - cb;
        L.bytes += 8.0 * (nbt * (nbt + 1) + 2.0 * nbt * K);
        L.flops += K * nbt * (nbt + 1);
        // column by column: the first columns feed the next group's feed tiles (and its bulk's first
        // columns), so their tickets come first and are done by the time those wait for them
        for (int J = 0; J < nt; ++J)
          for (int I = J; I < nt; ++I) {
            const int i0 = cb + 128 * I, j0 = cb + 128 * J;
            region(s, i0, i0 + 128, 64 * g0, gend, false);  // (L D)_I and L_J: the group's panels
            region(s, j0, j0 + 128, 64 * g0, gend, false);
            region(s, i0, i0 + 128, j0, j0 + 128, true);
            emit(s, g0 + kp - 1, I | (J << 16), 2);
          }
      }
    };
    for (int g0 = 0; g0 < maxsteps; g0 += kp) {
      // chain, per step: the critical tasks of every front first — trsm tiles 0 and 1 and the updates of
      // tiles (0, 0) (with the next diagonal block), (1, 0) and (1, 1), which the next step's first
      // tasks wait for — then the other trsm tiles and local updates
      for (int p = g0; p < std::min(g0 + kp, maxsteps); ++p)
        for (int phase2 = 0; phase2 < 2; ++phase2)
          for (int kind = 0; kind < 2; ++kind)
            for (int s : big) {
              const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
              const int npan = (int)cdiv(w, 64);
              if (npan <= p) continue;
              const int k0 = p * 64, kw = std::min(64, w - k0);
              const int nt = (int)cdiv(r - k0 - kw, 64);
              const double dk = kw, nb = r - k0 - kw;
              const int gl = std::min(g0 + kp, npan) - 1, gend = std::min(64 * (gl + 1), w);
              const bool local = !S.fused[s] && p < gl;  // local updates (then kw = 64, c0 = k0 + 64)
              const int c0 = k0 + 64;
              const int ncol = local ? (int)cdiv(gend - c0, 64) : 0;
              auto trsm = [&](int rt) {
                const int R0 = k0 + kw + 64 * rt;
                region(s, k0, k0 + kw, k0, k0 + kw, false);  // L11, D, M_K
                region(s, R0, R0 + 64, k0, k0 + kw, true);
              };
              auto upd = [&](int i, int j) {
                region(s, c0 + 64 * i, c0 + 64 * i + 64, k0, k0 + 64, false);
                region(s, c0 + 64 * j, c0 + 64 * j + 64, k0, k0 + 64, false);
                region(s, c0 + 64 * i, c0 + 64 * i + 64, c0 + 64 * j, std::min(c0 + 64 * j + 64, gend), true);
              };
              const bool crit = phase2 == 0;
              if (kind == 0) {
                if (crit) {
                  L.bytes += 8.0 * (2.0 * nb * dk + nt * (dk * (dk + 1) / 2 + 4 * 16 * 17));
                  L.flops += nb * dk * dk;
                  if (local) {
                    const double nc = gend - c0;
                    L.bytes += 8.0 * (2.0 * nb * nc + nb * dk + nc * dk);
                    L.flops += 2.0 * dk * nc * (nb - 0.5 * nc);
                  }
                }
                for (int rt = crit ? 0 : 2; rt < (crit ? std::min(nt, 2) : nt); ++rt) {
                  trsm(rt);
                  emit(s, p, rt, 0);
                }
              } else if (local) {
                for (int j = 0; j < ncol; ++j)
                  for (int i = j; i < nt; ++i) {
                    const bool c = (i == 1 && j <= 1) || (i == 0 && j == 0);
                    if (c != crit) continue;
                    upd(i, j);
                    emit(s, p, i | (j << 16), 1);
                  }
              }
            }
      if (g0 > 0) bulk(g0 - kp);
      // feed: the trailing update of the next group's columns, 64 x 64 tiles (k_big_update trailing mode)
      for (int s : big) {
        const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
        if ((int)cdiv(w, 64) <= g0 || S.fused[s]) continue;
        const int gend = std::min(64 * (g0 + kp), w);
        if (gend >= r) continue;
        const int nt = (int)cdiv(r - gend, 64), ncb = std::min(kp, nt);
        const double K = gend - 64 * g0, nbt = r - gend, nc = std::min(64.0 * kp, nbt);
        L.bytes += 8.0 * (2.0 * nbt * nc + (nbt + nc) * K);
        L.flops += 2.0 * K * nc * (nbt - 0.5 * nc);
        for (int j = 0; j < ncb; ++j)
          for (int i = j; i < nt; ++i) {
            const int i0 = gend + 64 * i, j0 = gend + 64 * j;
            region(s, i0, i0 + 64, 64 * g0, gend, false);
            region(s, j0, j0 + 64, 64 * g0, gend, false);
            region(s, i0, i0 + 64, j0, j0 + 64, true);
            emit(s, g0 + kp - 1, (int)((uint32_t)i | ((uint32_t)j << 16) | 0x80000000u), 1);
          }
      }
    }
    bulk(((maxsteps - 1) / kp) * kp);
    out.push_back(L);
    if (phase == 1 && S.atile_fz0[lev] < S.atile_lev[lev + 1]) {
      // the fused fronts' trailing tiles: assembled + updated after their panel (one launch)
      const int32_t t0 = S.atile_fz0[lev], t1 = S.atile_lev[lev + 1];
      Launch A{ASM_UPDATE, 0, t0, 4, t1 - t0};
      for (int32_t t = t0; t < t1; ++t) {
        const SymbolicPlan::AsmTile& at = S.atiles[t];
        const int f = at.front, r = S.nrows[f], w = S.first[f + 1] - S.first[f];
        A.nf = std::max(A.nf, (w + 3) & ~3);
        const int ti = at.tij & 0xffff, tj = (at.tij >> 16) & 0x7fff;
        const double nr = std::min(64, r - 64 * ti), nc = std::min(64, r - 64 * tj);
        A.bytes += 8.0 * (ti == tj ? nr * (nr + 1) / 2 : nr * nc) + (at.gptr >= 0 ? 4.0 * (S.g_ptr[at.gptr] + 2) : 0.0) +
                   8.0 * (nr + nc) * w;
        for (int k = at.bt0; k < at.bt1; ++k) {
          const int32_t* e = &S.bt[5 * k];
          for (int b = e[1]; b < e[2]; ++b) A.bytes += 8.0 * std::max(0, e[4] - std::max(b, e[3]));
        }
        A.flops += 2.0 * nr * nc * w;
      }
      out.push_back(A);
    }
  };
  auto build_fact = [&](int phase, std::vector<Launch>& out) {
    if (phase == 1 && !S.lb.empty()) {
      Launch L{LB_BUILD, 0, 0, 0, (int64_t)S.lb_mem.size()};
      for (const auto& G : S.lb) L.bytes += 8.0 * (double)G.m * G.n * 2.0 + 12.0 * G.n * G.m;
      for (int32_t c : S.lb_mem) L.alg += fact_alg_cols(c, c + 1);
      out.push_back(L);
    }
    auto ftree_launch = [&]() {  // factorisation tree: after every level-0 launch (the pre-leaves)
      asm_launch(2 * NL + 1, out);
      Launch L{FTREE, 0, 0, nftree_, (int64_t)nftree_};
      L.bytes = ftree_bytes_;
      L.alg = ftree_alg_;
      L.flops = ftree_flops_;
      L.lds_bytes = ftree_lds_;
      out.push_back(L);
    };
    for (int lev = 0; lev < NL; ++lev) {
      if (phase == 1 && lev == 1 && nftree_) ftree_launch();
      asm_launch(phase == 1 ? lev : NL + 1 + lev, out);
      if (phase == 1)
        for (int g : lb_at_level_[lev])
          if (!S.top(S.lb[g].parent)) lb_syrk_launch(g, out);  // top parents: after their external part
      std::vector<int32_t> cls[4], big, micro;
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) {
        const int s = S.level_list[q];
        if (!in_phase(s, phase) || S.ftree[s]) continue;
        if (S.parent[s] >= 0 && S.absorb[S.parent[s]]) continue;  // factorised by its absorbing parent
        const int r = S.nrows[s], w = S.first[s + 1] - S.first[s];
        if (r <= 32 && w <= 2 && S.fs_off[s] < 0 && !S.is_big[s])
          micro.push_back(s);
        else if (!S.is_big[s])
          cls[r <= 32 ? 0 : (r <= 64 ? 1 : (r <= 128 ? 2 : 3))].push_back(s);
        else
          big.push_back(s);
      }
      if (!micro.empty()) {
        Launch L{MICRO, 0, (int64_t)sched.size(), (int)micro.size(), (int64_t)micro.size()};
        for (int f : micro) {
          const double r = S.nrows[f], w = S.first[f + 1] - S.first[f];
          L.bytes += 8.0 * (r * w + (r - w) * (r - w + 1) / 2 + w) + 16.0 * (S.asm_ptr[f + 1] - S.asm_ptr[f]);
          L.alg += fact_alg(f);
          for (int t = 0; t < (int)w; ++t) L.flops += (r - t - 1) * (r - t);
        }
        out.push_back(L);
        sched.insert(sched.end(), micro.begin(), micro.end());
      }
      for (int c = 0; c < 4; ++c)
        if (!cls[c].empty()) {
          Launch L{c == 3 ? SMALL192 : SMALL32 + c, 0, (int64_t)sched.size(), (int)cls[c].size(), (int64_t)cls[c].size()};
          L.lds = false;
          for (int f : cls[c]) {
            L.lds = L.lds || S.fs_off[f] < 0;
            const int r = S.nrows[f];
            L.lds_bytes = std::max<int>(L.lds_bytes, c == 3 ? 8 * r * (r + 1) / 2 : 8 * r * (r | 1));
          }
          for (int f : cls[c]) {  // reads: K entries or the assembled front; writes: L panel, U block, D
            const double r = S.nrows[f], w = S.first[f + 1] - S.first[f];
            L.bytes += 8.0 * (r * w + (r - w) * (r - w) + w) +
                       (S.fs_off[f] >= 0 ? 8.0 * r * (r + 1) / 2 : 16.0 * (S.asm_ptr[f + 1] - S.asm_ptr[f]));
            L.alg += fact_alg(f);
            for (int t = 0; t < (int)w; ++t) L.flops += (r - t - 1) * (r - t);
          }
          out.push_back(L);
          sched.insert(sched.end(), cls[c].begin(), cls[c].end());
        }
      if (big.empty()) continue;
      if (big_dag_) {
        dag_level(big, lev, phase, out);
        continue;
      }
      int maxsteps = 0;
      for (int s : big) maxsteps = std::max<int>(maxsteps, (int)cdiv(S.first[s + 1] - S.first[s], 64));
      int64_t last_upd = -1;  // the latest update launch (it factorised the next step's diagonal blocks)
      for (int p = 0; p < maxsteps; ++p) {
        std::vector<int32_t> td, tt, tu, tu128;  // (front, item) pairs
        double kb[4] = {0, 0, 0, 0}, kf[4] = {0, 0, 0, 0}, ka = 0;
        for (int s : big) {
          const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
          const int npan = (int)cdiv(w, 64);
          if (npan <= p) continue;
          const int k0 = p * 64, kw = std::min(64, w - k0);
          const int nt = (int)cdiv(r - k0 - kw, 64);
          const double dk = kw, nb = r - k0 - kw;
          kb[0] += 8.0 * (dk * (dk + 1) + 4 * 16 * 17);  // diag: read + write lower, write the M blocks
          ka += fact_alg_cols(S.first[s] + k0, S.first[s] + k0 + kw);  // 8(d): the panel's columns
          kf[0] += dk * dk * dk / 3.0;
          kb[1] += 8.0 * (2.0 * nb * dk + nt * (dk * (dk + 1) / 2 + 4 * 16 * 17));  // trsm: rows in/out + L11, M per tile
          kf[1] += nb * dk * dk;
          if (p == 0) td.insert(td.end(), {s, 0});  // later panels: the previous update's task (0, 0)
          for (int i = 0; i < nt; ++i) tt.insert(tt.end(), {s, i});
          if (S.fused[s]) continue;  // its trailing update: k_asm_update (below)
          // deferred multi-panel update (k_big_update): panel groups of big_kpan_ panels; inside a
          // group each panel updates the group's later panels only (local tiles), the group's last
          // panel updates the rest of the front with K = the whole group (trailing tiles)
          const int g0 = (p / big_kpan_) * big_kpan_, gl = std::min(g0 + big_kpan_, npan) - 1;
          const int gend = std::min(64 * (gl + 1), w);
          if (p < gl) {
            const double nc = gend - (k0 + kw);  // the group's later columns
            for (int j = 0; j < (int)cdiv((int)nc, 64); ++j)
              for (int i = j; i < nt; ++i) tu.insert(tu.end(), {s, i | (j << 16)});
            kb[2] += 8.0 * (2.0 * nb * nc + nb * dk + nc * dk);  // C in/out + the panel rows once
            kf[2] += 2.0 * dk * nc * (nb - 0.5 * nc);
          } else {  // 128 x 128 tiles (k_big_upd128)
            const int c0 = gend, ntt = (int)cdiv(r - c0, 128);
            const double K = gend - 64 * g0, nbt = r - c0;
            for (int i = 0; i < ntt; ++i)
              for (int j = 0; j <= i; ++j) tu128.insert(tu128.end(), {s, i | (j << 16)});
            kb[3] += 8.0 * (nbt * (nbt + 1) + 2.0 * nbt * K);  // C in/out once per group + the group's panels
            kf[3] += K * nbt * (nbt + 1);
          }
        }
        const std::pair<int, std::vector<int32_t>*> kinds[4] = {
            {BIG_DIAG, &td}, {BIG_TRSM, &tt}, {BIG_UPDATE, &tu}, {BIG_UPDATE128, &tu128}};
        bool alg_done = false;  // the panels' 8(d) bytes ride on the step's first launch (k_big_diag at
                                // step 0, k_big_trsm after: the diagonal blocks are factorised by the
                                // previous step's update launch)
        for (int q = 0; q < 4; ++q) {
          const auto& kv = kinds[q];
          if (kv.second->empty()) continue;
          align2();
          Launch L{kv.first, p, (int64_t)sched.size(), 0, (int64_t)kv.second->size() / 2};
          L.bytes = kb[q];
          L.alg = alg_done ? 0.0 : ka;
          alg_done = true;
          if (kv.first == BIG_UPDATE || kv.first == BIG_UPDATE128) last_upd = (int64_t)out.size();
          if (kv.first == BIG_UPDATE128)  // K split over 2-4 workgroups per tile when the tiles alone
                                          // would leave most CUs idle (k_big_upd128; nf = the split)
            L.nf = !upd_split_ ? 1 : L.items <= 128 ? 4 : L.items <= 170 ? 3 : L.items <= 256 ? 2 : 1;
          L.flops = kf[q];
          out.push_back(L);
          sched.insert(sched.end(), kv.second->begin(), kv.second->end());
        }
        // a last panel without rows below (r == w) launches nothing: its diagonal block was factorised
        // by the previous step's update launch, which carries its bytes
        if (!alg_done && ka > 0.0 && last_upd >= 0) out[last_upd].alg += ka;
        if (p == 0 && phase == 1 && S.atile_fz0[lev] < S.atile_lev[lev + 1]) {
          // the fused fronts' trailing tiles: assembled + updated after their panel (one launch)
          const int32_t t0 = S.atile_fz0[lev], t1 = S.atile_lev[lev + 1];
          Launch L{ASM_UPDATE, 0, t0, 4, t1 - t0};
          for (int32_t t = t0; t < t1; ++t) {
            const SymbolicPlan::AsmTile& at = S.atiles[t];
            const int f = at.front, r = S.nrows[f], w = S.first[f + 1] - S.first[f];
            L.nf = std::max(L.nf, (w + 3) & ~3);
            const int ti = at.tij & 0xffff, tj = (at.tij >> 16) & 0x7fff;
            const double nr = std::min(64, r - 64 * ti), nc = std::min(64, r - 64 * tj);
            // the written entries + the chunk sums' offsets + the panel rows of I and J (+ big children)
            L.bytes += 8.0 * (ti == tj ? nr * (nr + 1) / 2 : nr * nc) + (at.gptr >= 0 ? 4.0 * (S.g_ptr[at.gptr] + 2) : 0.0) +
                       8.0 * (nr + nc) * w;
            for (int k = at.bt0; k < at.bt1; ++k) {
              const int32_t* e = &S.bt[5 * k];
              for (int b = e[1]; b < e[2]; ++b) L.bytes += 8.0 * std::max(0, e[4] - std::max(b, e[3]));
            }
            L.flops += 2.0 * nr * nc * w;
          }
          out.push_back(L);
        }
      }
    }
    if (phase == 1 && NL == 1 && nftree_) ftree_launch();
  };
  clk("  launch plans (before build_fact)");
  build_fact(1, fact1_);
  if (S.nshards > 1) {
    asm_launch(NL, fact1_);  // top fronts, external part (all-reduced next)
    for (size_t g = 0; g < S.lb.size(); ++g)  // this shard's batched leaves under top fronts: into it
      if (S.top(S.lb[g].parent)) lb_syrk_launch((int)g, fact1_);
    build_fact(2, fact2_);
  }
  if (!dtask.empty()) {  // DAG tasks, dependencies, flags, counters, per-panel M_K slots
    dag_tasks_.upload(dtask);
    dag_dptr_.upload(ddptr);
    dag_dlist_.upload(ddlist.empty() ? std::vector<int32_t>{0} : ddlist);
    dag_flags_.alloc((int64_t)dtask.size() / 4);
    dag_flags_.zero();
    dag_cnt_.alloc(2);
    dag_cnt_.zero();
    dag_m_.alloc(std::max<int64_t>(nmslot, 1) * BIG_MSZ);
    dag_mslot_.upload(mslot);
    int dev = 0, ncu = 0;
    MADIPM_HIP(hipGetDevice(&dev));
    MADIPM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    dag_grid_ = std::max(1, 2 * ncu);  // two workgroups per CU (80 KB of LDS, <= 256 registers)
    if (const char* ed = std::getenv("MADIPM_DAG_DEBUG"); ed && ed[0] == '1') {  // per-task stamps (diagnostics)
      dag_dbg_.alloc((int64_t)dtask.size());
      dag_dbg_.zero();
      dag_kind_ = dtask;
    }
  }
  {  // k_big_upd128's split-K scratch: partial products and per-tile tickets of the largest split launch
    int64_t np = 0, nt = 0;
    for (const auto* V : {&fact1_, &fact2_})
      for (const Launch& L : *V)
        if (L.kind == BIG_UPDATE128 && L.nf > 1) {
          np = std::max<int64_t>(np, L.items * L.nf);
          nt = std::max<int64_t>(nt, L.items);
        }
    if (np) {
      upsum_.alloc((size_t)np * UPD_PART);
      uptick_.alloc((size_t)nt);
      uptick_.zero();
    }
  }

  // ---- solve schedules: per level, small fronts (wave per front) and big fronts (task queues)
  clk("  build_fact + dag tables");
  std::vector<uint8_t> rootf(std::max(ns, 1), 0);  // roots solved by k_root_solve (1) / a k_fwd_tree task (2)
  std::vector<int32_t> tfront;                      // tree-solve task -> its (top) front
  {
    std::vector<int32_t> flag_off(ns, 0);
    int64_t nflags = 0;
    for (int s = 0; s < ns; ++s)
      if (!solve_small(s)) {
        flag_off[s] = (int32_t)nflags;
        nflags += cdiv(S.first[s + 1] - S.first[s], 64);
      }
    std::vector<int32_t> tasks, bp_off(ns, 0);
    int64_t nbpart = 0;
    auto build_solve = [&](int phase, std::vector<SolveLevel>& out) {
      for (int lev = 0; lev < NL; ++lev) {
        std::vector<int32_t> tiny, small, big, micro;
        for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) {
          const int s = S.level_list[q];
          if (!in_phase(s, phase) || (phase == 1 && (in_tree[s] || sleaf[s]))) continue;
          const int r = S.nrows[s], w = S.first[s + 1] - S.first[s];
          if (r <= 32 && w <= 2)
            micro.push_back(s);
          else if (solve_small(s))
            (r > 32 ? small : tiny).push_back(s);
          else
            big.push_back(s);
        }
        SolveLevel L{};
        L.micro_off = (int64_t)sched.size();
        L.nmicro = (int)micro.size();
        sched.insert(sched.end(), micro.begin(), micro.end());
        for (int f : micro) {
          const double r = S.nrows[f], w = S.first[f + 1] - S.first[f];
          L.micro_bytes += 8.0 * (r * w + 3.0 * r);
          L.micro_flops += 2.0 * (r * w - w * (w + 1) / 2);
          L.micro_alg += solve_alg(f);
        }
        L.tiny_off = (int64_t)sched.size();
        L.ntiny = (int)tiny.size();
        sched.insert(sched.end(), tiny.begin(), tiny.end());
        L.small_off = (int64_t)sched.size();
        L.nsmall = (int)small.size();
        sched.insert(sched.end(), small.begin(), small.end());
        L.big_off = (int64_t)sched.size();
        L.nbig = (int)big.size();
        sched.insert(sched.end(), big.begin(), big.end());
        align2();
        L.gat_off = (int64_t)sched.size();
        for (int s : big)
          for (int c = 0; c < cdiv(S.nrows[s], GAT_ROWS); ++c) sched.insert(sched.end(), {s, c});
        L.ngat = (int)(((int64_t)sched.size() - L.gat_off) / 2);
        L.below_off = (int64_t)sched.size();
        for (int s : big) {
          const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
          if (r == w) continue;
          const int np = (int)cdiv(w, 64), nch = (int)cdiv(r - w, BWD_CHUNK);
          bp_off[s] = (int32_t)nbpart;
          nbpart += (int64_t)np * nch;
          for (int p = 0; p < np; ++p)
            for (int c = 0; c < nch; ++c) sched.insert(sched.end(), {s, p | (c << 16)});
        }
        L.nbelow = (int)(((int64_t)sched.size() - L.below_off) / 2);
        int maxblk = 0, maxpan = 0;
        for (int s : big) {
          maxblk = std::max<int>(maxblk, (int)cdiv(S.nrows[s], 64));
          maxpan = std::max<int>(maxpan, (int)cdiv(S.first[s + 1] - S.first[s], 64));
        }
        L.ftask_off = (int64_t)tasks.size() / 2;
        for (int i = 0; i < maxblk; ++i)
          for (int s : big)
            if (i < cdiv(S.nrows[s], 64)) {
              tasks.push_back(s);
              tasks.push_back(i);
            }
        L.nftask = (int)((int64_t)tasks.size() / 2 - L.ftask_off);
        L.btask_off = (int64_t)tasks.size() / 2;
        for (int k = 0; k < maxpan; ++k)
          for (int s : big) {
            const int np = (int)cdiv(S.first[s + 1] - S.first[s], 64);
            if (k < np) {
              tasks.push_back(s);
              tasks.push_back(np - 1 - k);
            }
          }
        L.nbtask = (int)((int64_t)tasks.size() / 2 - L.btask_off);
        // algorithmic traffic of one sweep: the L panel once (+ the vectors), 2 flops per panel entry
        for (int f : small) {
          const double r = S.nrows[f], w = S.first[f + 1] - S.first[f];
          L.small_bytes += 8.0 * (r * w + 3.0 * r);
          L.small_flops += 2.0 * (r * w - w * (w + 1) / 2);
          L.small_alg += solve_alg(f);
          L.small_lds = std::max<int>(L.small_lds, 8 * (S.nrows[f] | 1) * (S.first[f + 1] - S.first[f]));
        }
        for (int f : tiny) {
          const double r = S.nrows[f], w = S.first[f + 1] - S.first[f];
          L.tiny_bytes += 8.0 * (r * w + 3.0 * r);
          L.tiny_flops += 2.0 * (r * w - w * (w + 1) / 2);
          L.tiny_alg += solve_alg(f);
        }
        for (int f : big) {
          const double r = S.nrows[f], w = S.first[f + 1] - S.first[f];
          L.big_bytes += 8.0 * (r * w + 3.0 * r);
          L.big_flops += 2.0 * (r * w - w * (w + 1) / 2);
          L.below_bytes += 8.0 * (r - w) * w;
          const double sa = solve_alg(f), da = std::min(sa, 4.0 * w * (w + 1));  // diagonal block / below it
          L.big_alg += da;
          L.below_alg += sa - da;
          L.gat_bytes += 8.0 * (2.0 * r + 2.0 * (S.sv_ptr[S.row_ptr[f + 1]] - S.sv_ptr[S.row_ptr[f]]));
        }
        out.push_back(L);
      }
    };
    build_solve(1, slev1_);
    {  // tree solve tables
      // elimination-tree roots (r == w, no parent) whose panel needs more LDS than the tree launches'
      // TREE_SOLVE_LDS (two workgroups per CU) go last, into their own forward launch with the LDS they
      // need (ex10's 120-column coupling root: 125 KB), solved forward and backward there in one pass
      // (r3: the root sized every tree task's LDS; r4's first cut streamed it in chunks: slower)
      auto big_root = [&](int s) {
        const int r = S.nrows[s], w = S.first[s + 1] - S.first[s];
        const int64_t need = 8 * tree_panel_doubles(s) + 8 * 1024;
        return S.parent[s] < 0 && r == w && r <= SMALL_SOLVE_MAX && need > TREE_SOLVE_LDS && need <= TREE_ROOT_LDS;
      };
      std::vector<int32_t> ord, roots;
      for (int lev = 0; lev < NL; ++lev)
        for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q)
          if (in_tree[S.level_list[q]]) (big_root(S.level_list[q]) ? roots : ord).push_back(S.level_list[q]);
      nroot_task_ = (int)roots.size();
      for (int s : roots) rootf[s] = 1;
      rargs_.n = std::min(nroot_task_, kRootArgs);
      for (int q = 0; q < rargs_.n; ++q) {
        const int s = roots[q];
        rargs_.s[q] = s;
        rargs_.f0[q] = S.first[s];
        rargs_.w[q] = S.first[s + 1] - S.first[s];
        rargs_.r[q] = S.nrows[s];
        rargs_.e0[q] = S.row_ptr[s];
        rargs_.loff[q] = S.l_off[s];
      }
      ord.insert(ord.end(), roots.begin(), roots.end());
      ntree_ = (int)ord.size();
      // children of tree fronts scatter their forward update entries straight into the parent's
      // gather range (sv order, gbuf); everyone else keeps its own update vector (uvec)
      // each tree-front row's gather entries: those of fronts solved by earlier launches (the flat
      // leaves, batched-leaf groups, level-path children) first, those of tree tasks (this launch)
      // last, sv_nt[row] of them — k_fwd_tree sums the first part before it waits for its children
      std::vector<int64_t> svs(S.sv_src);
      {
        std::vector<uint8_t> from_task((size_t)std::max<int64_t>(S.uvec_size, 1), 0);
        for (int s : ord)
          if (S.uvec_off[s] >= 0)
            for (int a = 0; a < S.nrows[s] - (S.first[s + 1] - S.first[s]); ++a) from_task[S.uvec_off[s] + a] = 1;
        std::vector<uint16_t> nt((size_t)std::max<int64_t>(S.row_ptr[ns], 1), 0);
        std::vector<int64_t> tail;
        for (int s : ord)
          for (int i = 0; i < S.nrows[s]; ++i) {
            const int64_t t = S.row_ptr[s] + i, p0 = S.sv_ptr[t], p1 = S.sv_ptr[t + 1];
            tail.clear();
            int64_t o = p0;
            for (int64_t p = p0; p < p1; ++p)
              if (from_task[S.sv_src[p]])
                tail.push_back(S.sv_src[p]);
              else
                svs[o++] = S.sv_src[p];
            for (int64_t v : tail) svs[o++] = v;
            MADIPM_REQUIRE(tail.size() <= 65535, "tree solve: tree-task entries of one row beyond 16 bits");
            nt[t] = (uint16_t)tail.size();
          }
        sv_src_.upload(svs);
        sv_nt_.upload(nt);
        MADIPM_HIP(hipStreamSynchronize(nullptr));  // the host vectors end with this block
      }
      std::vector<int64_t> inv((size_t)std::max<int64_t>(S.uvec_size, 1), -1), upm((size_t)std::max<int64_t>(S.rel_ptr[ns], 1), -1);
      for (int s : ord)
        for (int64_t p = S.sv_ptr[S.row_ptr[s]]; p < S.sv_ptr[S.row_ptr[s] + S.nrows[s]]; ++p) inv[svs[p]] = p;
      for (int c = 0; c < ns; ++c)
        if (S.parent[c] >= 0 && in_tree[S.parent[c]])
          for (int64_t a = 0; a < S.rel_ptr[c + 1] - S.rel_ptr[c]; ++a) {
            upm[S.rel_ptr[c] + a] = inv[S.uvec_off[c] + a];
            MADIPM_REQUIRE(upm[S.rel_ptr[c] + a] >= 0, "tree gather map");
          }
      auto inv_pos = [&](int c, int a) { return upm[S.rel_ptr[c] + a]; };
      tree_lds_ = 8 * 1024;
      std::vector<uint8_t> chunk(std::max(ns, 1), 0);
      for (int s : ord) {
        const double r = S.nrows[s], w = S.first[s + 1] - S.first[s];
        tree_bytes_ += 8.0 * (r * w + 3.0 * r);
        tree_flops_ += 2.0 * (r * w - w * (w + 1) / 2);
        tree_alg_ += solve_alg(s);
        chunk[s] = !big_root(s) && (S.nrows[s] > SMALL_SOLVE_MAX || 8 * tree_panel_doubles(s) + 8 * 1024 > TREE_SOLVE_LDS);
        if (big_root(s)) root_lds_ = std::max<int>(root_lds_, 8 * tree_panel_doubles(s));  // k_root_solve: the panel
      }
      tree_lds_ = TREE_SOLVE_LDS;  // the rest of the budget stages gather sources
      tchunk_.upload(chunk);
      // one task per tree front, in `ord` order (levels ascending): a task's forward dependencies (its
      // tree children) have earlier tickets, and in reverse order the backward one (its tree parent)
      // does.  (r3: chains of only-children solved back to back by one workgroup measured slower.)
      std::vector<int32_t> cptr{0}, clist, dptr{0}, dl, tops;
      std::vector<SolveLeaf> lv;
      std::vector<int2> lrow;
      for (int s : ord) {
        clist.push_back(s);
        for (int q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q)
          if (in_tree[S.child_list[q]]) dl.push_back(S.child_list[q]);
        cptr.push_back((int32_t)clist.size());
        dptr.push_back((int32_t)dl.size());
        tops.push_back(s);
      }
      // the flat leaf launches: every folded leaf, in postorder (L panels in order)
      for (int c = 0; c < ns; ++c) {
        if (!sleaf[c]) continue;
        const int r = S.nrows[c], w = S.first[c + 1] - S.first[c], f0 = S.first[c];
        lv.push_back(SolveLeaf{S.l_off[c], f0, r | (w << 8), S.perm[f0], w == 2 ? S.perm[f0 + 1] : -1,
                               (int32_t)lrow.size(), 0});
        for (int a = 0; a < r - w; ++a) {
          const int64_t g = inv_pos(c, a);
          MADIPM_REQUIRE(g >= 0 && g < INT32_MAX, "tree solve: folded leaf gather position");
          lrow.push_back(int2{(int32_t)g, S.rows[S.row_ptr[c] + w + a]});
        }
      }
      ntask_ = (int)tops.size();
      tfront = tops;
      {  // elimination-tree roots (r == w, no parent) solved backward by k_fwd_tree right after their forward
         // substitution, on the panel already in LDS (bitwise k_bwd_tree's x; r3: k_bwd_tree 52 -> 43 us)
        std::vector<uint8_t> rbv(std::max(ntask_, 1), 0);
        for (int t = 0; t < ntask_; ++t) {
          const int f = tops[t];
          rbv[t] = S.parent[f] < 0 && S.nrows[f] == S.first[f + 1] - S.first[f] && !chunk[f];
          if (rbv[t] && !rootf[f]) rootf[f] = 2;  // solved forward and backward by its k_fwd_tree task
        }
        trootbwd_.upload(rbv);
      }
      std::vector<int32_t> par;  // backward ticket t -> task ntask - 1 - t: the tree parent of its top
      for (int t = ntask_ - 1; t >= 0; --t) {
        const int p = S.parent[tops[t]];
        par.push_back(p >= 0 && in_tree[p] ? p : -1);
      }
      auto up = [](DBuf<int32_t>& d, const std::vector<int32_t>& v) { d.upload(v.empty() ? std::vector<int32_t>{0} : v); };
      up(tc_ptr_, cptr);
      up(tc_list_, clist);
      up(tdep_ptr_, dptr);
      up(tdep_, dl);
      up(tpar_, par);
      tleaf_.upload(lv.empty() ? std::vector<SolveLeaf>(1) : lv);
      lrow.push_back(int2{0, 0});  // padding: the leaf kernels' clamped loads of a leaf without update rows
      tlrow_.upload(lrow);
      nsleaf_ = (int64_t)lv.size();
      for (const SolveLeaf& L : lv) {
        const double r = L.rw & 255, w = L.rw >> 8;
        leaf_alg_ += 8.0 * (S.colcnt[L.f0] + (w == 2 ? S.colcnt[L.f0 + 1] : 0));
        leaf_bytes_ += 8.0 * (r * w + 3.0 * r) + 32.0 + 8.0 * (r - w);
        leaf_flops_ += 2.0 * (r * w - w * (w + 1) / 2);
      }
      tflags_.alloc(std::max(ns, 1));
      tflags_.zero();
      upos_.upload(upm);
      gbuf_.alloc(std::max<int64_t>(S.sv_ptr[S.row_ptr[ns]], 1));
      T_.upos = upos_;
      T_.gbuf = gbuf_;
      const char* dv = std::getenv("MADIPM_TREE_DEBUG");
      if (dv && dv[0] == '1' && ntree_) tdbg_.alloc((int64_t)8 * ntree_);
    }
    if (S.nshards > 1) {
      build_solve(2, slev2_);
      align2();
      xg_off_ = (int64_t)sched.size();
      for (int s = 0; s < ns; ++s)
        if (S.top(s))
          for (int c = 0; c < cdiv(S.nrows[s], NT); ++c) sched.insert(sched.end(), {s, c});
      nxg_ = (int)(((int64_t)sched.size() - xg_off_) / 2);
    }
    tasks_.upload(tasks.empty() ? std::vector<int32_t>{0, 0} : tasks);
    flag_off_.upload(flag_off);
    bp_off_.upload(bp_off);
    bpart_.alloc(std::max<int64_t>(nbpart, 1) * 64);
    flags_.alloc(std::max<int64_t>(nflags, 1));
    flags_.zero();
    // the big fronts' panel solutions as self-validating words (ll_put / ll_get): 64 values x 2 halves
    // per panel flag
    xll_.alloc(std::max<int64_t>(nflags, 1) * 128);
    xll_.zero();
    T_.xll = xll_;
    counters_.alloc(4 * std::max(NL, 1) + 4);  // + the tree-solve tickets (4 NL, 4 NL + 1)
    counters_.zero();
  }
  {  // the root tail: the launches after the last tree launch factorise only k_root_solve's fronts
    size_t ft = SIZE_MAX;
    for (size_t i = 0; i < fact1_.size(); ++i)
      if (fact1_[i].kind == FTREE) ft = i;
    // after it: assembly launches, the last of which assembles the roots, then ONE factorisation
    // launch (SMALL*) of <= 64 roots, all of them solved by k_root_solve
    const size_t nl = fact1_.size();
    bool ok = S.nshards == 1 && ntree_ > 0 && ft != SIZE_MAX && ft + 2 < nl && fact1_[nl - 2].kind == ASSEMBLE;
    for (size_t i = ft + 1; ok && i + 1 < nl; ++i) ok = fact1_[i].kind == ASSEMBLE;
    if (ok) {
      const Launch& L = fact1_[nl - 1];
      ok = (L.kind == SMALL64 || L.kind == SMALL128 || L.kind == SMALL192) && L.items <= 64;
      for (int64_t k = 0; ok && k < L.items; ++k) ok = rootf[sched[L.off + k]] != 0;
    }
    const char* ra = std::getenv("MADIPM_ROOT_ASYNC");
    // the tail's kernel waits on the device for a kernel of the caller's stream: never where kernels
    // are serialised (counter collection — rocprofv3 --pmc dispatches one kernel at a time, and the
    // waiting kernel would hold the GPU until its wait times out — AMD_SERIALIZE_KERNEL,
    // HIP_LAUNCH_BLOCKING)
    auto set = [](const char* k) {
      const char* v = std::getenv(k);
      return v && v[0] && v[0] != '0';
    };
    const bool serial = set("ROCPROF_COUNTER_COLLECTION") || set("ROCPROF_COUNTERS") || set("AMD_SERIALIZE_KERNEL") ||
                        set("HIP_LAUNCH_BLOCKING");
    root_async_ = ok && !serial && !(ra && ra[0] == '0');
    if (ra && ra[0] == '2') {  // diagnostics: why (not)
      std::string k;
      for (const Launch& L : fact1_) k += std::to_string(L.kind) + "/" + std::to_string(L.items) + " ";
      std::string rk;
      if (nl > 0)
        for (int64_t q = 0; q < std::min<int64_t>(fact1_[nl - 1].items, 8); ++q) {
          const int f = sched[fact1_[nl - 1].off + q];
          rk += std::to_string(f) + ":" + std::to_string(rootf[f]) + ":r" + std::to_string(S.nrows[f]) + " ";
        }
      fprintf(stderr, "root tail: async %d (roots %d, tree launch %lld, launches kind/items: %s; last launch fronts %s)\n",
              (int)root_async_, nroot_task_, ft == SIZE_MAX ? -1LL : (long long)ft, k.c_str(), rk.c_str());
    }
    if (root_async_) {
      side0_ = nl - 1;
      nroot_side_ = (int)fact1_[nl - 1].items;
      int lo = 0, hi = 0;  // the tail is the critical path beside the forward solve: the higher priority
      MADIPM_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      MADIPM_HIP(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, hi));
      MADIPM_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
      // the roots' assembly tiles on the side stream too, behind the chunk pass's block flags
      // (MADIPM_ROOT_ASM_SIDE=0: on the caller's stream)
      const char* ea = std::getenv("MADIPM_ROOT_ASM_SIDE");
      asm_side_ = fact1_[nl - 2].nchunk > 0 && !(ea && ea[0] == '0');
      const int64_t ncb = asm_side_ ? cdiv(fact1_[nl - 2].nchunk, NT) : 0;
      rflag_.alloc(2 + 64 + ncb);  // go, the assembly's tile counter, one done flag per root, chunk blocks
      rflag_.zero();
      // the k_fwd_tree tasks of the side roots wait for the tail themselves (supportcase10's root)
      std::vector<uint8_t> ts(std::max(ntask_, 1), 0);
      const Launch& L = fact1_[nl - 1];
      for (int64_t k = 0; k < L.items; ++k) {
        const int f = sched[L.off + k];
        if (rootf[f] == 2)
          for (int t = 0; t < ntask_; ++t)
            if (tfront[t] == f) ts[t] = 1, side_tree_ = true;
      }
      tside_.upload(ts);
    }
  }
  clk("  tree solve tables + root tail");
  sched_.upload(sched.empty() ? std::vector<int32_t>{0} : sched);
  arena_.alloc(std::max<int64_t>(S.arena_size, 2));
  if (S.nshards > 1) {  // top fronts: the strict upper triangles are never written, keep them 0
    MADIPM_HIP(hipMemset(arena_.p + S.top_lo, 0, sizeof(double) * (S.arena_size - S.top_lo)));
    // exchange buffer: the top fronts' lower triangles (column by column) + 4 status slots per shard
    std::vector<int64_t> tc;
    int64_t po = 0;
    for (int s = 0; s < ns; ++s)
      if (S.top(s)) {
        const int64_t r = S.nrows[s];
        for (int64_t c = 0; c < r; ++c) {
          tc.insert(tc.end(), {S.l_off[s] + c * r + c, po, r - c});
          po += r - c;
        }
      }
    ntopcol_ = (int)(tc.size() / 3);
    xpack_tri_ = po;
    topcol_.upload(tc.empty() ? std::vector<int64_t>{0, 0, 0} : tc);
    xpack_.alloc(po + 4 * S.nshards);
    xpack_.zero();
  }
  clk("  sched upload + arena");
  D_.alloc(std::max(S.N, 1));
  xi_.alloc(std::max(S.N, 1));
  uvec_.alloc(std::max<int64_t>(S.uvec_size, 1));
  vwork_.alloc(std::max<int64_t>(S.row_ptr[ns], 1));
  status_.alloc(1);
  MADIPM_HIP(hipHostMalloc((void**)&h_status_, sizeof(LDLStatus), hipHostMallocDefault));
  st_ = status_.p;
  h_st_ = h_status_;
  T_.err = &st_->err;
  status_.zero();
  h_st_->err = 0;
  static bool attr_done = false;
  if (!attr_done) {
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_small_factor<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   128 * 128 * 8));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_fwd_small, hipFuncAttributeMaxDynamicSharedMemorySize, 129 * 128 * 8));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_small_blocked<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   129 * 128 * 8));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_small_blocked<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   192 * 193 / 2 * 8));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_bwd_small, hipFuncAttributeMaxDynamicSharedMemorySize, 129 * 128 * 8));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_fwd_tree, hipFuncAttributeMaxDynamicSharedMemorySize, TREE_SOLVE_LDS));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_root_solve, hipFuncAttributeMaxDynamicSharedMemorySize, TREE_ROOT_LDS));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_fact_tree, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)SymbolicPlan::kFactTreeLdsMax));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_bwd_tree, hipFuncAttributeMaxDynamicSharedMemorySize, TREE_SOLVE_LDS));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_asm_update<int32_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   2 * 64 * AU_LDT * 8 + 8 * kAsmLdsSrc));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_asm_update<int64_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   2 * 64 * AU_LDT * 8 + 8 * kAsmLdsSrc));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_assemble<8, int32_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   8 * kAsmLdsSrc));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_assemble<8, int64_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   8 * kAsmLdsSrc));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_assemble<2, int32_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   8 * kAsmLdsSrc));
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_assemble<2, int64_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   8 * kAsmLdsSrc));
    {  // static + dynamic LDS of the assembly kernels must fit one CU (160 KB on gfx950), as k_fact_tree's
      int dev = 0, cu_lds = 0;
      MADIPM_HIP(hipGetDevice(&dev));
      MADIPM_HIP(hipDeviceGetAttribute(&cu_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
      auto chk = [&](const void* f, size_t dyn, const char* nm) {
        hipFuncAttributes fa{};
        MADIPM_HIP(hipFuncGetAttributes(&fa, f));
        MADIPM_REQUIRE(fa.sharedSizeBytes + dyn <= (size_t)cu_lds,
                       std::string(nm) + ": LDS " + std::to_string(fa.sharedSizeBytes) + " + " + std::to_string(dyn) +
                           " bytes exceeds the CU's " + std::to_string(cu_lds));
      };
      chk((const void*)k_assemble<2, int32_t>, 8 * kAsmLdsSrc, "k_assemble");
      chk((const void*)k_assemble<8, int64_t>, 8 * kAsmLdsSrc, "k_assemble");
      chk((const void*)k_asm_update<int32_t>, 2 * 64 * AU_LDT * 8 + 8 * kAsmLdsSrc, "k_asm_update");
      chk((const void*)k_asm_update<int64_t>, 2 * 64 * AU_LDT * 8 + 8 * kAsmLdsSrc, "k_asm_update");
    }
    attr_done = true;
  }
  clk("  buffers + attributes");
  MADIPM_HIP(hipDeviceSynchronize());
  clk("schedules + workspace");
}

LDLSolver::~LDLSolver() {
  if (side_) {  // a root tail never joined (a factorisation nothing solved with) ends before its buffers
    (void)hipStreamSynchronize(side_);
    (void)hipStreamDestroy(side_);
  }
  if (ev_join_) (void)hipEventDestroy(ev_join_);
  if (h_status_) (void)hipHostFree(h_status_);
  for (hipEvent_t e : evs_) (void)hipEventDestroy(e);
}

// bytes: the launch's staging-traffic model; alg: SURVEY 8(d)'s bytes of the same launch
#define TIMED(kind, bytes, alg, flops, launch)          \
  do {                                                  \
    const bool tm_ = t_begin(kind, s);                  \
    launch;                                             \
    if (tm_) t_end(kind, s, (bytes), (alg), (flops));   \
  } while (0)

const char* kernel_kind_name(int k) {
  static const char* names[KK_COUNT] = {"k_asm_chunks", "k_assemble",  "k_micro_factor", "k_small_blocked", "k_big_diag",
                                        "k_big_trsm",   "k_big_update", "k_inertia",    "k_fwd_small",    "k_fwd_gather",
                                        "k_fwd_big",    "k_bwd_below",  "k_bwd_big",    "k_bwd_small",
                                        "k_fwd_tiny",   "k_bwd_tiny",   "k_lb_build",   "k_lb_syrk",      "k_lb_gemv",
                                        "k_fwd_tree",   "k_bwd_tree",   "k_fact_tree",    "k_asm_update", "k_big_dag"};
  return (k >= 0 && k < KK_COUNT) ? names[k] : "?";
}

void LDLSolver::set_timing(unsigned mask) {
  tmask_ = mask;
  ev_used_ = 0;
  pend_.clear();
  for (auto& k : kst_) k = KernelStat{};
}

bool LDLSolver::t_begin(int kind, hipStream_t s) {
  if (!(tmask_ >> kind & 1u) || untimed_) return false;
  while (evs_.size() < ev_used_ + 2) {
    hipEvent_t e;  // no system-scope fence: the timestamps bracket the kernel, not a cache flush
    MADIPM_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    evs_.push_back(e);
  }
  pend_.push_back({kind, ev_used_, 0.0, 0.0, 0.0});
  MADIPM_HIP(hipEventRecord(evs_[ev_used_], s));
  ev_used_ += 2;
  return true;
}

void LDLSolver::t_end(int kind, hipStream_t s, double bytes, double alg, double flops) {
  Pending& p = pend_.back();
  (void)kind;
  p.bytes = bytes;
  p.alg = alg;
  p.flops = flops;
  MADIPM_HIP(hipEventRecord(evs_[p.e0 + 1], s));
}

void LDLSolver::kernel_stats(KernelStat out[KK_COUNT]) {
  for (const Pending& p : pend_) {
    MADIPM_HIP(hipEventSynchronize(evs_[p.e0 + 1]));
    float ms = 0.f;
    MADIPM_HIP(hipEventElapsedTime(&ms, evs_[p.e0], evs_[p.e0 + 1]));
    KernelStat& k = kst_[p.kind];
    k.launches++;
    k.ms += ms;
    k.bytes += p.bytes;
    k.alg_bytes += p.alg;
    k.flops += p.flops;
  }
  pend_.clear();
  ev_used_ = 0;
  for (int k = 0; k < KK_COUNT; ++k) out[k] = kst_[k];
}

// F_P[gpos, gpos] -= W D^{-1} W^T, one launch per K-chunk of LB_KCHUNK members
void LDLSolver::lb_syrk(int g, hipStream_t s) {
  const auto& G = S_.lb[g];
  const int P = G.parent;
  double* F = S_.is_big[P] ? arena_.p + S_.l_off[P] : fscratch_.p + S_.fs_off[P];
  const int nt = (int)cdiv(G.m, SYT);
  const unsigned ntile = (unsigned)(nt * (nt + 1) / 2);
  const double* dinv = lbd_.p + S_.lb_mem.size() + G.mem_off;
  for (int k0 = 0; k0 < G.n; k0 += LB_KCHUNK)
    k_lb_syrk<<<ntile, NT, 0, s>>>(lbW_.p + G.w_off, dinv, G.m, k0, std::min(G.n, k0 + LB_KCHUNK),
                                   lbgpos_.p + G.gpos_off, F, S_.nrows[P]);
}

void LDLSolver::lb_fwd(const double* b, hipStream_t s) {
  for (size_t g = 0; g < S_.lb.size(); ++g) {
    const auto& G = S_.lb[g];
    const int nch = (int)cdiv(G.n, LBF_COLS);
    int64_t poff = 0;
    for (size_t h = 0; h < g; ++h) poff += cdiv(S_.lb[h].n, LBF_COLS) * S_.lb[h].m;
    TIMED(KK_LB_GEMV, 8.0 * G.m * (double)G.n, lb_alg(g), 2.0 * G.m * (double)G.n,
          (k_lb_fwd1<<<dim3((unsigned)cdiv(G.m, NT), (unsigned)nch), NT, 0, s>>>(
              lbW_.p + G.w_off, lbd_, lbmem_, perm_, G.m, G.n, G.mem_off, b, xi_, lbpart_.p + poff)));
    k_lb_fwd2<<<(unsigned)cdiv(G.m, NT), NT, 0, s>>>(lbpart_.p + poff, G.m, nch, uvec_.p + G.uvec_off);
  }
}

void LDLSolver::lb_bwd(int g, double* b, hipStream_t s) {
  const auto& G = S_.lb[g];
  int64_t xoff = 0;
  for (int h = 0; h < g; ++h) xoff += S_.lb[h].m;
  TIMED(KK_LB_GEMV, 8.0 * G.m * (double)G.n, lb_alg(g), 2.0 * G.m * (double)G.n,
        (k_lb_bwd<<<(unsigned)cdiv(G.n, NT / 64), NT, 0, s>>>(lbW_.p + G.w_off, lbd_, lbmem_, perm_, lbxrow_.p + xoff,
                                                             G.m, G.n, G.mem_off, xi_, b)));
}

double LDLSolver::fact_alg_cols(int c0, int c1) const {
  double b = 0.0;
  for (int c = c0; c < c1; ++c) b += 8.0 * S_.colcnt[c] + 12.0 * S_.kcol[c];
  return b;
}
double LDLSolver::lb_alg(size_t g) const {  // solve bytes of a batched-leaf group: 8 nnzL of its members
  const auto& G = S_.lb[g];
  double b = 0.0;
  for (int64_t k = G.mem_off; k < G.mem_off + G.n; ++k) b += 8.0 * S_.colcnt[S_.lb_mem[k]];
  return b;
}
double LDLSolver::fact_alg(int s) const { return fact_alg_cols(S_.first[s], S_.first[s + 1]); }
double LDLSolver::solve_alg(int s) const {
  double b = 0.0;
  for (int c = S_.first[s]; c < S_.first[s + 1]; ++c) b += 8.0 * S_.colcnt[c];
  return b;
}

void LDLSolver::run_fact(const std::vector<Launch>& LL, const double* Kx, hipStream_t s, size_t b, size_t e,
                         LDLStatus* stamp) {
  if (b == 0) ++cepoch_;  // k_big_dag's flags: this factorisation's epoch (never 0)
  for (size_t li = b; li < std::min(e, LL.size()); ++li) {
    const Launch& L = LL[li];
    // the root tail (root_async_): the roots' assembly raises go, their factorisation waits for it
    int32_t* go = (root_async_ && &LL == &fact1_ && (li + 1 == side0_ || li == side0_)) ? rflag_.p : nullptr;
    const int32_t* list = sched_.p + L.off;
    switch (L.kind) {
      case ASSEMBLE: {
        // root_async_ with asm_side_: the roots' assembly (the launch before side0_) runs its chunk pass on
        // the caller's stream, each block raising a flag, and its tiles on side_, waiting for those flags
        const bool split = go && asm_side_ && li + 1 == side0_;
        const bool chunks = L.nchunk && !(split && side_phase_);
        const bool tiles = !(split && !side_phase_);
        int32_t* cfl = split ? rflag_.p + 2 + 64 : nullptr;
        const int ncw = split ? (int)cdiv(L.nchunk, NT) : 0;
        if (chunks)
          TIMED(KK_ASM_CHUNKS, L.bytes2, 0.0, L.flops2,
                (g_src32_.p ? k_asm_chunks<int32_t><<<(unsigned)cdiv(L.nchunk, NT), NT, 0, s>>>(
                                  chunk_ids_, g_chunk_, g_src32_, L.chunk0, L.nchunk, Kx, arena_, gpart_, cfl, repoch_)
                            : k_asm_chunks<int64_t><<<(unsigned)cdiv(L.nchunk, NT), NT, 0, s>>>(
                                  chunk_ids_, g_chunk_, g_src_, L.chunk0, L.nchunk, Kx, arena_, gpart_, cfl, repoch_)));
        if (tiles && g_src32_.p)
          TIMED(KK_ASSEMBLE, L.bytes, 0.0, L.flops,
                (L.items < 256 ? k_assemble<8, int32_t><<<(unsigned)L.items, ANT, 8 * kAsmLdsSrc, s>>>(
                                     T_, atiles_.p + L.off, g_ptr_, gpart_, brec_, arena_, fscratch_, g_src32_.p, Kx, go,
                                     repoch_, cfl, ncw)
                               : k_assemble<2, int32_t><<<(unsigned)L.items, ANT, 8 * kAsmLdsSrc, s>>>(
                                     T_, atiles_.p + L.off, g_ptr_, gpart_, brec_, arena_, fscratch_, g_src32_.p, Kx, go,
                                     repoch_, cfl, ncw)));
        else if (tiles)
          TIMED(KK_ASSEMBLE, L.bytes, 0.0, L.flops,
                (L.items < 256 ? k_assemble<8, int64_t><<<(unsigned)L.items, ANT, 8 * kAsmLdsSrc, s>>>(
                                     T_, atiles_.p + L.off, g_ptr_, gpart_, brec_, arena_, fscratch_, g_src_.p, Kx, go,
                                     repoch_, cfl, ncw)
                               : k_assemble<2, int64_t><<<(unsigned)L.items, ANT, 8 * kAsmLdsSrc, s>>>(
                                     T_, atiles_.p + L.off, g_ptr_, gpart_, brec_, arena_, fscratch_, g_src_.p, Kx, go,
                                     repoch_, cfl, ncw)));
        break;
      }
      case MICRO:
        TIMED(KK_TINY, L.bytes, L.alg, L.flops,
              (k_micro_factor<<<(unsigned)cdiv(L.items, NT / MG), NT, 0, s>>>(T_, list, (int)L.items, Kx, arena_, D_,
                                                                             st_, pivot_tol)));
        break;
      case SMALL32:
        TIMED(KK_TINY, L.bytes, L.alg, L.flops,
              (k_tiny_factor<<<(unsigned)cdiv(L.items, 4), NT, 0, s>>>(T_, list, (int)L.items, Kx, arena_, fscratch_, D_,
                                                                      st_, pivot_tol)));
        break;
      case SMALL64:
      case SMALL128:
        TIMED(KK_SMALL, L.bytes, L.alg, L.flops,
              (k_small_blocked<false><<<(unsigned)L.items, SBT, L.lds_bytes, s>>>(T_, list, Kx, arena_, fscratch_, D_,
                                                                                st_, pivot_tol, stamp, go, repoch_)));
        break;
      case SMALL192:
        TIMED(KK_SMALL, L.bytes, L.alg, L.flops,
              (k_small_blocked<true><<<(unsigned)L.items, SBT, L.lds_bytes, s>>>(T_, list, Kx, arena_, fscratch_, D_,
                                                                               st_, pivot_tol, stamp, go, repoch_)));
        break;
      case BIG_DIAG:
        TIMED(KK_DIAG, L.bytes, L.alg, L.flops,
              (k_big_diag<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.step, arena_, D_, minv_, st_, pivot_tol)));
        break;
      case BIG_TRSM:
        TIMED(KK_TRSM, L.bytes, L.alg, L.flops, (k_big_trsm<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.step, arena_, D_, minv_)));
        break;
      case BIG_UPDATE:
        TIMED(KK_UPDATE, L.bytes, L.alg, L.flops,
              (k_big_update<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.step, big_kpan_, arena_, D_, minv_, st_,
                                                              pivot_tol)));
        break;
      case ASM_UPDATE:  // nf = the launch's K rows (the widest panel, rounded up to 4)
        TIMED(KK_ASM_UPDATE, L.bytes, 0.0, L.flops,
              (g_src32_.p ? k_asm_update<int32_t><<<(unsigned)L.items, ANT, 2 * L.nf * AU_LDT * 8 + 8 * kAsmLdsSrc, s>>>(
                                T_, atiles_.p + L.off, g_ptr_, gpart_, brec_, arena_, D_, L.nf, g_src32_.p, Kx)
                          : k_asm_update<int64_t><<<(unsigned)L.items, ANT, 2 * L.nf * AU_LDT * 8 + 8 * kAsmLdsSrc, s>>>(
                                T_, atiles_.p + L.off, g_ptr_, gpart_, brec_, arena_, D_, L.nf, g_src_.p, Kx)));
        break;
      case BIG_DAG:  // off = the launch's first task (global index), items = its tasks
        TIMED(KK_BIG_DAG, L.bytes, L.alg, L.flops,
              (k_big_dag<<<(unsigned)std::min<int64_t>(L.items, dag_grid_), NT, 0, s>>>(
                  T_, reinterpret_cast<const DagTask*>(dag_tasks_.p) + L.off, dag_dptr_.p + L.off, dag_dlist_.p,
                  (int)L.items, dag_flags_.p + L.off, cepoch_, dag_cnt_.p, big_kpan_, arena_, D_, dag_m_, dag_mslot_,
                  st_, pivot_tol, &st_->err, dag_dbg_.p ? dag_dbg_.p + 4 * L.off : nullptr)));
        if (dag_dbg_.p) dag_debug_dump(s, L);
        break;
      case BIG_UPDATE128:
        TIMED(KK_UPDATE, L.bytes, L.alg, L.flops,
              (k_big_upd128<<<(unsigned)(L.items * std::max(1, L.nf)), NT, 0, s>>>(
                  T_, list, L.step, big_kpan_, arena_, D_, minv_, st_, pivot_tol, std::max(1, L.nf), upsum_, uptick_)));
        break;
      case LB_BUILD:
        TIMED(KK_LB_BUILD, L.bytes, L.alg, 0.0,
              (k_lb_build<<<(unsigned)L.items, NT, 0, s>>>(lbg_, lbgid_, lbmem_, lbcs_, lbce_, lbwbase_, lbwrow_, Kx, lbW_,
                                                          lbd_.p, lbd_.p + S_.lb_mem.size(), D_, st_, pivot_tol)));
        break;
      case LB_SYRK:
        TIMED(KK_LB_SYRK, L.bytes, 0.0, L.flops, lb_syrk((int)L.off, s));
        break;
      case FTREE:
        if (!ftree_checked_) {  // static + dynamic LDS must fit the CU (160 KB on gfx950)
          hipFuncAttributes fa{};
          MADIPM_HIP(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_fact_tree)));
          MADIPM_REQUIRE(fa.sharedSizeBytes + (size_t)L.lds_bytes <= 160 * 1024,
                         "k_fact_tree: LDS " + std::to_string(fa.sharedSizeBytes) + " + " +
                             std::to_string(L.lds_bytes) + " bytes exceeds 160 KB");
          ftree_checked_ = true;
        }
        ++fepoch_;
        TIMED(KK_FACT_TREE, L.bytes, L.alg, L.flops,
              (k_fact_tree<<<(unsigned)(nftree_ + nfhelp_), FTN, L.lds_bytes, s>>>(
                  T_, ft_order_, nftree_ + nfhelp_, nfhelp_, ft_dptr_, ft_dep_, fcnt_, fflags_, fepoch_, Kx, arena_,
                  fscratch_, D_, st_, pivot_tol, &st_->err, fdbg_.p)));
        if (fdbg_.p)  // (the helper tickets stamp nothing: the fronts' records follow them)
          tree_debug_dump(s, "fact", fdbg_.p + 24 * nfhelp_, nftree_, "stage", "wait", "push", "factor", "store", 24);
        break;
    }
  }
}

// Phase 1: this shard's subtrees (unsharded: the whole factorisation) + the top fronts' external
// assembly and the shard's status slot.
void LDLSolver::fact_phase1(const double* Kx, hipStream_t s) {
  if (S_.N == 0) return;
  join(s);  // the previous factorisation's root tail writes the same arena
  if (!(ext_reset && ext_status_ && !sharded())) k_status_init<<<1, 1, 0, s>>>(st_);
  const bool lazy = !sharded() && lazy_inertia && !spd && ext_status_;
  if (root_async_) {
    // the tree launch and the roots' assembly on s, the roots' factorisation on side_, where it waits
    // on the device for the assembly's go flag (no cross-stream event: its ~17 us of latency, r6_w).
    // s goes on to the caller's next kernels (the solve's right-hand side, forward leaves and tree
    // fronts), which read nothing the tail writes; k_root_solve waits for the tail's done flags.
    // Lazy inertia: the root kernel stamps t1.
    ++repoch_;
    run_fact(fact1_, Kx, s, 0, side0_);
    // not event-timed: the launch waits on the device from its enqueue (during the previous solve)
    // until the go flag, and events would count that wait as the kernel's time
    untimed_ = side_phase_ = true;
    run_fact(fact1_, Kx, side_, asm_side_ ? side0_ - 1 : side0_, fact1_.size(), lazy ? st_ : nullptr);
    untimed_ = side_phase_ = false;
    MADIPM_HIP(hipEventRecord(ev_join_, side_));
    root_pending_ = true;
    if (!lazy) join(s);  // k_inertia and the status copy below need the whole factor
  } else {
    run_fact(fact1_, Kx, s);
  }
  const int nb = (int)std::min<int64_t>(64, cdiv(S_.N, NT));
  const int spdf = spd ? 1 : 0;
  if (!sharded()) {
    if (lazy) {  // the driver's next kernel (root_async_: the root kernel) stamps t1
      inertia_stale_ = true;
      return;
    }
    TIMED(KK_INERTIA, 8.0 * S_.N, 0.0, 0.0, (k_inertia<<<nb, NT, 0, s>>>(D_, S_.N, st_, spdf, nullptr, 0)));
    MADIPM_HIP(hipGetLastError());
    if (!ext_status_) MADIPM_HIP(hipMemcpyAsync(h_st_, st_, sizeof(LDLStatus), hipMemcpyDeviceToHost, s));
    return;
  }
  TIMED(KK_INERTIA, 8.0 * S_.N, 0.0, 0.0, (k_inertia<<<nb, NT, 0, s>>>(D_, S_.N, st_, spdf, colmask_, 1)));
  k_pack_status<<<1, 64, 0, s>>>(st_, arena_.p + S_.top_hi, S_.shard, S_.nshards);
  if (ntopcol_) k_tri_pack<<<(unsigned)ntopcol_, NT, 0, s>>>(topcol_, arena_, xpack_, 0);
  MADIPM_HIP(hipMemcpyAsync(xpack_.p + xpack_tri_, arena_.p + S_.top_hi, sizeof(double) * 4 * S_.nshards,
                            hipMemcpyDeviceToDevice, s));
  MADIPM_HIP(hipGetLastError());
}

// Phase 2 (sharded): after the all-reduce of fact_xbuf(), every shard factorises the top fronts.
void LDLSolver::fact_phase2(hipStream_t s) {
  if (S_.N == 0 || !sharded()) return;
  if (ntopcol_) k_tri_pack<<<(unsigned)ntopcol_, NT, 0, s>>>(topcol_, arena_, xpack_, 1);
  MADIPM_HIP(hipMemcpyAsync(arena_.p + S_.top_hi, xpack_.p + xpack_tri_, sizeof(double) * 4 * S_.nshards,
                            hipMemcpyDeviceToDevice, s));
  k_unpack_status<<<1, 1, 0, s>>>(st_, arena_.p + S_.top_hi, S_.nshards);
  run_fact(fact2_, nullptr, s);
  const int nb = (int)std::min<int64_t>(64, cdiv(S_.N, NT));
  TIMED(KK_INERTIA, 8.0 * S_.N, 0.0, 0.0, (k_inertia<<<nb, NT, 0, s>>>(D_, S_.N, st_, spd ? 1 : 0, colmask_, 2)));
  MADIPM_HIP(hipGetLastError());
  MADIPM_HIP(hipMemcpyAsync(h_st_, st_, sizeof(LDLStatus), hipMemcpyDeviceToHost, s));
}

void LDLSolver::factorize_async(const double* Kx, hipStream_t s) {
  fact_phase1(Kx, s);
  if (!sharded() || S_.N == 0) return;
  MADIPM_REQUIRE(comm_ != nullptr, "sharded LDL^T without a communicator");
  comm_->allreduce_sum(fact_xbuf(), fact_xlen(), s);
  fact_phase2(s);
}

bool LDLSolver::external_status(LDLStatus* dev, LDLStatus* host) {
  if (sharded() || !dev || !host) return false;
  st_ = dev;
  h_st_ = host;
  T_.err = &st_->err;
  ext_status_ = true;
  k_status_init<<<1, 1, 0, nullptr>>>(st_, 1);
  MADIPM_HIP(hipDeviceSynchronize());
  return true;
}

void LDLSolver::join(hipStream_t s) {
  if (!root_pending_) return;
  MADIPM_HIP(hipStreamWaitEvent(s, ev_join_, 0));
  root_pending_ = false;
}

double LDLSolver::fact_seconds(hipStream_t s) {
  if (S_.N == 0) return 0.0;
  join(s);
  LDLStatus h;
  MADIPM_HIP(hipMemcpyAsync(&h, st_, sizeof(LDLStatus), hipMemcpyDeviceToHost, s));
  MADIPM_HIP(hipStreamSynchronize(s));
  int dev = 0, khz = 0;
  MADIPM_HIP(hipGetDevice(&dev));
  MADIPM_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  const uint64_t t = h.ticks + (h.t1 > h.t0 ? h.t1 - h.t0 : 0);
  return khz > 0 ? (double)t / (1e3 * khz) : 0.0;
}

// lazy_inertia: count the current factor's inertia now (inertia() of a driver that skips k_inertia)
void LDLSolver::count_inertia(hipStream_t s) {
  if (!inertia_stale_ || S_.N == 0) return;
  inertia_stale_ = false;
  join(s);
  const int nb = (int)std::min<int64_t>(64, cdiv(S_.N, NT));
  k_zero_counts<<<1, 1, 0, s>>>(st_);
  k_inertia<<<nb, NT, 0, s>>>(D_, S_.N, st_, 0, nullptr, 1);
  MADIPM_HIP(hipGetLastError());
  status(s, true);
}

int LDLSolver::status(hipStream_t s, bool sync) {
  if (S_.N == 0) {
    factorized = true;
    return 0;
  }
  if (sync) join(s);
  if (sync && ext_status_) MADIPM_HIP(hipMemcpyAsync(h_st_, st_, sizeof(LDLStatus), hipMemcpyDeviceToHost, s));
  if (sync) MADIPM_HIP(hipStreamSynchronize(s));
  if (h_st_->err) {  // a lost hand-off or a carve overflow gives a wrong factor or solve: never success
    const int e = h_st_->err;
    h_st_->err = 0;
    k_status_init<<<1, 1, 0, s>>>(st_, 1);
    MADIPM_HIP(hipStreamSynchronize(s));
    if (e & kErrAsmSrc)
      throw Error("LDL^T: an assembly tile's source count exceeded the LDS source path's windows (factor is invalid)", -5);
    if (e & kErrLdsCarve)
      throw Error("LDL^T: a front or folded-leaf batch exceeded k_fact_tree's LDS carve (factor is invalid)", -5);
    throw Error("LDL^T: a dependency hand-off between fronts timed out (factor or solve is invalid)", -5);
  }
  npos = h_st_->npos;
  nneg = h_st_->nneg;
  nzero = h_st_->nzero;
  const int fp = h_st_->fail_pivot;
  factorized = (fp == INT_MAX);
  return factorized ? 0 : fp;
}

// MADIPM_TREE_DEBUG=1: per-task wall-clock phases of the tree kernels (100 MHz counter), summarised
// per level on stderr for the first few launches (diagnostics only)
// MADIPM_DAG_DEBUG=1: per kind of k_big_dag task (trsm, 64-tile update, 128-tile update, diagonal
// block) the tasks, their mean wait for dependencies and mean run time, and the launch's span and the
// workgroup-time it kept busy / waiting (first few launches; 100 MHz clock)
void LDLSolver::dag_debug_dump(hipStream_t s, const Launch& L) {
  static int calls = 0;
  if (++calls > 12) return;
  MADIPM_HIP(hipStreamSynchronize(s));
  std::vector<int64_t> h((size_t)4 * L.items);
  MADIPM_HIP(hipMemcpy(h.data(), dag_dbg_.p + 4 * L.off, h.size() * 8, hipMemcpyDeviceToHost));
  double n[5] = {0, 0, 0, 0, 0}, wt[5] = {0, 0, 0, 0, 0}, rt[5] = {0, 0, 0, 0, 0};
  int64_t t0 = INT64_MAX, t1 = 0;
  for (int64_t t = 0; t < L.items; ++t) {
    const int k = dag_kind_[4 * (L.off + t) + 3];
    n[k] += 1;
    wt[k] += (double)(h[4 * t + 1] - h[4 * t]);
    rt[k] += (double)(h[4 * t + 2] - h[4 * t + 1]);
    t0 = std::min(t0, h[4 * t]);
    t1 = std::max(t1, h[4 * t + 2]);
  }
  const char* nm[5] = {"trsm", "upd64", "upd128", "diag", "step"};
  fprintf(stderr, "dag launch: %lld tasks, span %.1f us, wait %.1f / run %.1f WG-ms\n", (long long)L.items, (t1 - t0) / 100.0,
          (wt[0] + wt[1] + wt[2] + wt[3] + wt[4]) / 1e5, (rt[0] + rt[1] + rt[2] + rt[3] + rt[4]) / 1e5);
  for (int k = 0; k < 5; ++k)
    if (n[k] > 0)
      fprintf(stderr, "  %-7s %6.0f tasks  wait %7.2f us  run %7.2f us (mean)\n", nm[k], n[k], wt[k] / n[k] / 100.0, rt[k] / n[k] / 100.0);
}

void LDLSolver::tree_debug_dump(hipStream_t s, const char* what, const int64_t* dbuf, int nt, const char* p1,
                                const char* p2, const char* p3, const char* p4, const char* p5, int stride) {
  static int ndump = 0;
  if (ndump++ >= 8) return;
  std::vector<int64_t> hs((size_t)stride * nt), h((size_t)8 * nt);
  MADIPM_HIP(hipMemcpyAsync(hs.data(), dbuf, hs.size() * 8, hipMemcpyDeviceToHost, s));
  MADIPM_HIP(hipStreamSynchronize(s));
  for (int t = 0; t < nt; ++t)
    for (int k = 0; k < 8; ++k) h[8 * t + k] = hs[(size_t)stride * t + k];
  if (stride == 24) {  // factor sub-phases, leaf-folding phases, per level
    std::vector<double> ab((size_t)S_.nlevels * 6, 0.0), fo((size_t)S_.nlevels * 4, 0.0);
    std::vector<int> na(S_.nlevels, 0);
    for (int t = 0; t < nt; ++t) {
      const int lv = S_.level[(int)h[8 * t + 6]];
      na[lv]++;
      for (int k = 0; k < 6; ++k) ab[lv * 6 + k] += hs[(size_t)24 * t + 8 + k] * 0.01;
      for (int k = 0; k < 4; ++k) fo[lv * 4 + k] += hs[(size_t)24 * t + 16 + k] * 0.01;
    }
    for (int lv = 0; lv < S_.nlevels; ++lv)
      if (na[lv])
        fprintf(stderr, "  fold level %d: gather %.2f  pivots %.2f  L %.2f  products %.2f us\n", lv, fo[lv * 4] / na[lv],
                fo[lv * 4 + 1] / na[lv], fo[lv * 4 + 2] / na[lv], fo[lv * 4 + 3] / na[lv]);
    std::vector<double> sq((size_t)S_.nlevels * 3, 0.0);
    for (int t = 0; t < nt; ++t) {
      const int lv = S_.level[(int)h[8 * t + 6]];
      const int64_t* d = &hs[(size_t)24 * t];
      sq[lv * 3] += (d[14] - d[4]) * 0.01;
      sq[lv * 3 + 1] += (d[15] - d[14]) * 0.01;
      sq[lv * 3 + 2] += (d[5] - d[15]) * 0.01;
    }
    for (int lv = 0; lv < S_.nlevels; ++lv)
      if (na[lv])
        fprintf(stderr, "  store level %d: U issue %.2f  drain+flag %.2f  L/D %.2f us\n", lv, sq[lv * 3] / na[lv],
                sq[lv * 3 + 1] / na[lv], sq[lv * 3 + 2] / na[lv]);
    for (int lv = 0; lv < S_.nlevels; ++lv)
      if (na[lv] && T_.fpipe)
        fprintf(stderr,
                "  factor level %d: %d fronts  first16 %.2f  block steps %.2f  (wave 0: waits %.2f  diag factors %.2f; "
                "wave 1 waits %.2f)  schur %.2f us\n",
                lv, na[lv], ab[lv * 6] / na[lv], ab[lv * 6 + 1] / na[lv], ab[lv * 6 + 2] / na[lv], ab[lv * 6 + 3] / na[lv],
                ab[lv * 6 + 5] / na[lv], ab[lv * 6 + 4] / na[lv]);
      else if (na[lv])
        fprintf(stderr,
                "  factor level %d: %d fronts  first16 [kcyc/100] %.2f  first16 %.2f  panels %.2f  J0 %.2f  look %.2f  schur %.2f us\n",
                lv, na[lv], ab[lv * 6 + 5] / na[lv], ab[lv * 6] / na[lv], ab[lv * 6 + 1] / na[lv], ab[lv * 6 + 2] / na[lv],
                ab[lv * 6 + 3] / na[lv], ab[lv * 6 + 4] / na[lv]);
  }
  // tasks that stamped nothing (the big roots: k_root_solve) are skipped; a stamp a path did not
  // take (a chunked front's) repeats the previous one
  for (int t = 0; t < nt; ++t) {
    int64_t* d = &h[8 * t];
    if (d[0] == 0) continue;
    for (int k = 1; k <= 5; ++k)
      if (d[k] == 0) d[k] = d[k - 1];
  }
  int64_t t0 = INT64_MAX, t1 = 0;
  for (int t = 0; t < nt; ++t)
    if (h[8 * t]) t0 = std::min(t0, h[8 * t]), t1 = std::max(t1, h[8 * t + 5]);
  std::vector<double> acc((size_t)S_.nlevels * 8, 0.0);
  std::vector<int> cnt(S_.nlevels, 0);
  for (int t = 0; t < nt; ++t) {
    const int64_t* d = &h[8 * t];
    if (d[0] == 0) continue;
    const int lv = S_.level[(int)d[6]];
    cnt[lv]++;
    acc[lv * 8 + 0] += (d[0] - t0) * 0.01;
    for (int k = 1; k <= 5; ++k) acc[lv * 8 + k] += (d[k] - d[k - 1]) * 0.01;
    acc[lv * 8 + 6] = std::max(acc[lv * 8 + 6], (d[5] - t0) * 0.01);
  }
  fprintf(stderr, "tree %s: %d tasks, span %.1f us\n", what, nt, (t1 - t0) * 0.01);
  if (stride == 24) {  // the critical path: from the last front to end, back through the latest child
    std::vector<int> task_of(S_.nsuper, -1);
    for (int t = 0; t < nt; ++t) task_of[(int)h[8 * t + 6]] = t;
    int t = 0;
    for (int q = 1; q < nt; ++q)
      if (h[8 * q + 5] > h[8 * t + 5]) t = q;
    for (int depth = 0; t >= 0 && depth < 12; ++depth) {
      const int64_t* d = &h[8 * t];
      const int sf = (int)d[6];
      auto us = [&](int k) { return (d[k] - t0) * 0.01; };
      fprintf(stderr, "  crit front %6d lev %d r %3d w %3d: start %6.1f %s %6.1f %s %6.1f %s %6.1f %s %6.1f %s %6.1f\n", sf,
              S_.level[sf], S_.nrows[sf], S_.first[sf + 1] - S_.first[sf], us(0), p1, us(1), p2, us(2), p3, us(3), p4,
              us(4), p5, us(5));
      int nxt = -1;
      for (int q = S_.child_ptr[sf]; q < S_.child_ptr[sf + 1]; ++q) {
        const int c = S_.child_list[q], tc = task_of[c];
        if (tc >= 0 && (nxt < 0 || h[8 * tc + 5] > h[8 * nxt + 5])) nxt = tc;
      }
      t = nxt;
    }
  }
  for (int lv = 0; lv < S_.nlevels; ++lv)
    if (cnt[lv])
      fprintf(stderr, "  level %d: %5d fronts  start %.1f  %s %.2f  %s %.2f  %s %.2f  %s %.2f  %s %.2f  last end %.1f us\n", lv,
              cnt[lv], acc[lv * 8] / cnt[lv], p1, acc[lv * 8 + 1] / cnt[lv], p2, acc[lv * 8 + 2] / cnt[lv], p3,
              acc[lv * 8 + 3] / cnt[lv], p4, acc[lv * 8 + 4] / cnt[lv], p5, acc[lv * 8 + 5] / cnt[lv], acc[lv * 8 + 6]);
}

void LDLSolver::fwd_levels(const std::vector<SolveLevel>& V, int phase, double* b, hipStream_t s) {
  const SolveTask* tasks = reinterpret_cast<const SolveTask*>(tasks_.p);
  const int efwd = 2 * epoch_ - 1;
  int32_t* cnt = counters_.p + phase * 2 * S_.nlevels;
  if (phase == 0 && !S_.lb.empty()) lb_fwd(b, s);
  for (int lev = 0; lev < (int)V.size(); ++lev) {
    const SolveLevel& L = V[lev];
    if (L.nmicro)
      TIMED(KK_FWD_TINY, L.micro_bytes, L.micro_alg, L.micro_flops,
            (k_fwd_micro<<<(unsigned)cdiv(L.nmicro, NT / MG), NT, 0, s>>>(T_, sched_.p + L.micro_off, L.nmicro, arena_, b,
                                                                         xi_, uvec_)));
    if (L.ntiny)
      TIMED(KK_FWD_TINY, L.tiny_bytes, L.tiny_alg, L.tiny_flops,
            (k_fwd_tiny<<<(unsigned)cdiv(L.ntiny, 2 * SW), NT, 0, s>>>(T_, sched_.p + L.tiny_off, L.ntiny, arena_, b, xi_,
                                                                      uvec_)));
    if (L.nsmall)
      TIMED(KK_FWD_SMALL, L.small_bytes, L.small_alg, L.small_flops,
            (k_fwd_small<<<(unsigned)L.nsmall, NT, L.small_lds, s>>>(T_, sched_.p + L.small_off, L.nsmall, arena_, b, xi_,
                                                                    uvec_)));
    if (L.nbig) {
      TIMED(KK_FWD_GATHER, L.gat_bytes, 0.0, 0.0,
            (k_fwd_gather<<<L.ngat, NT, 0, s>>>(T_, sched_.p + L.gat_off, b, uvec_, vwork_)));
      TIMED(KK_FWD_BIG, L.big_bytes, L.big_alg + L.below_alg, L.big_flops,
            (k_fwd_big<<<std::min(L.nftask, big_solve_wg_), NT, 0, s>>>(T_, tasks + L.ftask_off, L.nftask, cnt + 2 * lev,
                                                               flags_, flag_off_, efwd, arena_, vwork_, xi_, uvec_, &st_->err)));
    }
    if (lev == 0 && phase == 0 && ntree_ && nsleaf_)
      TIMED(KK_FWD_TINY, leaf_bytes_, leaf_alg_, leaf_flops_,
            (k_fwd_leaves<<<(unsigned)cdiv(nsleaf_ * LPL, NT), NT, 0, s>>>(tleaf_, (int)nsleaf_, tlrow_, arena_, b, xi_,
                                                                         T_.gbuf)));
    if (lev == 0 && phase == 0 && ntree_)
    {
      const int nlo = ntask_ - nroot_task_;  // the big roots last, in their own launch (more LDS)
      if (nlo > 0)
        TIMED(KK_FWD_TREE, tree_bytes_, tree_alg_, tree_flops_,
              (k_fwd_tree<<<(unsigned)nlo, NT, tree_lds_, s>>>(
                  T_, tc_ptr_, tc_list_, nlo, tdep_ptr_, tdep_, counters_.p + 4 * S_.nlevels, tflags_, efwd, tree_lds_ / 8,
                  arena_, b, xi_, uvec_, &st_->err, tdbg_.p, trootbwd_, D_, tchunk_, tside_.p,
                  rflag_.p ? rflag_.p + 2 : nullptr, root_pending_ && side_tree_ ? nroot_side_ : 0, repoch_)));
      if (side_tree_) root_pending_ = false;  // (root_async_) its side roots waited for the tail
      if (nroot_task_)
        TIMED(KK_FWD_TREE, nlo > 0 ? 0.0 : tree_bytes_, nlo > 0 ? 0.0 : tree_alg_, nlo > 0 ? 0.0 : tree_flops_,
              (k_root_solve<<<(unsigned)nroot_task_, RSN, root_lds_, s>>>(
                  T_, tc_list_.p + nlo, arena_, b, xi_, D_, tflags_, efwd, rflag_.p ? rflag_.p + 2 : nullptr,
                  root_pending_ ? nroot_side_ : 0, repoch_, tdbg_.p ? tdbg_.p + 8 * nlo : nullptr, rargs_)));
      if (nroot_task_ && tdbg_.p) {  // MADIPM_TREE_DEBUG: the root solve's phases
        std::vector<int64_t> h(8 * nroot_task_);
        MADIPM_HIP(hipMemcpyAsync(h.data(), tdbg_.p + 8 * nlo, h.size() * 8, hipMemcpyDeviceToHost, s));
        MADIPM_HIP(hipMemsetAsync(tdbg_.p + 8 * nlo, 0, h.size() * 8, s));  // not tree tasks' stamps
        MADIPM_HIP(hipStreamSynchronize(s));
        for (int q = 0; q < nroot_task_; ++q) {
          const int64_t* d = &h[8 * q];
          fprintf(stderr, "root solve %d: gather %.2f  wait %.2f  panel %.2f  fwd %.2f  bwd %.2f  store %.2f us\n", q,
                  (d[1] - d[0]) * 0.01, (d[2] - d[1]) * 0.01, (d[3] - d[2]) * 0.01, (d[4] - d[3]) * 0.01,
                  (d[5] - d[4]) * 0.01, (d[6] - d[5]) * 0.01);
        }
      }
      root_pending_ = false;  // (root_async_) the first k_root_solve after a factorisation waited for its tail
    }
    if (lev == 0 && phase == 0 && ntree_ && tdbg_.p)
      tree_debug_dump(s, "fwd", tdbg_.p, ntask_, "leaves", "wait", "gather", "subst", "store", 8);
    if (lev == 0) join(s);  // (no-op: root_async_ has no fronts above the tree)
  }
}

void LDLSolver::bwd_levels(const std::vector<SolveLevel>& V, int phase, double* b, hipStream_t s) {
  const SolveTask* tasks = reinterpret_cast<const SolveTask*>(tasks_.p);
  const int ebwd = 2 * epoch_;
  int32_t* cnt = counters_.p + phase * 2 * S_.nlevels;
  for (int lev = (int)V.size() - 1; lev >= 0; --lev) {
    const SolveLevel& L = V[lev];
    if (lev == 0 && phase == 0 && ntree_)
      TIMED(KK_BWD_TREE, tree_bytes_, tree_alg_, tree_flops_,
            (k_bwd_tree<<<(unsigned)ntask_, NT, tree_lds_, s>>>(T_, tc_ptr_, tc_list_, ntask_, tpar_,
                                                                 counters_.p + 4 * S_.nlevels + 1, tflags_, ebwd, arena_, D_,
                                                                 xi_, b, &st_->err, trootbwd_, tchunk_)));
    if (lev == 0 && phase == 0 && ntree_ && nsleaf_)
      TIMED(KK_BWD_TINY, leaf_bytes_, leaf_alg_, leaf_flops_,
            (k_bwd_leaves<<<(unsigned)cdiv(nsleaf_ * LPL, NT), NT, 0, s>>>(tleaf_, (int)nsleaf_, tlrow_, arena_, D_, xi_,
                                                                         b)));
    if (L.nbelow)
      TIMED(KK_BWD_BELOW, L.below_bytes, L.below_alg, 0.25 * L.below_bytes,
            (k_bwd_below<<<L.nbelow, NT, 0, s>>>(T_, sched_.p + L.below_off, bp_off_, arena_, xi_, bpart_)));
    if (L.nbig)
      TIMED(KK_BWD_BIG, L.big_bytes - L.below_bytes, L.big_alg, L.big_flops - 0.25 * L.below_bytes,
            (k_bwd_big<<<std::min(L.nbtask, big_solve_wg_), NT, 0, s>>>(T_, tasks + L.btask_off, L.nbtask, cnt + 2 * lev + 1,
                                                               flags_, flag_off_, ebwd, arena_, D_, xi_, b, bp_off_, bpart_,
                                                               &st_->err)));
    if (L.nsmall)
      TIMED(KK_BWD_SMALL, L.small_bytes, L.small_alg, L.small_flops,
            (k_bwd_small<<<(unsigned)L.nsmall, NT, L.small_lds, s>>>(T_, sched_.p + L.small_off, L.nsmall, arena_, D_, xi_,
                                                                    b)));
    if (L.ntiny)
      TIMED(KK_BWD_TINY, L.tiny_bytes, L.tiny_alg, L.tiny_flops,
            (k_bwd_tiny<<<(unsigned)cdiv(L.ntiny, 2 * SW), NT, 0, s>>>(T_, sched_.p + L.tiny_off, L.ntiny, arena_, D_, xi_,
                                                                      b)));
    if (L.nmicro)
      TIMED(KK_BWD_TINY, L.micro_bytes, L.micro_alg, L.micro_flops,
            (k_bwd_micro<<<(unsigned)cdiv(L.nmicro, NT / MG), NT, 0, s>>>(T_, sched_.p + L.micro_off, L.nmicro, arena_, D_,
                                                                         xi_, b)));
    if (phase == 0)
      for (int g : lb_at_level_[lev]) lb_bwd(g, b, s);
  }
}

// Phase 1: forward over this shard's subtrees; unsharded it is the whole solve, sharded it ends with
// the top fronts' external forward contribution in solve_xbuf().
void LDLSolver::solve_phase1(double* b, hipStream_t s) {
  if (S_.N == 0) return;
  ++epoch_;
  // the big-front task queues need zeroed counters; the tree kernels reset their own tickets
  bool queues = false;
  for (const SolveLevel& L : slev1_) queues |= L.nbig > 0;
  for (const SolveLevel& L : slev2_) queues |= L.nbig > 0;
  if (queues) MADIPM_HIP(hipMemsetAsync(counters_.p, 0, counters_.n * sizeof(int32_t), s));
  fwd_levels(slev1_, 0, b, s);
  join(s);
  if (!sharded()) {
    bwd_levels(slev1_, 0, b, s);
  } else if (nxg_) {
    k_ext_gather<<<nxg_, NT, 0, s>>>(T_, sched_.p + xg_off_, S_.shard == 0 ? 1 : 0, sx_ptr_, sx_src_, b, uvec_, xch_);
  }
  MADIPM_HIP(hipGetLastError());
}

// Phase 2 (sharded): after the all-reduce of solve_xbuf(): top forward + backward (redundant on every
// shard, which each write the top x to b), then this shard's subtrees backward, and this shard's
// subtree x packed into its slice of solve_gbuf() (other slices zeroed) for the all-gather.
void LDLSolver::solve_phase2(double* b, hipStream_t s) {
  if (S_.N == 0 || !sharded()) return;
  fwd_levels(slev2_, 1, b, s);
  bwd_levels(slev2_, 1, b, s);
  bwd_levels(slev1_, 0, b, s);
  const int64_t n = S_.nshards * gper_;
  k_gather_pack<<<(unsigned)std::min<int64_t>(1024, cdiv(n, NT)), NT, 0, s>>>(gidx_, n, gper_, S_.shard, b, gsol_);
  MADIPM_HIP(hipGetLastError());
}

// Phase 3 (sharded): after the all-gather of solve_gbuf(): the other shards' subtree x into b (every
// entry of b is then this solve's x: top and own entries from phase 2, the rest from the gather).
void LDLSolver::solve_phase3(double* b, hipStream_t s) {
  if (S_.N == 0 || !sharded()) return;
  const int64_t n = S_.nshards * gper_;
  k_gather_scatter<<<(unsigned)std::min<int64_t>(1024, cdiv(n, NT)), NT, 0, s>>>(gidx_, n, gper_, S_.shard, gsol_,
                                                                                  b);
  MADIPM_HIP(hipGetLastError());
}

void LDLSolver::solve_async(double* b, hipStream_t s) {
  solve_phase1(b, s);
  if (!sharded() || S_.N == 0) return;
  MADIPM_REQUIRE(comm_ != nullptr, "sharded LDL^T without a communicator");
  MADIPM_REQUIRE(comm_->size == S_.nshards && comm_->rank == S_.shard, "communicator does not match the shards");
  comm_->allreduce_sum(solve_xbuf(), solve_xlen(), s);
  solve_phase2(b, s);
  comm_->allgather_inplace(solve_gbuf(), gper_, s);
  solve_phase3(b, s);
}

// ------------------------------------------------------------------ ShardGroup (P shards, one device)
void local_allreduce(double* const* bufs, int nbuf, int64_t n, hipStream_t s) {
  MADIPM_REQUIRE(nbuf >= 1 && nbuf <= 16, "local_allreduce: 1..16 buffers");
  if (n <= 0) return;
  BufList B{};
  for (int q = 0; q < nbuf; ++q) B.p[q] = bufs[q];
  k_local_allreduce<<<(unsigned)std::min<int64_t>(2048, cdiv(n, NT)), NT, 0, s>>>(B, nbuf, n);
  MADIPM_HIP(hipGetLastError());
}

ShardGroup::ShardGroup(int nshards, int n, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& sopt,
                       double pivot_tol, const int32_t* user_perm) {
  MADIPM_REQUIRE(nshards >= 1 && nshards <= 16, "ShardGroup: 1..16 shards");
  for (int r = 0; r < nshards; ++r) {
    SymbolicOptions o = sopt;
    o.nshards = nshards;
    o.shard = r;
    sh_.push_back(std::make_unique<LDLSolver>(n, colptr, rowval, o, pivot_tol, user_perm));
  }
  rhs_.resize(nshards);
  for (int r = 1; r < nshards; ++r) rhs_[r].alloc(std::max(n, 1));
}

void ShardGroup::factorize_async(const double* Kx, hipStream_t s) {
  const int P = (int)sh_.size();
  for (auto& h : sh_) h->spd = spd;
  for (int r = 0; r < P; ++r) sh_[r]->fact_phase1(Kx, s);
  if (P > 1) {
    std::vector<double*> bufs;
    for (auto& h : sh_) bufs.push_back(h->fact_xbuf());
    local_allreduce(bufs.data(), P, sh_[0]->fact_xlen(), s);
  }
  for (int r = 0; r < P; ++r) sh_[r]->fact_phase2(s);
}

int ShardGroup::status(hipStream_t s, bool sync) {
  int st = sh_[0]->status(s, sync);
  for (size_t r = 1; r < sh_.size(); ++r)
    MADIPM_REQUIRE(sh_[r]->status(s, false) == st, "ShardGroup: shards disagree on the factorisation status");
  return st;
}

void ShardGroup::solve_async(double* b, hipStream_t s) {
  const int P = (int)sh_.size();
  const int n = sh_[0]->n();
  std::vector<double*> rhs(P);
  rhs[0] = b;
  for (int r = 1; r < P; ++r) {
    rhs[r] = rhs_[r].p;
    MADIPM_HIP(hipMemcpyAsync(rhs[r], b, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
  }
  for (int r = 0; r < P; ++r) sh_[r]->solve_phase1(rhs[r], s);
  if (P == 1) return;
  std::vector<double*> xb;
  for (auto& h : sh_) xb.push_back(h->solve_xbuf());
  local_allreduce(xb.data(), P, sh_[0]->solve_xlen(), s);
  for (int r = 0; r < P; ++r) sh_[r]->solve_phase2(rhs[r], s);
  std::vector<double*> gb;
  for (auto& h : sh_) gb.push_back(h->solve_gbuf());
  local_allreduce(gb.data(), P, P * sh_[0]->solve_gper(), s);  // the gather (slices zero elsewhere)
  sh_[0]->solve_phase3(b, s);  // the other shards' copies are scratch
}

}  // namespace madipm
