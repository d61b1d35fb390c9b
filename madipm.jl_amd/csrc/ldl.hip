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
#include <climits>
#include <cmath>

#include "ldl.hpp"

namespace madipm {
namespace {

constexpr int NT = 256;
typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool bad_pivot(double d, double tol) { return !(fabs(d) > tol) || isinf(d); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// largest k in [0, nf) with prefix[k] <= bid
__device__ __forceinline__ int find_item(const int32_t* __restrict__ prefix, int nf, int bid) {
  int lo = 0, hi = nf - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= bid)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
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

__global__ void k_status_init(LDLStatus* st) {
  st->fail_pivot = INT_MAX;
  st->npos = st->nneg = st->nzero = 0;
}

// ------------------------------------------------------------------ small fronts (LDS)
__global__ __launch_bounds__(NT) void k_small_factor(FrontTab T, const int32_t* __restrict__ fronts,
                                                     const double* __restrict__ Kx, double* __restrict__ arena,
                                                     double* __restrict__ D, LDLStatus* st, double tol) {
  extern __shared__ __attribute__((aligned(16))) double F[];  // r x r, col-major, ld r
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s];
  const int w = T.first[s + 1] - f0;
  const int r = T.nrows[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int q = tid; q < r * r; q += NT) F[q] = 0.0;
  __syncthreads();
  for (int64_t q = T.asm_ptr[s] + tid; q < T.asm_ptr[s + 1]; q += NT) F[T.asm_dst[q]] = Kx[T.asm_src[q]];
  __syncthreads();
  // extend-add, "pull" form: thread i owns parent row i and adds its contributions child by child
  // (fixed order => deterministic; distinct rows => no conflicts, no atomics)
  for (int i = tid; i < r; i += NT) {
    const int64_t e1 = T.crow[T.crow_off[s] + i + 1];
    for (int64_t e = T.crow[T.crow_off[s] + i]; e < e1; ++e) {
      const int c = T.ce_child[e], a = T.ce_row[e];
      const double* __restrict__ U = arena + T.u_off[c] + a;
      const int64_t ldc = T.u_ld[c];
      const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
      double* Fi = F + i;
      for (int b = 0; b <= a; ++b) Fi[rel[b] * r] += U[b * ldc];
    }
  }
  __syncthreads();
  // right-looking LDL^T; column t stays unscaled until the write-out
  for (int t = 0; t < w; ++t) {
    const double dinv = 1.0 / F[t + t * r];
    for (int j = t + 1 + wv; j < r; j += NT / 64) {
      const double ljd = F[j + t * r] * dinv;
      for (int i = j + lane; i < r; i += 64) F[i + j * r] -= F[i + t * r] * ljd;
    }
    __syncthreads();
  }
  double* __restrict__ L = arena + T.l_off[s];
  for (int t = wv; t < w; t += NT / 64) {
    const double d = F[t + t * r];
    const double dinv = 1.0 / d;
    for (int i = lane; i < r; i += 64)
      L[i + (int64_t)t * r] = (i > t) ? F[i + t * r] * dinv : (i == t ? d : 0.0);
    if (lane == 0) {
      D[f0 + t] = d;
      if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + t + 1);
    }
  }
  const int u = r - w;
  if (u > 0) {
    double* __restrict__ Uo = arena + T.u_off[s];
    for (int b = wv; b < u; b += NT / 64)
      for (int a = b + lane; a < u; a += 64) Uo[a + (int64_t)b * u] = F[(w + a) + (w + b) * r];
  }
}

// ------------------------------------------------------------------ big fronts (HBM)
__device__ __forceinline__ void tile_of(int tile, int& ti, int& tj) {
  ti = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
  while (ti * (ti + 1) / 2 > tile) --ti;
  tj = tile - ti * (ti + 1) / 2;
}

// Assembly 1/3: zero a 64x64 lower tile of F and write the original K entries that fall in it.
__global__ __launch_bounds__(NT) void k_big_tiles(FrontTab T, const int32_t* __restrict__ list, int nf,
                                                  const double* __restrict__ Kx, double* __restrict__ arena) {
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  int ti, tj;
  tile_of(blockIdx.x - prefix[k], ti, tj);
  const int r = T.nrows[s];
  const int I0 = ti * 64, I1 = min(r, I0 + 64), J0 = tj * 64, J1 = min(r, J0 + 64);
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int j = J0 + wv; j < J1; j += NT / 64) {
    const int i = I0 + lane;
    if (i < I1 && i >= j) F[i + (int64_t)j * r] = 0.0;
  }
  __syncthreads();
  // original entries: per column j, the destinations j*r + [max(I0,j), I1) form a contiguous key range
  const int64_t a0 = T.asm_ptr[s], a1 = T.asm_ptr[s + 1];
  if (a1 > a0) {
    for (int j = J0 + wv; j < J1; j += NT / 64) {
      const int64_t base = (int64_t)j * r;
      const int64_t lo = lower_bound_dev<int64_t>(T.asm_dst, a0, a1, base + max(I0, j));
      const int64_t hi = lower_bound_dev<int64_t>(T.asm_dst, lo, a1, base + I1);
      for (int64_t q = lo + lane; q < hi; q += 64) F[T.asm_dst[q]] = Kx[T.asm_src[q]];
    }
  }
}

// Assembly 2/3: children with small update blocks, "pull" form (thread = parent row, children in order).
__global__ __launch_bounds__(NT) void k_big_pull(FrontTab T, const int32_t* __restrict__ list, int nf,
                                                 double* __restrict__ arena) {
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  const int r = T.nrows[s];
  const int i = (blockIdx.x - prefix[k]) * NT + threadIdx.x;
  if (i >= r) return;
  double* __restrict__ Fi = arena + T.l_off[s] + i;
  const int64_t e1 = T.crow[T.crow_off[s] + i + 1];
  for (int64_t e = T.crow[T.crow_off[s] + i]; e < e1; ++e) {
    const int c = T.ce_child[e], a = T.ce_row[e];
    const double* __restrict__ U = arena + T.u_off[c] + a;
    const int64_t ldc = T.u_ld[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    for (int b = 0; b <= a; ++b) Fi[(int64_t)rel[b] * r] += U[b * ldc];
  }
}

// Assembly 3/3: children with large update blocks, column-wise per 64x64 tile, children in order.
__global__ __launch_bounds__(NT) void k_big_bigch(FrontTab T, const int32_t* __restrict__ list, int nf,
                                                  double* __restrict__ arena) {
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  int ti, tj;
  tile_of(blockIdx.x - prefix[k], ti, tj);
  const int r = T.nrows[s];
  const int I0 = ti * 64, I1 = min(r, I0 + 64), J0 = tj * 64, J1 = min(r, J0 + 64);
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int ci = T.bigch_ptr[s]; ci < T.bigch_ptr[s + 1]; ++ci) {
    const int c = T.bigch_list[ci];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const double* __restrict__ U = arena + T.u_off[c];
    const int64_t ldc = T.u_ld[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    const int b0 = (int)lower_bound_dev<int32_t>(rel, 0, uc, J0);
    const int b1 = (int)lower_bound_dev<int32_t>(rel, b0, uc, J1);
    const int c0 = (int)lower_bound_dev<int32_t>(rel, b0, uc, I0);
    const int c1 = (int)lower_bound_dev<int32_t>(rel, c0, uc, I1);
    for (int b = b0 + wv; b < b1; b += NT / 64) {
      const int64_t rb = (int64_t)rel[b] * r;
      for (int a = max(b, c0) + lane; a < c1; a += 64) F[rel[a] + rb] += U[a + b * ldc];
    }
    __syncthreads();
  }
}

// Diagonal block of 64-column panel `step` (one workgroup per front): factor it in LDS, write
// L11 and D, and form M = L11^{-T} D^{-1} for the MFMA solve of the rows below (k_big_trsm).
__global__ __launch_bounds__(NT) void k_big_diag(FrontTab T, const int32_t* __restrict__ list, int nf, int step,
                                                 double* __restrict__ arena, double* __restrict__ D,
                                                 double* __restrict__ Mbuf, LDLStatus* st, double tol) {
  constexpr int LD = 65;
  __shared__ double A[64 * LD];
  __shared__ double X[64 * 65];
  __shared__ double dinv[64];
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  const int rb = blockIdx.x - prefix[k];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int k0 = step * 64, kw = min(64, w - k0);
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int j = wv; j < kw; j += NT / 64)
    if (lane >= j && lane < kw) A[lane + j * LD] = F[(k0 + lane) + (int64_t)(k0 + j) * r];
  __syncthreads();
  for (int t = 0; t < kw; ++t) {
    const double di = 1.0 / A[t + t * LD];
    for (int j = t + 1 + wv; j < kw; j += NT / 64) {
      const double ljd = A[j + t * LD] * di;
      if (lane >= j && lane < kw) A[lane + j * LD] -= A[lane + t * LD] * ljd;
    }
    __syncthreads();
  }
  if (tid < kw) dinv[tid] = 1.0 / A[tid + tid * LD];
  __syncthreads();
  for (int j = wv; j < kw; j += NT / 64)
    if (lane > j && lane < kw) A[lane + j * LD] *= dinv[j];
  __syncthreads();
  (void)rb;
  for (int j = wv; j < kw; j += NT / 64)
    if (lane >= j && lane < kw) F[(k0 + lane) + (int64_t)(k0 + j) * r] = A[lane + j * LD];
  if (tid < kw) {
    const double d = A[tid + tid * LD];
    D[f0 + k0 + tid] = d;
    if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + k0 + tid + 1);
  }
  // M = L11^{-T} D^{-1} (so that the rows below solve as L21 = F21 M, an MFMA product):
  // thread j forms column j of X = L11^{-1} by forward substitution (all lanes step through the
  // same (i, k) so the L11 reads broadcast), then writes row j of M: M[j][t] = X[t][j] / d_t.
  if (tid < 64) {
    const int j = tid;
    for (int i = 0; i < 64; ++i) X[i * 65 + j] = (i == j) ? 1.0 : 0.0;
    for (int i = 1; i < kw; ++i) {
      double acc = 0.0;
      for (int q = 0; q < i; ++q) acc += A[i + q * LD] * X[q * 65 + j];
      if (i > j) X[i * 65 + j] = -acc;
    }
    double* __restrict__ Mrow = Mbuf + (int64_t)T.bigslot[s] * 4096 + j * 64;
    for (int t = 0; t < 64; ++t) Mrow[t] = (t < kw && j < kw && t >= j) ? X[t * 65 + j] * dinv[t] : 0.0;
  }
}

// Rows below the diagonal block of panel `step`: L21 = F21 * M (64-row tiles, f64 MFMA 16x16x4),
// computed as the transpose D'[t][i] = sum_k M[k][t] F21[i][k] so that lanes run along F's rows.
__global__ __launch_bounds__(NT) void k_big_trsm(FrontTab T, const int32_t* __restrict__ list, int nf, int step,
                                                 double* __restrict__ arena, const double* __restrict__ Mbuf) {
  constexpr int LDT = 80;
  __shared__ __attribute__((aligned(16))) double Ms[64 * LDT];
  __shared__ __attribute__((aligned(16))) double At[64 * LDT];
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  const int rt = blockIdx.x - prefix[k];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int k0 = step * 64, kw = min(64, w - k0);
  const int I0 = k0 + kw + rt * 64;
  double* __restrict__ F = arena + T.l_off[s];
  const double* __restrict__ M = Mbuf + (int64_t)T.bigslot[s] * 4096;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  (void)f0;
  for (int kk = wv; kk < 64; kk += 4) {
    Ms[kk * LDT + lane] = M[kk * 64 + lane];
    At[kk * LDT + lane] = (kk < kw && I0 + lane < r) ? F[(I0 + lane) + (int64_t)(k0 + kk) * r] : 0.0;
  }
  __syncthreads();
  const int qt = (wv >> 1) * 32, qi = (wv & 1) * 32;
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int kk = ks * 4 + (lane >> 4);
    const double a0 = Ms[kk * LDT + qt + (lane & 15)];
    const double a1 = Ms[kk * LDT + qt + 16 + (lane & 15)];
    const double b0 = At[kk * LDT + qi + (lane & 15)];
    const double b1 = At[kk * LDT + qi + 16 + (lane & 15)];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
#pragma unroll
  for (int bt = 0; bt < 2; ++bt)
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = I0 + qi + bi * 16 + (lane & 15);
        const int t = qt + bt * 16 + (lane >> 4) + 4 * g;
        if (i < r && t < kw) F[i + (int64_t)(k0 + t) * r] = acc[bt][bi][g];
      }
}

// Trailing update of one 64x64 lower tile: C -= (L_I D) L_J^T, f64 MFMA 16x16x4.
__global__ __launch_bounds__(NT) void k_big_update(FrontTab T, const int32_t* __restrict__ list, int nf, int step,
                                                   double* __restrict__ arena, const double* __restrict__ D) {
  constexpr int LDT = 80;  // [k][row] layout: conflict-free ds_read_b64 for the 16x4 operand pattern
  __shared__ __attribute__((aligned(16))) double Wt[32 * LDT];
  __shared__ __attribute__((aligned(16))) double Lt[32 * LDT];
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  const int tile = blockIdx.x - prefix[k];
  int ti = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
  while (ti * (ti + 1) / 2 > tile) --ti;
  const int tj = tile - ti * (ti + 1) / 2;
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int k0 = step * 64, kw = min(64, w - k0), c0 = k0 + kw;
  const int I0 = c0 + ti * 64, J0 = c0 + tj * 64;
  double* __restrict__ F = arena + T.l_off[s];
  const double* __restrict__ Dp = D + f0 + k0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int qr = (wv >> 1) * 32, qc = (wv & 1) * 32;
  dbl4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  for (int kc = 0; kc < kw; kc += 32) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = wv + 4 * e;
      const int kg = kc + kk;
      double wvv = 0.0, lv = 0.0;
      if (kg < kw) {
        const int64_t col = (int64_t)(k0 + kg) * r;
        if (I0 + lane < r) wvv = F[(I0 + lane) + col] * Dp[kg];
        if (J0 + lane < r) lv = F[(J0 + lane) + col];
      }
      Wt[kk * LDT + lane] = wvv;
      Lt[kk * LDT + lane] = lv;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
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
    __syncthreads();
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
        if (i < r && j < r) F[i + (int64_t)j * r] -= acc[bj][bi][g];
      }
}

__global__ void k_inertia(const double* __restrict__ D, int n, LDLStatus* st) {
  int pos = 0, neg = 0, zero = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const double d = D[i];
    pos += d > 0.0;
    neg += d < 0.0;
    zero += !(d > 0.0) && !(d < 0.0);
  }
  for (int o = 32; o > 0; o >>= 1) {
    pos += __shfl_down(pos, o, 64);
    neg += __shfl_down(neg, o, 64);
    zero += __shfl_down(zero, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&st->npos, pos);
    atomicAdd(&st->nneg, neg);
    atomicAdd(&st->nzero, zero);
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
constexpr int SMALL_SOLVE = 128;
constexpr int SW = 4;  // waves (= small fronts) per workgroup

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

__global__ __launch_bounds__(NT) void k_fwd_small(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                  const double* __restrict__ arena, const double* __restrict__ b,
                                                  double* __restrict__ xi, double* __restrict__ uvec) {
  __shared__ double vs[SW][SMALL_SOLVE];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = blockIdx.x * SW + wv;
  if (q >= nf) return;
  const int s = fronts[q];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  double* v = vs[wv];
  const double* __restrict__ L = arena + T.l_off[s];
  for (int i = lane; i < r; i += 64) v[i] = (i < w) ? b[T.perm[f0 + i]] : 0.0;
  wave_sync();
  for (int ci = T.child_ptr[s]; ci < T.child_ptr[s + 1]; ++ci) {
    const int c = T.child_list[ci];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const double* __restrict__ uv = uvec + T.uvec_off[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    for (int t = lane; t < uc; t += 64) v[rel[t]] += uv[t];
    wave_sync();
  }
  for (int t = 0; t < w; ++t) {
    const double xt = v[t];
    const double* __restrict__ Lc = L + t * r;
    for (int i = t + 1 + lane; i < r; i += 64) v[i] -= Lc[i] * xt;
    wave_sync();
  }
  double* __restrict__ uo = uvec + T.uvec_off[s];
  for (int i = lane; i < r; i += 64) {
    if (i < w)
      xi[f0 + i] = v[i];
    else
      uo[i - w] = v[i];
  }
}

__global__ __launch_bounds__(NT) void k_bwd_small(FrontTab T, const int32_t* __restrict__ fronts, int nf,
                                                  const double* __restrict__ arena, const double* __restrict__ D,
                                                  double* __restrict__ xi, double* __restrict__ out) {
  __shared__ double vs[SW][SMALL_SOLVE];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = blockIdx.x * SW + wv;
  if (q >= nf) return;
  const int s = fronts[q];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  double* v = vs[wv];
  const double* __restrict__ L = arena + T.l_off[s];
  const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
  for (int i = lane; i < r; i += 64) v[i] = (i < w) ? xi[f0 + i] / D[f0 + i] : xi[rows[i]];
  wave_sync();
  // v[t] -= L21(:,t)^T x(below), four columns per pass
  for (int t0 = 0; t0 < w; t0 += 4) {
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = w + lane; i < r; i += 64) {
      const double vi = v[i];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (t0 + k < w) a[k] += L[i + (t0 + k) * r] * vi;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = wave_sum(a[k]);
    if (lane == 0)
      for (int k = 0; k < 4 && t0 + k < w; ++k) v[t0 + k] -= a[k];
  }
  wave_sync();
  for (int t = w - 1; t > 0; --t) {
    const double xt = v[t];
    for (int i = lane; i < t; i += 64) v[i] -= L[t + i * r] * xt;
    wave_sync();
  }
  for (int i = lane; i < w; i += 64) {
    xi[f0 + i] = v[i];
    out[T.perm[f0 + i]] = v[i];
  }
}

// initial forward vector of a big front (own b entries + children's update vectors), in HBM
__global__ __launch_bounds__(NT) void k_fwd_gather(FrontTab T, const int32_t* __restrict__ fronts,
                                                   const double* __restrict__ b, const double* __restrict__ uvec,
                                                   double* __restrict__ vwork) {
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  double* __restrict__ v = vwork + T.row_ptr[s];
  for (int i = threadIdx.x; i < r; i += NT) v[i] = (i < w) ? b[T.perm[f0 + i]] : 0.0;
  __syncthreads();
  for (int ci = T.child_ptr[s]; ci < T.child_ptr[s + 1]; ++ci) {
    const int c = T.child_list[ci];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const double* __restrict__ uv = uvec + T.uvec_off[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    for (int t = threadIdx.x; t < uc; t += NT) v[rel[t]] += uv[t];
    __syncthreads();
  }
}

__device__ __forceinline__ bool wait_flag(int32_t* f, int epoch, int32_t* err) {
  int spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 25)) {
      atomicExch(err, 1);
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

// Forward, big fronts: task = (front, 64-row block i).  acc(rows) = v(rows) - sum_{panels p < i} L(rows,p) x_p,
// then (pivot block) x_i = L_ii^{-1} acc, published through flags[flag_off[front] + i].
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
    // prefetch the diagonal block (columns row0 .. row0+kw-1 of this row block) into LDS
    for (int tt = g; tt < kw; tt += 4)
      Ld[tt * 65 + lane] = (lane < nrow) ? L[row + (int64_t)(row0 + tt) * r] : 0.0;
    double acc = 0.0;
    for (int p = 0; p < np; ++p) {
      double lv[16];
      const int cb = p * 64 + g * 16;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc)
        lv[cc] = (lane < nrow && cb + cc < w) ? L[row + (int64_t)(cb + cc) * r] : 0.0;
      if (tid == 0) wait_flag(&flags[flag_off[s] + p], epoch, err);
      __syncthreads();
      if (tid < 64) {
        const int c = p * 64 + tid;
        xs[tid] = (c < w) ? xi[f0 + c] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) acc += lv[cc] * xs[g * 16 + cc];
      __syncthreads();
    }
    part[g][lane] = acc;
    __syncthreads();
    if (g == 0) {
      double a = (lane < nrow) ? vwork[T.row_ptr[s] + row] - ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]))
                               : 0.0;
      for (int tt = 0; tt < kw; ++tt) {
        const double xt = __shfl(a, tt, 64);
        if (lane > tt) a -= Ld[tt * 65 + lane] * xt;
      }
      if (lane < nrow) {
        if (row < w)
          xi[f0 + row] = a;
        else
          uvec[T.uvec_off[s] + row - w] = a;
      }
      if (pivot_blk) publish_flag(&flags[flag_off[s] + i], epoch);
    }
    __syncthreads();
  }
}

// Backward, big fronts: task = (front, 64-column pivot panel p), processed from the last panel down.
// acc(cols) = D^{-1} y(cols) - L(below,cols)^T x(below) - sum_{q > p} L(q-block,cols)^T x_q; x_p = L_pp^{-T} acc.
__global__ __launch_bounds__(NT) void k_bwd_big(FrontTab T, const SolveTask* __restrict__ tasks, int ntasks,
                                                int32_t* counter, int32_t* flags, const int32_t* __restrict__ flag_off,
                                                int epoch, const double* __restrict__ arena,
                                                const double* __restrict__ D, double* __restrict__ xi,
                                                double* __restrict__ out, int32_t* err) {
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
    const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
    const int c0 = p * 64, kw = min(64, w - c0);
    const int npan = (w + 63) >> 6;
    // diagonal block L(c0+i, c0+j) -> Ld[i*65+j]
    for (int j = g; j < kw; j += 4) Ld[lane * 65 + j] = (lane < kw) ? L[(c0 + lane) + (int64_t)(c0 + j) * r] : 0.0;
    double acc = 0.0;  // partial for column c0+lane over this wave's rows of each tile
    // row tiles: below rows first (independent), then pivot panels q = npan-1 .. p+1 (wait for each)
    const int nbelow = (r - w + 63) >> 6;
    for (int k = 0; k < nbelow + (npan - 1 - p); ++k) {
      int rb, nr;
      const bool below = k < nbelow;
      if (below) {
        rb = w + k * 64;
        nr = min(64, r - rb);
      } else {
        const int q = npan - 1 - (k - nbelow);
        rb = q * 64;
        nr = min(64, w - rb);
        if (tid == 0) wait_flag(&flags[flag_off[s] + q], epoch, err);
        __syncthreads();
      }
      // stage the 64 x 64 tile L(rb.., c0..) (coalesced over rows) and the x values of its rows
      for (int j = g; j < kw; j += 4) tile[lane * 65 + j] = (lane < nr) ? L[(rb + lane) + (int64_t)(c0 + j) * r] : 0.0;
      if (tid < 64) xr[tid] = (tid < nr) ? (below ? xi[rows[rb + tid]] : xi[f0 + rb + tid]) : 0.0;
      __syncthreads();
      // column c0+lane, rows g*16 .. g*16+15 of the tile
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) acc += tile[(g * 16 + rr) * 65 + lane] * xr[g * 16 + rr];
      __syncthreads();
    }
    part[g][lane] = acc;
    __syncthreads();
    if (g == 0) {
      double a = 0.0;
      if (lane < kw) {
        const int c = f0 + c0 + lane;
        a = xi[c] / D[c] - ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]));
      }
      for (int tt = kw - 1; tt > 0; --tt) {
        const double xt = __shfl(a, tt, 64);
        if (lane < tt) a -= Ld[tt * 65 + lane] * xt;
      }
      if (lane < kw) {
        const int c = f0 + c0 + lane;
        xi[c] = a;
        out[T.perm[c]] = a;
      }
      publish_flag(&flags[flag_off[s] + p], epoch);
    }
    __syncthreads();
  }
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace

LDLSolver::LDLSolver(int n, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& sopt,
                     double ptol, const int32_t* user_perm)
    : pivot_tol(ptol) {
  symbolic_analyze(n, colptr, rowval, sopt, user_perm, S_);
  const SymbolicPlan& S = S_;
  first_.upload(S.first);
  nrows_.upload(S.nrows);
  row_ptr_.upload(S.row_ptr);
  rows_.upload(S.rows);
  l_off_.upload(S.l_off);
  u_off_.upload(S.u_off);
  u_ld_.upload(S.u_ld);
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
  crow_off_.upload(S.crow_off);
  crow_.upload(S.crow);
  ce_child_.upload(S.ce_child);
  ce_row_.upload(S.ce_row);
  bigch_ptr_.upload(S.bigch_ptr);
  bigch_list_.upload(S.bigch_list);
  T_.crow_off = crow_off_;
  T_.crow = crow_;
  T_.ce_child = ce_child_;
  T_.ce_row = ce_row_;
  T_.bigch_ptr = bigch_ptr_;
  T_.bigch_list = bigch_list_;
  {
    std::vector<int32_t> slot(std::max(S.nsuper, 1), -1);
    int nslot = 0;
    for (int s = 0; s < S.nsuper; ++s)
      if (S.is_big[s]) slot[s] = nslot++;
    bigslot_.upload(slot);
    minv_.alloc((int64_t)std::max(nslot, 1) * 4096);
    T_.bigslot = bigslot_;
  }

  // ---- launch schedule
  std::vector<int32_t> sched;
  const int ns = S.nsuper;
  for (int lev = 0; lev < S.nlevels; ++lev) {
    std::vector<int32_t> cls[3], big;
    for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) {
      const int s = S.level_list[q];
      const int r = S.nrows[s];
      if (!S.is_big[s])
        cls[r <= 32 ? 0 : (r <= 64 ? 1 : 2)].push_back(s);
      else
        big.push_back(s);
    }
    for (int c = 0; c < 3; ++c)
      if (!cls[c].empty()) {
        fact_.push_back({SMALL32 + c, 0, (int64_t)sched.size(), (int)cls[c].size(), (int64_t)cls[c].size()});
        sched.insert(sched.end(), cls[c].begin(), cls[c].end());
      }
    if (big.empty()) continue;
    auto add_big = [&](int kind, int step, const std::vector<int32_t>& fl, const std::vector<int64_t>& cnt) {
      std::vector<int32_t> f2;
      std::vector<int64_t> c2;
      for (size_t q = 0; q < fl.size(); ++q)
        if (cnt[q] > 0) {
          f2.push_back(fl[q]);
          c2.push_back(cnt[q]);
        }
      if (f2.empty()) return;
      Launch L{kind, step, (int64_t)sched.size(), (int)f2.size(), 0};
      sched.insert(sched.end(), f2.begin(), f2.end());
      int64_t acc = 0;
      for (size_t q = 0; q < f2.size(); ++q) {
        sched.push_back((int32_t)acc);
        acc += c2[q];
      }
      sched.push_back((int32_t)acc);
      MADIPM_REQUIRE(acc < INT_MAX, "launch too large");
      L.items = acc;
      fact_.push_back(L);
    };
    std::vector<int64_t> ctile(big.size()), cpull(big.size()), cbig(big.size());
    int maxsteps = 0;
    for (size_t q = 0; q < big.size(); ++q) {
      const int s = big[q];
      const int64_t nt = cdiv(S.nrows[s], 64);
      ctile[q] = nt * (nt + 1) / 2;
      const bool has_pull = S.crow[S.crow_off[s] + S.nrows[s]] > S.crow[S.crow_off[s]];
      cpull[q] = has_pull ? cdiv(S.nrows[s], NT) : 0;
      cbig[q] = (S.bigch_ptr[s + 1] > S.bigch_ptr[s]) ? ctile[q] : 0;
      maxsteps = std::max<int>(maxsteps, (int)cdiv(S.first[s + 1] - S.first[s], 64));
    }
    add_big(BIG_TILES, 0, big, ctile);
    add_big(BIG_PULL, 0, big, cpull);
    add_big(BIG_BIGCH, 0, big, cbig);
    for (int p = 0; p < maxsteps; ++p) {
      std::vector<int64_t> cd(big.size(), 0), ct(big.size(), 0), cu(big.size(), 0);
      for (size_t q = 0; q < big.size(); ++q) {
        const int s = big[q];
        const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
        if (cdiv(w, 64) <= p) continue;
        const int k0 = p * 64, kw = std::min(64, w - k0);
        const int64_t below = r - k0 - kw;
        cd[q] = 1;
        const int64_t nt = cdiv(below, 64);
        ct[q] = nt;
        cu[q] = nt * (nt + 1) / 2;
      }
      add_big(BIG_DIAG, p, big, cd);
      add_big(BIG_TRSM, p, big, ct);
      add_big(BIG_UPDATE, p, big, cu);
    }
  }
  // ---- solve schedule: per level, small fronts (wave per front) and big fronts (task queues)
  {
    std::vector<int32_t> flag_off(ns, 0);
    int64_t nflags = 0;
    for (int s = 0; s < ns; ++s)
      if (S.nrows[s] > 128) {
        flag_off[s] = (int32_t)nflags;
        nflags += cdiv(S.first[s + 1] - S.first[s], 64);
      }
    std::vector<int32_t> tasks;
    for (int lev = 0; lev < S.nlevels; ++lev) {
      std::vector<int32_t> small, big;
      for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) {
        const int s = S.level_list[q];
        (S.nrows[s] > 128 ? big : small).push_back(s);
      }
      SolveLevel L{};
      L.small_off = (int64_t)sched.size();
      L.nsmall = (int)small.size();
      sched.insert(sched.end(), small.begin(), small.end());
      L.big_off = (int64_t)sched.size();
      L.nbig = (int)big.size();
      sched.insert(sched.end(), big.begin(), big.end());
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
      slev_.push_back(L);
    }
    tasks_.upload(tasks);
    flag_off_.upload(flag_off);
    flags_.alloc(std::max<int64_t>(nflags, 1));
    flags_.zero();
    counters_.alloc(2 * std::max(S.nlevels, 1));
    err_.alloc(1);
    err_.zero();
  }
  sched_.upload(sched);
  arena_.alloc(std::max<int64_t>(S.arena_size, 2));
  D_.alloc(std::max(S.N, 1));
  xi_.alloc(std::max(S.N, 1));
  uvec_.alloc(std::max<int64_t>(S.uvec_size, 1));
  vwork_.alloc(std::max<int64_t>(S.row_ptr[ns], 1));
  status_.alloc(1);
  MADIPM_HIP(hipHostMalloc((void**)&h_status_, sizeof(LDLStatus), hipHostMallocDefault));
  static bool attr_done = false;
  if (!attr_done) {
    MADIPM_HIP(hipFuncSetAttribute((const void*)k_small_factor, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   128 * 128 * 8));
    attr_done = true;
  }
  MADIPM_HIP(hipDeviceSynchronize());
}

LDLSolver::~LDLSolver() {
  if (h_status_) (void)hipHostFree(h_status_);
}

void LDLSolver::factorize_async(const double* Kx, hipStream_t s) {
  if (S_.N == 0) return;
  k_status_init<<<1, 1, 0, s>>>(status_);
  for (const Launch& L : fact_) {
    const int32_t* list = sched_.p + L.off;
    switch (L.kind) {
      case SMALL32:
      case SMALL64:
      case SMALL128: {
        const int R = L.kind == SMALL32 ? 32 : (L.kind == SMALL64 ? 64 : 128);
        k_small_factor<<<(unsigned)L.items, NT, R * R * 8, s>>>(T_, list, Kx, arena_, D_, status_, pivot_tol);
        break;
      }
      case BIG_TILES:
        k_big_tiles<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, Kx, arena_);
        break;
      case BIG_PULL:
        k_big_pull<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, arena_);
        break;
      case BIG_BIGCH:
        k_big_bigch<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, arena_);
        break;
      case BIG_DIAG:
        k_big_diag<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, L.step, arena_, D_, minv_, status_, pivot_tol);
        break;
      case BIG_TRSM:
        k_big_trsm<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, L.step, arena_, minv_);
        break;
      case BIG_UPDATE:
        k_big_update<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, L.step, arena_, D_);
        break;
    }
  }
  const int nb = (int)std::min<int64_t>(1024, cdiv(S_.N, NT));
  k_inertia<<<nb, NT, 0, s>>>(D_, S_.N, status_);
  MADIPM_HIP(hipGetLastError());
  MADIPM_HIP(hipMemcpyAsync(h_status_, status_.p, sizeof(LDLStatus), hipMemcpyDeviceToHost, s));
}

int LDLSolver::status(hipStream_t s) {
  if (S_.N == 0) {
    factorized = true;
    return 0;
  }
  MADIPM_HIP(hipStreamSynchronize(s));
  npos = h_status_->npos;
  nneg = h_status_->nneg;
  nzero = h_status_->nzero;
  const int fp = h_status_->fail_pivot;
  factorized = (fp == INT_MAX);
  return factorized ? 0 : fp;
}

void LDLSolver::solve_async(double* b, hipStream_t s) {
  if (S_.N == 0) return;
  ++epoch_;
  const int efwd = 2 * epoch_ - 1, ebwd = 2 * epoch_;
  MADIPM_HIP(hipMemsetAsync(counters_.p, 0, counters_.n * sizeof(int32_t), s));
  const SolveTask* tasks = reinterpret_cast<const SolveTask*>(tasks_.p);
  const int nl = (int)slev_.size();
  for (int lev = 0; lev < nl; ++lev) {
    const SolveLevel& L = slev_[lev];
    if (L.nsmall) k_fwd_small<<<(unsigned)cdiv(L.nsmall, SW), NT, 0, s>>>(T_, sched_.p + L.small_off, L.nsmall, arena_, b, xi_, uvec_);
    if (L.nbig) {
      k_fwd_gather<<<L.nbig, NT, 0, s>>>(T_, sched_.p + L.big_off, b, uvec_, vwork_);
      k_fwd_big<<<std::min(L.nftask, 512), NT, 0, s>>>(T_, tasks + L.ftask_off, L.nftask, counters_.p + 2 * lev, flags_,
                                                         flag_off_, efwd, arena_, vwork_, xi_, uvec_, err_);
    }
  }
  for (int lev = nl - 1; lev >= 0; --lev) {
    const SolveLevel& L = slev_[lev];
    if (L.nbig)
      k_bwd_big<<<std::min(L.nbtask, 512), NT, 0, s>>>(T_, tasks + L.btask_off, L.nbtask, counters_.p + 2 * lev + 1,
                                                         flags_, flag_off_, ebwd, arena_, D_, xi_, b, err_);
    if (L.nsmall) k_bwd_small<<<(unsigned)cdiv(L.nsmall, SW), NT, 0, s>>>(T_, sched_.p + L.small_off, L.nsmall, arena_, D_, xi_, b);
  }
  MADIPM_HIP(hipGetLastError());
}

}  // namespace madipm
