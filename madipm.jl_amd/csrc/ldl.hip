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
constexpr int SOLVE_LDS = 4096;  // doubles of LDS for the solve work vector
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
  for (int ci = T.child_ptr[s]; ci < T.child_ptr[s + 1]; ++ci) {
    const int c = T.child_list[ci];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const double* __restrict__ U = arena + T.u_off[c];
    const int ldc = T.u_ld[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    for (int b = wv; b < uc; b += NT / 64) {
      const int rb = rel[b] * r;
      for (int a = b + lane; a < uc; a += 64) F[rel[a] + rb] += U[a + (int64_t)b * ldc];
    }
    __syncthreads();
  }
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
__global__ __launch_bounds__(NT) void k_big_assemble(FrontTab T, const int32_t* __restrict__ list, int nf,
                                                     const double* __restrict__ Kx, double* __restrict__ arena) {
  const int32_t* prefix = list + nf;
  const int k = find_item(prefix, nf, blockIdx.x);
  const int s = list[k];
  const int cb = blockIdx.x - prefix[k];
  const int r = T.nrows[s];
  const int j0 = cb * 64, j1 = min(r, j0 + 64);
  double* __restrict__ F = arena + T.l_off[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int j = j0 + wv; j < j1; j += NT / 64)
    for (int i = j + lane; i < r; i += 64) F[i + (int64_t)j * r] = 0.0;
  __syncthreads();
  {
    const int64_t lo = lower_bound_dev<int64_t>(T.asm_dst, T.asm_ptr[s], T.asm_ptr[s + 1], (int64_t)j0 * r);
    const int64_t hi = lower_bound_dev<int64_t>(T.asm_dst, lo, T.asm_ptr[s + 1], (int64_t)j1 * r);
    for (int64_t q = lo + tid; q < hi; q += NT) F[T.asm_dst[q]] = Kx[T.asm_src[q]];
  }
  __syncthreads();
  for (int ci = T.child_ptr[s]; ci < T.child_ptr[s + 1]; ++ci) {
    const int c = T.child_list[ci];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const double* __restrict__ U = arena + T.u_off[c];
    const int64_t ldc = T.u_ld[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    const int b0 = (int)lower_bound_dev<int32_t>(rel, 0, uc, j0);
    const int b1 = (int)lower_bound_dev<int32_t>(rel, b0, uc, j1);
    for (int b = b0 + wv; b < b1; b += NT / 64) {
      const int64_t rb = (int64_t)rel[b] * r;
      for (int a = b + lane; a < uc; a += 64) F[rel[a] + rb] += U[a + b * ldc];
    }
    __syncthreads();
  }
}

// One 64-column panel: factor the diagonal block in LDS, solve the rows below.
__global__ __launch_bounds__(NT) void k_big_panel(FrontTab T, const int32_t* __restrict__ list, int nf, int step,
                                                  double* __restrict__ arena, double* __restrict__ D,
                                                  LDLStatus* st, double tol) {
  constexpr int LD = 65;
  __shared__ double A[64 * LD];
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
  if (rb == 0) {
    for (int j = wv; j < kw; j += NT / 64)
      if (lane >= j && lane < kw) F[(k0 + lane) + (int64_t)(k0 + j) * r] = A[lane + j * LD];
    if (tid < kw) {
      const double d = A[tid + tid * LD];
      D[f0 + k0 + tid] = d;
      if (bad_pivot(d, tol)) atomicMin(&st->fail_pivot, f0 + k0 + tid + 1);
    }
  }
  const int i = k0 + kw + rb * NT + tid;
  if (i < r) {
    double x[64];
#pragma unroll
    for (int t = 0; t < 64; ++t)
      if (t < kw) x[t] = F[i + (int64_t)(k0 + t) * r];
#pragma unroll
    for (int t = 1; t < 64; ++t) {
      if (t < kw) {
        double acc = x[t];
#pragma unroll
        for (int q = 0; q < t; ++q) acc -= A[t + q * LD] * x[q];
        x[t] = acc;
      }
    }
#pragma unroll
    for (int t = 0; t < 64; ++t)
      if (t < kw) F[i + (int64_t)(k0 + t) * r] = x[t] * dinv[t];
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
// Forward (multifrontal form): v = [b(own cols); 0] + extend-add of children's update vectors;
// v[0:w] <- L11^{-1} v[0:w]; v[w:] -= L21 v[0:w]; own part -> xi, rest -> this front's update vector.
__global__ __launch_bounds__(NT) void k_fwd(FrontTab T, const int32_t* __restrict__ fronts,
                                            const double* __restrict__ arena, const double* __restrict__ b,
                                            double* __restrict__ xi, double* __restrict__ uvec,
                                            double* __restrict__ vwork) {
  __shared__ double vl[SOLVE_LDS];
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int tid = threadIdx.x;
  double* v = (r <= SOLVE_LDS) ? vl : vwork + T.row_ptr[s];
  const double* __restrict__ L = arena + T.l_off[s];
  for (int t = tid; t < r; t += NT) v[t] = (t < w) ? b[T.perm[f0 + t]] : 0.0;
  __syncthreads();
  for (int ci = T.child_ptr[s]; ci < T.child_ptr[s + 1]; ++ci) {
    const int c = T.child_list[ci];
    const int uc = T.nrows[c] - (T.first[c + 1] - T.first[c]);
    const double* __restrict__ uv = uvec + T.uvec_off[c];
    const int32_t* __restrict__ rel = T.rel + T.rel_ptr[c];
    for (int t = tid; t < uc; t += NT) v[rel[t]] += uv[t];
    __syncthreads();
  }
  for (int t = 0; t < w; ++t) {
    const double xt = v[t];
    const double* __restrict__ Lc = L + (int64_t)t * r;
    for (int i = t + 1 + tid; i < r; i += NT) v[i] -= Lc[i] * xt;
    __syncthreads();
  }
  double* __restrict__ uo = uvec + T.uvec_off[s];
  for (int t = tid; t < r; t += NT) {
    if (t < w)
      xi[f0 + t] = v[t];
    else
      uo[t - w] = v[t];
  }
}

// Backward: v[0:w] = D^{-1} xi(own) - L21^T x(below); then unit upper solve with L11^T.
__global__ __launch_bounds__(NT) void k_bwd(FrontTab T, const int32_t* __restrict__ fronts,
                                            const double* __restrict__ arena, const double* __restrict__ D,
                                            double* __restrict__ xi, double* __restrict__ out,
                                            double* __restrict__ vwork) {
  __shared__ double vl[SOLVE_LDS];
  const int s = fronts[blockIdx.x];
  const int f0 = T.first[s], w = T.first[s + 1] - f0, r = T.nrows[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double* v = (r <= SOLVE_LDS) ? vl : vwork + T.row_ptr[s];
  const double* __restrict__ L = arena + T.l_off[s];
  const int32_t* __restrict__ rows = T.rows + T.row_ptr[s];
  for (int t = tid; t < r; t += NT) v[t] = (t < w) ? xi[f0 + t] / D[f0 + t] : xi[rows[t]];
  __syncthreads();
  for (int t = wv; t < w; t += NT / 64) {
    const double* __restrict__ Lc = L + (int64_t)t * r;
    double acc = 0.0;
    for (int i = w + lane; i < r; i += 64) acc += Lc[i] * v[i];
    acc = wave_sum(acc);
    if (lane == 0) v[t] -= acc;
  }
  __syncthreads();
  for (int t = w - 1; t > 0; --t) {
    const double xt = v[t];
    for (int i = tid; i < t; i += NT) v[i] -= L[t + (int64_t)i * r] * xt;
    __syncthreads();
  }
  for (int t = tid; t < w; t += NT) {
    xi[f0 + t] = v[t];
    out[T.perm[f0 + t]] = v[t];
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
    std::vector<int64_t> cnt(big.size());
    int maxsteps = 0;
    for (size_t q = 0; q < big.size(); ++q) {
      const int s = big[q];
      cnt[q] = cdiv(S.nrows[s], 64);
      maxsteps = std::max<int>(maxsteps, (int)cdiv(S.first[s + 1] - S.first[s], 64));
    }
    add_big(BIG_ASM, 0, big, cnt);
    for (int p = 0; p < maxsteps; ++p) {
      std::vector<int64_t> cp(big.size(), 0), cu(big.size(), 0);
      for (size_t q = 0; q < big.size(); ++q) {
        const int s = big[q];
        const int w = S.first[s + 1] - S.first[s], r = S.nrows[s];
        if (cdiv(w, 64) <= p) continue;
        const int k0 = p * 64, kw = std::min(64, w - k0);
        const int64_t below = r - k0 - kw;
        cp[q] = std::max<int64_t>(1, cdiv(below, NT));
        const int64_t nt = cdiv(below, 64);
        cu[q] = nt * (nt + 1) / 2;
      }
      add_big(BIG_PANEL, p, big, cp);
      add_big(BIG_UPDATE, p, big, cu);
    }
  }
  for (int lev = 0; lev < S.nlevels; ++lev) {
    solve_.push_back({(int64_t)sched.size(), S.level_ptr[lev + 1] - S.level_ptr[lev]});
    for (int q = S.level_ptr[lev]; q < S.level_ptr[lev + 1]; ++q) sched.push_back(S.level_list[q]);
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
      case BIG_ASM:
        k_big_assemble<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, Kx, arena_);
        break;
      case BIG_PANEL:
        k_big_panel<<<(unsigned)L.items, NT, 0, s>>>(T_, list, L.nf, L.step, arena_, D_, status_, pivot_tol);
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
  for (const SolveLaunch& L : solve_)
    k_fwd<<<L.nf, NT, 0, s>>>(T_, sched_.p + L.off, arena_, b, xi_, uvec_, vwork_);
  for (auto it = solve_.rbegin(); it != solve_.rend(); ++it)
    k_bwd<<<it->nf, NT, 0, s>>>(T_, sched_.p + it->off, arena_, D_, xi_, b, vwork_);
  MADIPM_HIP(hipGetLastError());
}

}  // namespace madipm
