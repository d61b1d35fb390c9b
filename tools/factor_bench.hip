// Microbenchmark (diagnostics): one workgroup factorising an r x r front in LDS with the library's
// blocked LDL^T (copied from csrc/ldl.hip with clock64 phase accumulators).
// build: hipcc --offload-arch=gfx950 -O3 -o factor_bench factor_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
constexpr int NT = 256;
constexpr int LDM = 17;
typedef double dbl4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
template <bool PK>
__device__ __forceinline__ int fidx(int i, int j, int r, int ld) {
  return PK ? ((j * (2 * r - j - 1)) >> 1) + i : i + j * ld;
}

template <bool PK>
__device__ __forceinline__ void factor16g(double* A, int r, int ld, int k0, int kw, double* Dl, double* MK, double* cb,
                                          double* xb, int lane) {
  const int il = lane & 15, cg = lane >> 4;
  double a[4], x[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int jl = cg + 4 * m;
    a[m] = (il < kw && jl < kw) ? (jl <= il ? A[fidx<PK>(k0 + il, k0 + jl, r, ld)] : 0.0) : (il == jl ? 1.0 : 0.0);
    x[m] = (jl == il) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (cg == (t & 3)) cb[t * LDM + il] = a[t >> 2];
    if (il == t) {
#pragma unroll
      for (int m = 0; m < 4; ++m) xb[t * LDM + cg + 4 * m] = x[m];
    }
    wave_sync();
    const double dt = cb[t * LDM + t];
    const double li = (il > t) ? cb[t * LDM + il] / dt : 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int jl = cg + 4 * m;
      const double cj = cb[t * LDM + jl];
      const double xt = xb[t * LDM + jl];
      a[m] = fma(jl > t ? -li : 0.0, cj, a[m]);
      x[m] = fma(jl > t ? 0.0 : -li, xt, x[m]);
    }
  }
  wave_sync();
  const double di = cb[il * LDM + il];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int jl = cg + 4 * m;
    if (jl < il && il < kw) A[fidx<PK>(k0 + il, k0 + jl, r, ld)] = a[m] / cb[jl * LDM + jl];
    MK[jl * LDM + il] = (jl <= il) ? x[m] / di : 0.0;
  }
  if (cg == 0 && il < kw) Dl[k0 + il] = di;
  wave_sync();
}

template <bool PK>
__device__ __forceinline__ void blocked_factor_lds(double* A, int r, int w, int ld, double* Dl, double* MK, double* cbuf, long long* tacc) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int k0 = 0; k0 < w; k0 += 16) {
    const int kw = min(16, w - k0);
    const int R0 = k0 + kw;                       // first row / column after the pivots
    const int nbr = (r - R0 + 15) >> 4;           // 16-row blocks below
    long long c0 = clock64();
    if (wv == ((k0 >> 4) & 3)) factor16g<PK>(A, r, ld, k0, kw, Dl, MK, cbuf, cbuf + 16 * LDM, lane);
    __syncthreads();
    long long c1 = clock64(); if (tid == 0) tacc[0] += c1 - c0;
    // panel: L_R = A[R, k0:k0+kw] M_K, row block per wave
    for (int b = wv; b < nbr; b += 4) {
      const int rb = R0 + 16 * b;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + (lane >> 4), row = rb + (lane & 15);
        const double av = (k < kw && row < r) ? A[fidx<PK>(row, k0 + k, r, ld)] : 0.0;
        const double bv = MK[k * LDM + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
      // acc[g]: row rb + (lane>>4) + 4g ... D[m][n] with m = (lane>>4)+4g, n = lane&15: here the A
      // operand carried the rows (m) and M_K the columns (n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = rb + (lane >> 4) + 4 * g, col = lane & 15;
        if (row < r && col < kw) A[fidx<PK>(row, k0 + col, r, ld)] = acc[g];
      }
    }
    __syncthreads();
    long long c2 = clock64(); if (tid == 0) tacc[1] += c2 - c1;
    // trailing update of the lower triangle of A[R0:, R0:]: tile (I, J), J <= I
    const int ntile = nbr * (nbr + 1) / 2;
    for (int q = wv; q < ntile; q += 4) {
      int I = 0, rem = q;
      while (rem > I) {
        rem -= I + 1;
        ++I;
      }
      const int J = rem;
      const int i0 = R0 + 16 * I, j0 = R0 + 16 * J;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + (lane >> 4);
        const int rj = j0 + (lane & 15), ri = i0 + (lane & 15);
        const double av = (k < kw && rj < r) ? A[fidx<PK>(rj, k0 + k, r, ld)] : 0.0;       // L_J (rows m)
        const double bv = (k < kw && ri < r) ? A[fidx<PK>(ri, k0 + k, r, ld)] * Dl[k0 + k] : 0.0;  // (L_I D) (cols n)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + (lane >> 4) + 4 * g, i = i0 + (lane & 15);
        if (i < r && j < r && i >= j) A[fidx<PK>(i, j, r, ld)] -= acc[g];
      }
    }
    __syncthreads();
    if (tid == 0) tacc[2] += clock64() - c2;
  }
}



// ---------------- optimised variants (unconditional clamped LDS loads, reciprocal pivots)
__device__ __forceinline__ double rcp_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  return r;
}
template <bool PK>
__device__ __forceinline__ void factor16v(double* A, int r, int ld, int k0, int kw, double* Dl, double* MK, double* cb,
                                          double* xb, int lane) {
  const int il = lane & 15, cg = lane >> 4;
  const int ilc = min(il, kw - 1);
  double a[4], x[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int jl = cg + 4 * m;
    const double v = A[fidx<PK>(k0 + max(ilc, min(jl, kw - 1)), k0 + min(jl, ilc), r, ld)];
    a[m] = (il < kw && jl < kw) ? (jl <= il ? v : 0.0) : (il == jl ? 1.0 : 0.0);
    x[m] = (jl == il) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (cg == (t & 3)) cb[t * LDM + il] = a[t >> 2];
    if (il == t) {
#pragma unroll
      for (int m = 0; m < 4; ++m) xb[t * LDM + cg + 4 * m] = x[m];
    }
    wave_sync();
    const double dinv = rcp_f64(cb[t * LDM + t]);
    const double li = (il > t) ? cb[t * LDM + il] * dinv : 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int jl = cg + 4 * m;
      const double cj = cb[t * LDM + jl];
      const double xt = xb[t * LDM + jl];
      a[m] = fma(jl > t ? -li : 0.0, cj, a[m]);
      x[m] = fma(jl > t ? 0.0 : -li, xt, x[m]);
    }
  }
  wave_sync();
  const double di = cb[il * LDM + il];
  const double dii = rcp_f64(di);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int jl = cg + 4 * m;
    if (jl < il && il < kw) A[fidx<PK>(k0 + il, k0 + jl, r, ld)] = a[m] * rcp_f64(cb[jl * LDM + jl]);
    MK[jl * LDM + il] = (jl <= il) ? x[m] * dii : 0.0;
  }
  if (cg == 0 && il < kw) Dl[k0 + il] = di;
  wave_sync();
}

template <bool PK>
__device__ __forceinline__ void blocked_factor_v(double* A, int r, int w, int ld, double* Dl, double* MK, double* cbuf, long long* tacc) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int k0 = 0; k0 < w; k0 += 16) {
    const int kw = min(16, w - k0);
    const int R0 = k0 + kw;
    const int nbr = (r - R0 + 15) >> 4;
    long long c0 = clock64();
    if (wv == ((k0 >> 4) & 3)) factor16v<PK>(A, r, ld, k0, kw, Dl, MK, cbuf, cbuf + 16 * LDM, lane);
    __syncthreads();
    long long c1 = clock64(); if (tid == 0) tacc[0] += c1 - c0;
    const int kc = min(4 * 0 + (lane >> 4), 0);  (void)kc;
    for (int b = wv; b < nbr; b += 4) {
      const int rb = R0 + 16 * b;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
      double av[4], bv[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + (lane >> 4), row = rb + (lane & 15);
        const double v = A[fidx<PK>(min(row, r - 1), k0 + min(k, kw - 1), r, ld)];
        av[ks] = (k < kw && row < r) ? v : 0.0;
        bv[ks] = MK[k * LDM + (lane & 15)];
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = rb + (lane >> 4) + 4 * g, col = lane & 15;
        if (row < r && col < kw) A[fidx<PK>(row, k0 + col, r, ld)] = acc[g];
      }
    }
    __syncthreads();
    long long c2 = clock64(); if (tid == 0) tacc[1] += c2 - c1;
    const int ntile = nbr * (nbr + 1) / 2;
    double dk[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) dk[ks] = Dl[k0 + min(4 * ks + (lane >> 4), kw - 1)];
    for (int q = wv; q < ntile; q += 4) {
      int I = 0, rem = q;
      while (rem > I) { rem -= I + 1; ++I; }
      const int J = rem;
      const int i0 = R0 + 16 * I, j0 = R0 + 16 * J;
      const int rj = min(j0 + (lane & 15), r - 1), ri = min(i0 + (lane & 15), r - 1);
      double av[4], bv[4], cv[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + (lane >> 4);
        const int kc = k0 + min(k, kw - 1);
        const double va = A[fidx<PK>(rj, kc, r, ld)], vb = A[fidx<PK>(ri, kc, r, ld)];
        av[ks] = (k < kw) ? va : 0.0;
        bv[ks] = (k < kw) ? vb * dk[ks] : 0.0;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = min(j0 + (lane >> 4) + 4 * g, r - 1), i = ri;
        cv[g] = A[fidx<PK>(max(i, j), min(i, j), r, ld)];
      }
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + (lane >> 4) + 4 * g, i = i0 + (lane & 15);
        if (i < r && j < r && i >= j) A[fidx<PK>(i, j, r, ld)] = cv[g] - acc[g];
      }
    }
    __syncthreads();
    if (tid == 0) tacc[2] += clock64() - c2;
  }
}

// ---------------- variant 2: loads forced unconditional (asm pin), selects after, one wait per tile
#define PIN(x) asm volatile("" : "+v"(x))
template <bool PK>
__device__ __forceinline__ void factor16w(double* A, int r, int ld, int k0, int kw, double* Dl, double* MK, double* cb,
                                          double* xb, int lane) {
  const int il = lane & 15, cg = lane >> 4;
  const int ilc = min(il, kw - 1);
  double a[4], x[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int jl = cg + 4 * m;
    const int jc = min(jl, kw - 1);
    double v = A[fidx<PK>(k0 + max(ilc, jc), k0 + min(ilc, jc), r, ld)];
    PIN(v);
    a[m] = (il < kw && jl < kw) ? (jl <= il ? v : 0.0) : (il == jl ? 1.0 : 0.0);
    x[m] = (jl == il) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (cg == (t & 3)) cb[t * LDM + il] = a[t >> 2];
    if (il == t) {
#pragma unroll
      for (int m = 0; m < 4; ++m) xb[t * LDM + cg + 4 * m] = x[m];
    }
    wave_sync();
    double dt = cb[t * LDM + t], ci = cb[t * LDM + il];
    double cj[4], xt[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      cj[m] = cb[t * LDM + cg + 4 * m];
      xt[m] = xb[t * LDM + cg + 4 * m];
    }
    const double dinv = rcp_f64(dt);
    const double li = (il > t) ? ci * dinv : 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int jl = cg + 4 * m;
      a[m] = fma(jl > t ? -li : 0.0, cj[m], a[m]);
      x[m] = fma(jl > t ? 0.0 : -li, xt[m], x[m]);
    }
  }
  wave_sync();
  const double di = cb[il * LDM + il];
  double dj[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) dj[m] = cb[(cg + 4 * m) * LDM + (cg + 4 * m)];
  const double dii = rcp_f64(di);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int jl = cg + 4 * m;
    if (jl < il && il < kw) A[fidx<PK>(k0 + il, k0 + jl, r, ld)] = a[m] * rcp_f64(dj[m]);
    MK[jl * LDM + il] = (jl <= il) ? x[m] * dii : 0.0;
  }
  if (cg == 0 && il < kw) Dl[k0 + il] = di;
  wave_sync();
}

template <bool PK>
__device__ __forceinline__ void blocked_factor_w(double* A, int r, int w, int ld, double* Dl, double* MK, double* cbuf, long long* tacc) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int k0 = 0; k0 < w; k0 += 16) {
    const int kw = min(16, w - k0);
    const int R0 = k0 + kw;
    const int nbr = (r - R0 + 15) >> 4;
    long long c0 = clock64();
    if (wv == ((k0 >> 4) & 3)) factor16w<PK>(A, r, ld, k0, kw, Dl, MK, cbuf, cbuf + 16 * LDM, lane);
    __syncthreads();
    long long c1 = clock64(); if (tid == 0) tacc[0] += c1 - c0;
    const int kl = lane >> 4;
    for (int b = wv; b < nbr; b += 4) {
      const int rb = R0 + 16 * b;
      double av[4], bv[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + kl, row = rb + (lane & 15);
        av[ks] = A[fidx<PK>(min(row, r - 1), k0 + min(k, kw - 1), r, ld)];
        bv[ks] = MK[k * LDM + (lane & 15)];
        PIN(av[ks]);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) av[ks] = (4 * ks + kl < kw) ? av[ks] : 0.0;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = rb + kl + 4 * g, col = lane & 15;
        if (row < r && col < kw) A[fidx<PK>(row, k0 + col, r, ld)] = acc[g];
      }
    }
    __syncthreads();
    long long c2 = clock64(); if (tid == 0) tacc[1] += c2 - c1;
    const int ntile = nbr * (nbr + 1) / 2;
    double dk[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) dk[ks] = (4 * ks + kl < kw) ? Dl[k0 + min(4 * ks + kl, kw - 1)] : 0.0;
    int I = 0, J = 0, q = 0;
    // tile q -> (I, J), J <= I, advanced incrementally (wave-uniform)
    for (int s0 = 0; s0 < wv; ++s0) { if (J == I) { ++I; J = 0; } else ++J; }
    for (q = wv; q < ntile; q += 4) {
      const int i0 = R0 + 16 * I, j0 = R0 + 16 * J;
      const int rj = min(j0 + (lane & 15), r - 1), ri = min(i0 + (lane & 15), r - 1);
      double av[4], bv[4], cv[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kc = k0 + min(4 * ks + kl, kw - 1);
        av[ks] = A[fidx<PK>(rj, kc, r, ld)];
        bv[ks] = A[fidx<PK>(ri, kc, r, ld)];
        PIN(av[ks]);
        PIN(bv[ks]);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = min(j0 + kl + 4 * g, r - 1);
        cv[g] = A[fidx<PK>(max(ri, j), min(ri, j), r, ld)];
        PIN(cv[g]);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) bv[ks] *= dk[ks];
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + kl + 4 * g, i = i0 + (lane & 15);
        if (i < r && j < r && i >= j) A[fidx<PK>(i, j, r, ld)] = cv[g] - acc[g];
      }
      for (int s0 = 0; s0 < 4; ++s0) { if (J == I) { ++I; J = 0; } else ++J; }
    }
    __syncthreads();
    if (tid == 0) tacc[2] += clock64() - c2;
  }
}

template <bool PK>
__device__ __forceinline__ void blocked_factor_m(double* A, int r, int w, int ld, double* Dl, double* MK, double* cbuf, long long* tacc, int mode) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int k0 = 0; k0 < w; k0 += 16) {
    const int kw = min(16, w - k0);
    const int R0 = k0 + kw;
    const int nbr = (r - R0 + 15) >> 4;
    long long c0 = clock64();
    if (wv == ((k0 >> 4) & 3)) factor16w<PK>(A, r, ld, k0, kw, Dl, MK, cbuf, cbuf + 16 * LDM, lane);
    __syncthreads();
    long long c1 = clock64(); if (tid == 0) tacc[0] += c1 - c0;
    const int kl = lane >> 4;
    for (int b = wv; b < nbr; b += 4) {
      const int rb = R0 + 16 * b;
      double av[4], bv[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + kl, row = rb + (lane & 15);
        av[ks] = A[fidx<PK>(min(row, r - 1), k0 + min(k, kw - 1), r, ld)];
        bv[ks] = MK[k * LDM + (lane & 15)];
        PIN(av[ks]);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) av[ks] = (4 * ks + kl < kw) ? av[ks] : 0.0;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = rb + kl + 4 * g, col = lane & 15;
        if (row < r && col < kw) A[fidx<PK>(row, k0 + col, r, ld)] = acc[g];
      }
    }
    __syncthreads();
    long long c2 = clock64(); if (tid == 0) tacc[1] += c2 - c1;
    const int ntile = nbr * (nbr + 1) / 2;
    double dk[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) dk[ks] = (4 * ks + kl < kw) ? Dl[k0 + min(4 * ks + kl, kw - 1)] : 0.0;
    int I = 0, J = 0, q = 0;
    // tile q -> (I, J), J <= I, advanced incrementally (wave-uniform)
    for (int s0 = 0; s0 < wv; ++s0) { if (J == I) { ++I; J = 0; } else ++J; }
    for (q = wv; q < ntile; q += 4) {
      const int i0 = R0 + 16 * I, j0 = R0 + 16 * J;
      const int rj = min(j0 + (lane & 15), r - 1), ri = min(i0 + (lane & 15), r - 1);
      double av[4], bv[4], cv[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kc = k0 + min(4 * ks + kl, kw - 1);
        av[ks] = (mode & 1) ? (double)(rj + kc) : A[fidx<PK>(rj, kc, r, ld)];
        bv[ks] = (mode & 1) ? (double)(ri - kc) : A[fidx<PK>(ri, kc, r, ld)];
        PIN(av[ks]);
        PIN(bv[ks]);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = min(j0 + kl + 4 * g, r - 1);
        cv[g] = (mode & 1) ? 1.0 * j : A[fidx<PK>(max(ri, j), min(ri, j), r, ld)];
        PIN(cv[g]);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) bv[ks] *= dk[ks];
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + kl + 4 * g, i = i0 + (lane & 15);
        if (!(mode & 2) && i < r && j < r && i >= j) A[fidx<PK>(i, j, r, ld)] = cv[g] - acc[g];
        if ((mode & 2)) Dl[191] += cv[g] - acc[g];
      }
      for (int s0 = 0; s0 < 4; ++s0) { if (J == I) { ++I; J = 0; } else ++J; }
    }
    __syncthreads();
    if (tid == 0) tacc[2] += clock64() - c2;
  }
}

namespace nw {
// Same contract as factor16g, register-resident: lane i (& 15) keeps row i of the 16 x 16 diagonal
// block (and row i of X = L_KK^{-1}) in registers; pivot t and the column below it are broadcast
// with readlane (no LDS round trip in the pivot chain, the column reads overlap the reciprocal).
// Identity-padded past kw.  Writes the strictly-lower L_KK into A, d into Dl[k0 + i] and
// M_K = L_KK^{-T} D^{-1} (ld LDM, zero above the diagonal) into MK.
template <bool PK>
__device__ __forceinline__ void factor16r(double* A, int r, int ld, int k0, int kw, double* Dl, double* MK, int lane) {
  const int i = lane & 15;
  const int ic = min(i, kw - 1);
  double a[16], x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int jc = min(j, kw - 1);
    double v = A[fidx<PK>(k0 + max(ic, jc), k0 + min(ic, jc), r, ld)];  // upper part mirrored (never read)
    asm volatile("" : "+v"(v));  // keep the load unconditional (no per-load branch + wait)
    a[j] = (i < kw && j < kw) ? v : (i == j ? 1.0 : 0.0);
    x[j] = (i == j) ? 1.0 : 0.0;
  }
  double dmine = 1.0;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const double dt = readlane_f64(a[t], t);
    double col[16], xr[16];
#pragma unroll
    for (int j = t + 1; j < 16; ++j) col[j] = readlane_f64(a[t], j);  // L-part (j, t), unscaled
#pragma unroll
    for (int j = 0; j <= t; ++j) xr[j] = readlane_f64(x[j], t);       // row t of X
    const double li = (i > t) ? a[t] / dt : 0.0;  // IEEE quotient: keeps the level path's rounding
#pragma unroll
    for (int j = t + 1; j < 16; ++j) a[j] = fma(-li, col[j], a[j]);
#pragma unroll
    for (int j = 0; j <= t; ++j) x[j] = fma(-li, xr[j], x[j]);
    if (i == t) dmine = dt;
    if (i > t) a[t] = li;
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < i && i < kw) A[fidx<PK>(k0 + i, k0 + j, r, ld)] = a[j];
      MK[j * LDM + i] = (j <= i) ? x[j] / dmine : 0.0;
    }
    if (i < kw) Dl[k0 + i] = dmine;
  }
  wave_sync();
}

#define LDL_PIN(x) asm volatile("" : "+v"(x))

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
        LDL_PIN(av[u][ks]);
      }
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
                                            const double (&dk)[4], int lane) {
  const int kl = lane >> 4, il = lane & 15;
  const int i0 = R0 + 16 * I;
  const int ri = min(i0 + il, r - 1);
  double bv[4], av[NS][4], cv[NS][4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int kc = k0 + min(4 * ks + kl, kw - 1);
    bv[ks] = A[fidx<PK>(ri, kc, r, ld)];
    LDL_PIN(bv[ks]);
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int rj = min(R0 + 16 * (J0 + t) + il, r - 1);
      av[t][ks] = A[fidx<PK>(rj, kc, r, ld)];
      LDL_PIN(av[t][ks]);
    }
  }
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = min(R0 + 16 * (J0 + t) + kl + 4 * g, r - 1);
      cv[t][g] = A[fidx<PK>(max(ri, j), min(ri, j), r, ld)];
      LDL_PIN(cv[t][g]);
    }
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
      if (i < r && j < r && i >= j) A[fidx<PK>(i, j, r, ld)] = cv[t][g] - acc[t][g];
    }
}

// C_IJ -= L_J (L_I D)^T over the 16 x 16 tiles (I, J) of the trailing lower triangle with
// jlo <= J <= min(I, jhi), I < nbr; strips (I, J0 .. J0+3) dealt to waves w0, w0 + wstep, ...
template <bool PK>
__device__ __forceinline__ void trail_strips(double* A, int r, int ld, int k0, int kw, int R0, int nbr, int jlo, int jhi,
                                             const double (&dk)[4], int w0, int wstep, int lane) {
  int I = jlo, J0 = jlo;
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
      case 1: trail_strip<PK, 1>(A, r, ld, k0, kw, R0, I, J0, dk, lane); break;
      case 2: trail_strip<PK, 2>(A, r, ld, k0, kw, R0, I, J0, dk, lane); break;
      case 3: trail_strip<PK, 3>(A, r, ld, k0, kw, R0, I, J0, dk, lane); break;
      default: trail_strip<PK, 4>(A, r, ld, k0, kw, R0, I, J0, dk, lane); break;
    }
    for (int s = 0; s < wstep; ++s) adv();
  }
}

template <bool PK>
__device__ __forceinline__ void blocked_factor_lds(double* A, int r, int w, int ld, double* Dl, double* MK, double* cbuf, long long* tacc) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = (w + 15) >> 4;
  if (wv == 0) factor16r<PK>(A, r, ld, 0, min(16, w), Dl, MK, lane);
  __syncthreads();
  for (int kb = 0; kb < nblk; ++kb) {
    const int k0 = 16 * kb, kw = min(16, w - k0);
    const int R0 = k0 + kw;                       // first row / column after the pivots
    const int nbr = (r - R0 + 15) >> 4;           // 16-row blocks below
    long long c0 = clock64();
    panel_blocks<PK>(A, r, ld, k0, kw, R0, nbr, MK, wv, 4, lane);
    __syncthreads();
    long long c1 = clock64(); if (tid == 0) tacc[1] += c1 - c0;
    double dk[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = 4 * ks + (lane >> 4);
      dk[ks] = (k < kw) ? Dl[k0 + min(k, kw - 1)] : 0.0;
    }
    if (kb + 1 < nblk) {
      // the next pivot block's columns (J = 0: its diagonal block and panel rows) first ...
      trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 0, 0, dk, wv, 4, lane);
      __syncthreads();
      if (tid == 0) tacc[0] += clock64() - c1;
      // ... then one wave factorises it while the other three update the rest (J >= 1)
      const int fw = (kb + 1) & 3;
      if (wv == fw)
        factor16r<PK>(A, r, ld, R0, min(16, w - R0), Dl, MK, lane);
      else
        trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 1, nbr, dk, (wv - fw + 3) & 3, 3, lane);
    } else {
      trail_strips<PK>(A, r, ld, k0, kw, R0, nbr, 0, nbr, dk, wv, 4, lane);
    }
    __syncthreads();
    if (tid == 0) tacc[2] += clock64() - c1;
  }
}

}

template <bool PK>
__global__ __launch_bounds__(NT) void k_bench(const double* F, int r, int w, double* Dout, long long* tm, int variant) {
  extern __shared__ double A[];
  __shared__ double Dl[192];
  __shared__ double MK[16 * LDM];
  __shared__ double cbuf[2 * 16 * LDM];
  __shared__ long long tacc[4];
  const int ld = PK ? 0 : (r | 1);
  if (threadIdx.x < 4) tacc[threadIdx.x] = 0;
  for (int q = threadIdx.x; q < r * r; q += NT) {
    const int j = q / r, i = q - j * r;
    if (i >= j) A[fidx<PK>(i, j, r, ld)] = F[q];
  }
  __syncthreads();
  const long long c0 = clock64();
  if (variant == 0) blocked_factor_lds<PK>(A, r, w, ld, Dl, MK, cbuf, tacc); else if (variant == 1) blocked_factor_v<PK>(A, r, w, ld, Dl, MK, cbuf, tacc); else if (variant == 2) blocked_factor_w<PK>(A, r, w, ld, Dl, MK, cbuf, tacc); else if (variant == 6) nw::blocked_factor_lds<PK>(A, r, w, ld, Dl, MK, cbuf, tacc); else blocked_factor_m<PK>(A, r, w, ld, Dl, MK, cbuf, tacc, variant - 2);
  const long long c1 = clock64();
  if (threadIdx.x == 0) { tm[0] = c1 - c0; tm[1] = tacc[0]; tm[2] = tacc[1]; tm[3] = tacc[2]; }
  if (threadIdx.x < w) Dout[threadIdx.x] = Dl[threadIdx.x];
}

int main() {
  const int cases[][3] = {{143, 16, 1}, {147, 65, 1}, {119, 58, 0}, {120, 120, 0}, {82, 50, 0}};
  for (int variant : {0, 6})
  for (auto& c : cases) {
    const int r = c[0], w = c[1], pk = c[2];
    std::vector<double> F((size_t)r * r, 0.0);
    for (int j = 0; j < r; ++j) for (int i = j; i < r; ++i) F[i + (size_t)j * r] = (i == j) ? (j < w ? 4.0 + r : -(4.0 + r)) : 0.5 * (((i * 7 + j * 13) % 11) - 5) / 5.0;
    double *dF, *dD; long long* dt;
    hipMalloc(&dF, F.size() * 8); hipMalloc(&dD, 256 * 8); hipMalloc(&dt, 8 * 8);
    hipMemcpy(dF, F.data(), F.size() * 8, hipMemcpyHostToDevice);
    const int lds = pk ? r * (r + 1) / 2 * 8 : r * (r | 1) * 8;
    for (int it = 0; it < 3; ++it) {
      if (pk) { hipFuncSetAttribute((const void*)k_bench<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); k_bench<true><<<1, NT, lds>>>(dF, r, w, dD, dt, variant); }
      else { hipFuncSetAttribute((const void*)k_bench<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); k_bench<false><<<1, NT, lds>>>(dF, r, w, dD, dt, variant); }
      hipDeviceSynchronize();
    }
    long long h[4]; hipMemcpy(h, dt, sizeof(h), hipMemcpyDeviceToHost);
    std::vector<double> dd(w); hipMemcpy(dd.data(), dD, 8 * w, hipMemcpyDeviceToHost); double d0 = 0; for (double x : dd) d0 += x;
    printf("v%d r=%3d w=%3d %s: total %7lld cyc (%.2f us) | diag16 %lld  panel %lld  trailing %lld | blocks %d  d0 %.4f\n", variant, r, w, pk ? "packed" : "square",
           h[0], h[0] / 2400.0, h[1], h[2], h[3], (w + 15) / 16, d0);
    hipFree(dF); hipFree(dD); hipFree(dt);
  }
  return 0;
}
