// Microbenchmark (diagnostics): one workgroup, one wave substituting a w x w unit-lower panel staged
// in LDS, timed twice in a row (cold vs warm instruction cache) with s_memtime and wall_clock64.
// build: hipcc --offload-arch=gfx950 -O3 -o subst_bench subst_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

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
    if (k < kb) {
      xs[k] = readlane_f64(v[HB], (t0 & 63) + k);
      v[HB] = fma(-lb[HB][k], xs[k], v[HB]);
    }
  }
#pragma unroll
  for (int h = HB + 1; h < 3; ++h)
#pragma unroll
    for (int k = 0; k < 16; ++k) v[h] = fma(-lb[h][k], xs[k], v[h]);
}
__device__ void fwd_subst16(double (&v)[3], const double* Ls, int rl, int r, int w, int lane) {
  for (int t0 = 0; t0 < w; t0 += 16) {
    const int kb = min(16, w - t0);
    if (t0 < 64) fwd_block16<0>(v, Ls, rl, r, t0, kb, lane);
    else if (t0 < 128) fwd_block16<1>(v, Ls, rl, r, t0, kb, lane);
    else fwd_block16<2>(v, Ls, rl, r, t0, kb, lane);
  }
}
// variant 6: blocked substitution with unconditional (clamped) LDS loads and select masks
template <int HB>
__device__ __forceinline__ void fwd_block16u(double (&v)[3], const double* Ls, int rl, int r, int w, int t0, int kb, int lane) {
  double lb[3][16];
#pragma unroll
  for (int h = HB; h < 3; ++h) {
    const int i = lane + 64 * h;
    const int ic = min(i, r - 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double l = Ls[ic + min(t0 + k, w - 1) * rl];
      lb[h][k] = (k < kb && i > t0 + k && i < r) ? l : 0.0;
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double xt = readlane_f64(v[HB], (t0 & 63) + k);
    v[HB] = fma(-lb[HB][k], xt, v[HB]);
#pragma unroll
    for (int h = HB + 1; h < 3; ++h) v[h] = fma(-lb[h][k], xt, v[h]);
  }
}
__device__ void fwd_subst16u(double (&v)[3], const double* Ls, int rl, int r, int w, int lane) {
  for (int t0 = 0; t0 < w; t0 += 16) {
    const int kb = min(16, w - t0);
    if (t0 < 64) fwd_block16u<0>(v, Ls, rl, r, w, t0, kb, lane);
    else if (t0 < 128) fwd_block16u<1>(v, Ls, rl, r, w, t0, kb, lane);
    else fwd_block16u<2>(v, Ls, rl, r, w, t0, kb, lane);
  }
}
// variant 7: as 6 but the chain only on v[HB]; other thirds after the block with 4 accumulators
template <int HB>
__device__ __forceinline__ void fwd_block16v(double (&v)[3], const double* Ls, int rl, int r, int w, int t0, int kb, int lane) {
  double lb[3][16], xs[16];
#pragma unroll
  for (int h = HB; h < 3; ++h) {
    const int i = lane + 64 * h;
    const int ic = min(i, r - 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double l = Ls[ic + min(t0 + k, w - 1) * rl];
      lb[h][k] = (k < kb && i > t0 + k && i < r) ? l : 0.0;
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    xs[k] = readlane_f64(v[HB], (t0 & 63) + k);
    v[HB] = fma(-lb[HB][k], xs[k], v[HB]);
  }
#pragma unroll
  for (int h = HB + 1; h < 3; ++h) {
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int k = 0; k < 16; k += 4) {
      c0 = fma(lb[h][k], xs[k], c0); c1 = fma(lb[h][k + 1], xs[k + 1], c1);
      c2 = fma(lb[h][k + 2], xs[k + 2], c2); c3 = fma(lb[h][k + 3], xs[k + 3], c3);
    }
    v[h] -= (c0 + c1) + (c2 + c3);
  }
}
__device__ void fwd_subst16v(double (&v)[3], const double* Ls, int rl, int r, int w, int lane) {
  for (int t0 = 0; t0 < w; t0 += 16) {
    const int kb = min(16, w - t0);
    if (t0 < 64) fwd_block16v<0>(v, Ls, rl, r, w, t0, kb, lane);
    else if (t0 < 128) fwd_block16v<1>(v, Ls, rl, r, w, t0, kb, lane);
    else fwd_block16v<2>(v, Ls, rl, r, w, t0, kb, lane);
  }
}
// variant B: full-width blocks without the kb guard (padded panel: columns >= w hold 0), rolled k loop
__device__ void fwd_rolled(double (&v)[3], const double* Ls, int rl, int r, int w, int lane) {
  for (int t = 0; t < w; ++t) {
    const double xt = (t < 64) ? readlane_f64(v[0], t) : (t < 128 ? readlane_f64(v[1], t - 64) : readlane_f64(v[2], t - 128));
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      const int i = min(lane + 64 * h, r - 1);
      const double l = Ls[i + t * rl];
      v[h] = fma(lane + 64 * h > t ? -l : 0.0, xt, v[h]);
    }
  }
}

// variant 2: readlane + fma chain only (registers); 3: dependent fma chain only; 4: readlane of an int chain
__device__ void chain_rl_fma(double (&v)[3], int w, int lane) {
  for (int t = 0; t < w; ++t) {
    const double xt = readlane_f64(v[0], t & 63);
    v[0] = fma(-0.001 * lane, xt, v[0]);
  }
}
__device__ void chain_fma(double (&v)[3], int w, int lane) {
  for (int t = 0; t < w; ++t) v[0] = fma(v[0], 0.999, 0.001 * lane);
}
__device__ void chain_rl_int(double (&v)[3], int w, int lane) {
  int x = lane;
  for (int t = 0; t < w; ++t) x = __builtin_amdgcn_readlane(x, t & 63) + lane;
  v[0] += x;
}
// variant 5: DPP-free broadcast through LDS (ds_write by lane t, ds_read by all)
__device__ void chain_lds(double (&v)[3], double* bc, int w, int lane) {
  for (int t = 0; t < w; ++t) {
    if (lane == (t & 63)) bc[0] = v[0];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const double xt = bc[0];
    v[0] = fma(-0.001 * lane, xt, v[0]);
  }
}

__global__ __launch_bounds__(256) void k_bench(const double* L, int r, int w, int variant, double* out, long long* tm) {
  extern __shared__ double Ls[];
  const int rl = r | 1;
  for (int q = threadIdx.x; q < r * w; q += 256) {
    const int j = q / r, i = q - j * r;
    Ls[i + j * rl] = L[q];
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  double v[3];
  for (int rep = 0; rep < 3; ++rep) {
    for (int h = 0; h < 3; ++h) v[h] = (lane + 64 * h < r) ? 1.0 : 0.0;
    const long long c0 = clock64(), w0 = wall_clock64();
    if (variant == 0) fwd_subst16(v, Ls, rl, r, w, lane);
    else if (variant == 1) fwd_rolled(v, Ls, rl, r, w, lane);
    else if (variant == 2) chain_rl_fma(v, w, lane);
    else if (variant == 3) chain_fma(v, w, lane);
    else if (variant == 4) chain_rl_int(v, w, lane);
    else if (variant == 5) chain_lds(v, Ls + 150 * 100, w, lane);
    else if (variant == 6) fwd_subst16u(v, Ls, rl, r, w, lane);
    else fwd_subst16v(v, Ls, rl, r, w, lane);
    __builtin_amdgcn_s_waitcnt(0);
    const long long c1 = clock64(), w1 = wall_clock64();
    if (lane == 0) { tm[2 * rep] = c1 - c0; tm[2 * rep + 1] = w1 - w0; }
  }
  for (int h = 0; h < 3; ++h) if (lane + 64 * h < r) out[lane + 64 * h] = v[h];
}

int main() {
  const int r = 147, w = 65;
  std::vector<double> L(r * w);
  for (int j = 0; j < w; ++j) for (int i = 0; i < r; ++i) L[i + j * r] = (i > j) ? 0.01 * ((i * 7 + j * 3) % 13 - 6) : 0.0;
  double *dL, *dout; long long* dt;
  hipMalloc(&dL, L.size() * 8); hipMalloc(&dout, 256 * 8); hipMalloc(&dt, 64 * 8);
  hipMemcpy(dL, L.data(), L.size() * 8, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)k_bench, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  for (int variant = 0; variant < 8; ++variant) {
    for (int it = 0; it < 2; ++it) {
      k_bench<<<1, 256, 150 * 1024>>>(dL, r, w, variant, dout, dt);
      hipDeviceSynchronize();
      long long h[6];
      hipMemcpy(h, dt, sizeof(h), hipMemcpyDeviceToHost);
      std::vector<double> o(r);
      hipMemcpy(o.data(), dout, r * 8, hipMemcpyDeviceToHost);
      printf("variant %d launch %d: rep0 %lld cyc %.2f us | rep1 %lld cyc %.2f us | rep2 %lld cyc %.2f us  (chk %.6f)\n", variant, it,
             h[0], h[1] * 0.01, h[2], h[3] * 0.01, h[4], h[5] * 0.01, o[r - 1]);
    }
  }
  return 0;
}
