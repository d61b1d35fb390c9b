// Microbenchmark (diagnostics): one workgroup running the trailing-update tile loop of the in-LDS
// blocked LDL^T (square storage), with / without LDS loads and stores, timed with clock64.
// build: hipcc --offload-arch=gfx950 -O3 -o tile_bench tile_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));
#define PIN(x) asm volatile("" : "+v"(x))
template <int MODE>
__global__ __launch_bounds__(256) void k_tile(double* out, long long* tm, int r, int R0, int k0, int kw) {
  extern __shared__ double A[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ld = r | 1;
  for (int q = tid; q < r * ld; q += 256) A[q] = 1.0 + 1e-6 * q;
  __syncthreads();
  const int kl = lane >> 4;
  const int nbr = (r - R0 + 15) >> 4;
  const int ntile = nbr * (nbr + 1) / 2;
  double dk[4] = {1.0, 1.0, 1.0, 1.0};
  long long c0 = clock64();
  int I = 0, J = 0;
  for (int s0 = 0; s0 < wv; ++s0) {
    if (J == I) {
      ++I;
      J = 0;
    } else {
      ++J;
    }
  }
  double sink = 0;
  for (int q = wv; q < ntile; q += 4) {
    const int i0 = R0 + 16 * I, j0 = R0 + 16 * J;
    const int rj = min(j0 + (lane & 15), r - 1), ri = min(i0 + (lane & 15), r - 1);
    double av[4], bv[4], cv[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kc = k0 + min(4 * ks + kl, kw - 1);
      if (MODE & 1) {
        av[ks] = rj + kc;
        bv[ks] = ri - kc;
      } else {
        av[ks] = A[rj + kc * ld];
        bv[ks] = A[ri + kc * ld];
        PIN(av[ks]);
        PIN(bv[ks]);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = min(j0 + kl + 4 * g, r - 1);
      if (MODE & 1) {
        cv[g] = j;
      } else {
        cv[g] = A[max(ri, j) + min(ri, j) * ld];
        PIN(cv[g]);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) bv[ks] *= dk[ks];
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = j0 + kl + 4 * g, i = i0 + (lane & 15);
      if (MODE & 2)
        sink += cv[g] - acc[g];
      else if (i < r && j < r && i >= j)
        A[i + j * ld] = cv[g] - acc[g];
    }
    for (int s0 = 0; s0 < 4; ++s0) {
      if (J == I) {
        ++I;
        J = 0;
      } else {
        ++J;
      }
    }
  }
  __syncthreads();
  long long c1 = clock64();
  if (tid == 0) tm[MODE] = c1 - c0;
  out[tid] = sink + A[tid];
}

int main() {
  double* o;
  long long* t;
  (void)hipMalloc(&o, 256 * 8);
  (void)hipMalloc(&t, 64);
  const int r = 119, R0 = 16;
  (void)hipFuncSetAttribute((const void*)k_tile<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)k_tile<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)k_tile<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)k_tile<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int it = 0; it < 2; ++it) {
    k_tile<0><<<1, 256, r * (r | 1) * 8>>>(o, t, r, R0, 0, 16);
    k_tile<1><<<1, 256, r * (r | 1) * 8>>>(o, t, r, R0, 0, 16);
    k_tile<2><<<1, 256, r * (r | 1) * 8>>>(o, t, r, R0, 0, 16);
    k_tile<3><<<1, 256, r * (r | 1) * 8>>>(o, t, r, R0, 0, 16);
    (void)hipDeviceSynchronize();
  }
  long long h[4];
  (void)hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
  const int nbr = (r - R0 + 15) / 16;
  printf("tiles %d: mode0 (lds ld+st) %lld  mode1 (no ld) %lld  mode2 (no st) %lld  mode3 (mfma only) %lld cycles\n",
         nbr * (nbr + 1) / 2, h[0], h[1], h[2], h[3]);
  return 0;
}
