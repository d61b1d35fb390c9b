// Microbenchmark (diagnostics): latency / throughput of single-wave primitives on gfx950 (clock64).
// build: hipcc --offload-arch=gfx950 -O3 -o prim_bench prim_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));
__global__ void k_prim(double* out, long long* tm, int n, int nw) {
  __shared__ double S[4096];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int q = threadIdx.x; q < 4096; q += blockDim.x) S[q] = 1.0 + q * 1e-6;
  __syncthreads();
  if (wv >= nw) return;
  double a = 1.0 + lane * 1e-3, b = 0.5;
  dbl4 acc = {0, 0, 0, 0}, acc2 = acc, acc3 = acc, acc4 = acc;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);  // dependent
  long long t1 = clock64();
  for (int i = 0; i < n; i += 4) {  // 4 independent chains
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
    acc4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc4, 0, 0, 0);
  }
  long long t2 = clock64();
  int idx = lane;
  double s = 0;
  for (int i = 0; i < n; ++i) {  // dependent LDS loads (pointer chase via value)
    const double v = S[idx];
    s += v;
    idx = (idx + 64 + (int)(v * 0.0)) & 4095;
  }
  long long t3 = clock64();
  double x = a;
  for (int i = 0; i < n; ++i) x = fma(x, 0.999, 1e-3);  // dependent fma
  long long t4 = clock64();
  double y = a;
  for (int i = 0; i < n; ++i) y = y / (1.0 + i * 1e-9);  // dependent division
  long long t5 = clock64();
  out[threadIdx.x] = acc[0] + acc2[1] + acc3[2] + acc4[3] + s + x + y;
  if (threadIdx.x == 0) { tm[0] = t1 - t0; tm[1] = t2 - t1; tm[2] = t3 - t2; tm[3] = t4 - t3; tm[4] = t5 - t4; }
}
int main() {
  double* o; long long* t; hipMalloc(&o, 1024 * 8); hipMalloc(&t, 64);
  for (int nw = 1; nw <= 4; nw *= 2) {
    for (int it = 0; it < 2; ++it) { k_prim<<<1, 256>>>(o, t, 256, nw); hipDeviceSynchronize(); }
    long long h[5]; hipMemcpy(h, t, 40, hipMemcpyDeviceToHost);
    printf("waves %d: per op cycles: mfma_f64 dep %.1f  mfma_f64 indep %.1f  lds dep %.1f  fma dep %.1f  div dep %.1f\n", nw,
           h[0] / 256.0, h[1] / 256.0, h[2] / 256.0, h[3] / 256.0, h[4] / 256.0);
  }
  return 0;
}
