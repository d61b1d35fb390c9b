// Measures the sustained rate of v_mfma_f64_16x16x4f64 on the whole chip (peak for bench.py's
// roofline): every wave issues independent MFMA chains back to back from registers.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
  dbl4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  const double s = (c0[0] + c1[1]) + (c2[2] + c3[3]);
  if (s == 12345.678) out[threadIdx.x] = s;
}

int main() {
  double* out;
  hipMalloc(&out, 256 * sizeof(double));
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 20000;
  for (int wpc = 1; wpc <= 4; wpc *= 2) {  // workgroups (of 4 waves) per CU
    const int grid = ncu * wpc;
    hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, out, 100);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 16 * 16 * 4 * 4.0 * iters * 4.0 * grid;  // per MFMA 2*16*16*4, 4 chains, 4 waves
    printf("CUs %d, %d WG/CU: %.2f TFLOP/s f64 MFMA (16x16x4)\n", ncu, wpc, flops / (ms * 1e-3) / 1e12);
  }
  return 0;
}
