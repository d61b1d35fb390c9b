// Microbenchmark (diagnostics): the cost of the MPC loop's one-block reduction finaliser (k_final)
// after a 2048-block producer, against an empty kernel in the same place, for several finaliser
// shapes.  Times are per (producer; consumer) pair minus the producer alone, from hipEvents over
// many back-to-back pairs.  build: hipcc --offload-arch=gfx950 -O3 -o final_bench final_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int MAXB = 2048, NV = 3;

__global__ __launch_bounds__(256) void k_prod(double* part, int nb) {
  // block partials of NV values, value-major, written by thread 0..NV-1 (as block_partials)
  __shared__ double sh[NV];
  if (threadIdx.x < NV) sh[threadIdx.x] = blockIdx.x * 1e-3 + threadIdx.x;
  __syncthreads();
  if (threadIdx.x < NV) part[threadIdx.x * MAXB + blockIdx.x] = sh[threadIdx.x];
}

// the same partials after streaming `nbig` doubles of writes (a producer with a large dirty footprint,
// like the MPC's residual / right-hand-side kernels)
__global__ __launch_bounds__(256) void k_prod_big(double* part, int nb, double* big, int64_t nbig) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nbig; i += (int64_t)gridDim.x * 256) big[i] = (double)i;
  __shared__ double sh[NV];
  if (threadIdx.x < NV) sh[threadIdx.x] = blockIdx.x * 1e-3 + threadIdx.x;
  __syncthreads();
  if (threadIdx.x < NV) part[threadIdx.x * MAXB + blockIdx.x] = sh[threadIdx.x];
}

__global__ void k_empty(double* out) {
  if (threadIdx.x == 0 && out[0] == 12345.0) out[1] = 1.0;
}

template <int NTF>
__global__ __launch_bounds__(NTF) void k_fin(const double* part, int nb, double* out) {
  constexpr int PER = MAXB / NTF;  // blocks per thread
  __shared__ double sh[NV][NTF / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double v[NV][PER];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < PER; j += 2) {
      const int b = PER * threadIdx.x + j;
      const double2 q = (b < nb) ? *reinterpret_cast<const double2*>(part + k * MAXB + b) : double2{0.0, 0.0};
      v[k][j] = q.x;
      v[k][j + 1] = q.y;
    }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < PER; ++j) a = fmax(a, v[k][j]);
    for (int o = 32; o > 0; o >>= 1) a = fmax(a, __shfl_down(a, o, 64));
    if (lane == 0) sh[k][wv] = a;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double a = sh[threadIdx.x][0];
    for (int w = 1; w < NTF / 64; ++w) a = fmax(a, sh[threadIdx.x][w]);
    out[threadIdx.x] = a;
  }
}

int main() {
  double *part, *out;
  hipMalloc(&part, sizeof(double) * 16 * MAXB);
  hipMalloc(&out, sizeof(double) * 16);
  hipMemset(part, 0, sizeof(double) * 16 * MAXB);
  hipMemset(out, 0, sizeof(double) * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int nb = 1929, R = 400;
  double* big;
  const int64_t NBIG = 8ll << 20;  // 64 MiB
  hipMalloc(&big, NBIG * 8);
  int64_t nbig = 0;
  auto prod = [&]() {
    if (nbig)
      k_prod_big<<<nb, 256>>>(part, nb, big, nbig);
    else
      k_prod<<<nb, 256>>>(part, nb);
  };
  auto run = [&](int which) {
    for (int it = 0; it < 20; ++it) prod();
    hipEventRecord(e0);
    for (int it = 0; it < R; ++it) {
      prod();
      if (which == 1) k_empty<<<1, 64>>>(out);
      if (which == 2) k_fin<1024><<<1, 1024>>>(part, nb, out);
      if (which == 3) k_fin<256><<<1, 256>>>(part, nb, out);
      if (which == 4) k_fin<512><<<1, 512>>>(part, nb, out);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return 1e3 * ms / R;
  };
  const char* nm[] = {"", "empty kernel", "k_fin 1024 thr", "k_fin 256 thr", "k_fin 512 thr"};
  for (int64_t nbg : {0ll, 1ll << 20, 4ll << 20, 8ll << 20}) {
    nbig = nbg;
    const double base = run(0);
    std::printf("producer (+ %3lld MiB written) alone %7.2f us\n", (long long)(nbg * 8 >> 20), base);
    for (int w = 1; w <= 4; ++w) std::printf("  + %-20s %7.2f us\n", nm[w], run(w) - base);
  }
  return 0;
}
