// Microbenchmark (diagnostics): how fast does ONE workgroup (256 threads, the shape of the tree /
// reduction kernels) read a buffer that the previous kernel wrote?  Variants: 8-byte vs 16-byte loads,
// 16 loads in flight per thread, plain vs sc1 (agent-scope) loads, first vs second pass (warm L2/TLB).
// build: hipcc --offload-arch=gfx950 -O3 -o ld_bench ld_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fill(double* p, long n, double v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v + i;
}

template <int MODE>  // 0: 8 B plain, 1: 8 B sc1, 2: 16 B plain
__global__ __launch_bounds__(256) void k_read(const double* p, int nbytes, double* out, long long* tm, int pass) {
  const int tid = threadIdx.x;
  double acc = 0.0;
  __syncthreads();
  const long long c0 = wall_clock64();
  if (MODE == 2) {
    const double2* q = reinterpret_cast<const double2*>(p);
    const int n = nbytes / 16;
    for (int base = 0; base < n; base += 256 * 16) {
      double2 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int e = base + k * 256 + tid;
        v[k] = (e < n) ? q[e] : double2{0.0, 0.0};
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += v[k].x + v[k].y;
    }
  } else {
    const int n = nbytes / 8;
    for (int base = 0; base < n; base += 256 * 16) {
      double v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int e = base + k * 256 + tid;
        if (MODE == 1)
          v[k] = (e < n) ? __hip_atomic_load(p + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        else
          v[k] = (e < n) ? p[e] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += v[k];
    }
  }
  __syncthreads();
  const long long c1 = wall_clock64();
  out[tid] = acc;
  if (tid == 0) tm[pass] = c1 - c0;
}

int main() {
  const long n = 64L << 20;  // 512 MB buffer; each test reads a fresh region
  double *p, *o;
  long long* tm;
  (void)hipMalloc(&p, n * 8);
  (void)hipMalloc(&o, 256 * 8);
  (void)hipMalloc(&tm, 64);
  const int sizes[] = {4096, 32768, 65536, 262144};
  long off = 0;
  for (int mode = 0; mode < 3; ++mode)
    for (int sz : sizes) {
      k_fill<<<1024, 256>>>(p + off, sz / 8, 1.0);
      for (int pass = 0; pass < 2; ++pass) {
        if (mode == 0) k_read<0><<<1, 256>>>(p + off, sz, o, tm, pass);
        if (mode == 1) k_read<1><<<1, 256>>>(p + off, sz, o, tm, pass);
        if (mode == 2) k_read<2><<<1, 256>>>(p + off, sz, o, tm, pass);
      }
      long long h[2];
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h, tm, 16, hipMemcpyDeviceToHost);
      printf("%s %7d B: first %.2f us (%.1f GB/s)  second %.2f us (%.1f GB/s)\n",
             mode == 0 ? "8B plain" : (mode == 1 ? "8B sc1  " : "16B plain"), sz, h[0] * 0.01, sz / (h[0] * 10.0),
             h[1] * 0.01, sz / (h[1] * 10.0));
      off += (sz / 8 + (1 << 18)) & ~((1L << 18) - 1);  // next test on fresh 2 MB-aligned region
    }
  return 0;
}
