// Calibration (diagnostics): what rocprofv3's FETCH_SIZE reports on gfx950 for reads of a known byte
// count at several access widths, so the per-kernel PMC traffic (tools/pmc_traffic.py) is corrected
// only where the correction holds.  Each kernel reads every byte of a 256 MiB buffer exactly once:
//   k_w16  16 B / lane coalesced (double2)       k_w8  8 B / lane coalesced (double)
//   k_w4   4 B / lane coalesced (float)          k_g8  8 B / lane gather (a random permutation of
//                                                      the doubles, as the solves' and assembly's reads)
// build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
// run:   rocprofv3 --pmc FETCH_SIZE -d OUT -o calib --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

constexpr int64_t NB = 256ll << 20;  // bytes
constexpr int64_t ND = NB / 8;

__global__ __launch_bounds__(256) void k_w16(const double2* a, double* out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < ND / 2; i += (int64_t)gridDim.x * 256) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
__global__ __launch_bounds__(256) void k_w8(const double* a, double* out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < ND; i += (int64_t)gridDim.x * 256) s += a[i];
  if (s == 12345.678) out[0] = s;
}
__global__ __launch_bounds__(256) void k_w4(const float* a, double* out) {
  float s = 0.0f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < 2 * ND; i += (int64_t)gridDim.x * 256) s += a[i];
  if (s == 12345.678f) out[0] = s;
}
// the index stream (4 B per double read) is part of the fetched bytes: expected NB + NB / 2
__global__ __launch_bounds__(256) void k_g8(const double* a, const int32_t* idx, double* out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < ND; i += (int64_t)gridDim.x * 256) s += a[idx[i]];
  if (s == 12345.678) out[0] = s;
}

int main() {
  double *a, *out;
  int32_t* idx;
  hipMalloc(&a, NB);
  hipMalloc(&out, 64);
  hipMalloc(&idx, ND * 4);
  hipMemset(a, 0, NB);
  std::vector<int32_t> h(ND);
  for (int64_t i = 0; i < ND; ++i) h[i] = (int32_t)i;
  std::shuffle(h.begin(), h.end(), std::mt19937(7));
  hipMemcpy(idx, h.data(), ND * 4, hipMemcpyHostToDevice);
  const int G = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    k_w16<<<G, 256>>>(reinterpret_cast<const double2*>(a), out);
    k_w8<<<G, 256>>>(a, out);
    k_w4<<<G, 256>>>(reinterpret_cast<const float*>(a), out);
    k_g8<<<G, 256>>>(a, idx, out);
  }
  hipDeviceSynchronize();
  std::printf("read %lld bytes per kernel (k_g8: + %lld index bytes)\n", (long long)NB, (long long)(ND * 4));
  return 0;
}
