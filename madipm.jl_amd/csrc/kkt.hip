// Array-type overrides of MadIPM's GPU extension, as C-ABI entry points (gfx950).
//
// The reference's CUDA extension (ext/MadIPMCUDAExt/cuda_wrapper.jl, MadIPMCUDAExt.jl) overrides a
// handful of array-type methods so that MPCSolver runs on CuArrays.  These are their MI355X
// counterparts, each taking device pointers and a HIP stream (declared in include/madipm_hip.h):
//
//   MadNLP.transfer!                cuda_wrapper.jl:4-24     -> madipm_transfer_*      (k_transfer)
//   compress_jacobian!              cuda_wrapper.jl:32-41    -> madipm_compress_jacobian (k_compress_jac)
//   MadIPMOperator + mul!           cuda_wrapper.jl:43-94    -> madipm_spmv_*          (k_spmv_rows, k_spmv_cols)
//   MadIPM.coo_to_csr               cuda_wrapper.jl:96-106, src/utils.jl:158-201 -> madipm_coo_to_csr
//   MadIPM.assemble_normal_system!  cuda_wrapper.jl:108-156, src/utils.jl:276-308 -> k_normal_merge
//   MadIPM.build_normal_system      cuda_wrapper.jl:158-234, src/utils.jl:209-274 -> host (as normalkkt.jl:104)
//   fill_structure!                 MadIPMCUDAExt.jl:15-32   -> madipm_csr_fill_structure
//   NLPModels.obj / grad!           MadIPMCUDAExt.jl:34-45   -> madipm_qp_obj / madipm_qp_grad
//
// Unlike the reference's kernels (an un-synchronised scatter in transfer!, cuSPARSE's unspecified
// SpMV order), every sum here has a fixed order: results are bitwise reproducible, and the
// scatter-adds / normal-equation products follow the reference CPU loops' order and association
// exactly (FMA contraction off where products are summed), so they equal the CPU methods bit for bit
// on finite inputs (assemble_normal_system!'s CPU loop also adds 0 * x for the columns two rows do not
// share, which the merge-join skips: with Inf / NaN values, or for the sign of a zero, they differ).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <memory>
#include <numeric>
#include <vector>

#include "../../include/madipm_hip.h"
#include "common.hpp"

namespace madipm {
namespace {

constexpr int NT = 256;

inline unsigned grid_for(int64_t n, int per_block = NT, unsigned cap = 65536) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cap, (n + per_block - 1) / per_block));
}

template <class T>
std::vector<T> to_host(const T* p, int64_t n, bool on_device) {
  std::vector<T> h(n);
  if (n == 0) return h;
  if (on_device)
    MADIPM_HIP(hipMemcpy(h.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
  else
    std::memcpy(h.data(), p, n * sizeof(T));
  return h;
}

// ------------------------------------------------------------------ transfer! (cuda_wrapper.jl:4-24)
// dest[e] = sum of src[k] over the k with map[k] == e, in ascending k (MadNLP's CPU transfer! loop:
// fill!(dest, 0); dest[map[k]] += src[k]).  One thread per destination entry; sources listed by
// destination (host counting sort of the map at plan creation).
__global__ __launch_bounds__(NT) void k_transfer(int64_t ndest, const int64_t* __restrict__ ptr,
                                                 const int64_t* __restrict__ idx, const double* __restrict__ src,
                                                 double* __restrict__ dest) {
  for (int64_t e = blockIdx.x * (int64_t)NT + threadIdx.x; e < ndest; e += (int64_t)gridDim.x * NT) {
    double s = 0.0;
    for (int64_t q = ptr[e]; q < ptr[e + 1]; ++q) s += src[idx[q]];
    dest[e] = s;
  }
}

// ------------------------------------------------------------------ compress_jacobian! (normalkkt.jl:163-172)
__global__ __launch_bounds__(NT) void k_compress_jac(double* __restrict__ AV, int64_t nnz, int32_t nslack,
                                                     const int64_t* __restrict__ map, double* __restrict__ ATnz) {
  // A.V[end-nslack+1:end] .= -1 happens before the gather; the gather may read those entries, so the
  // -1 is substituted in the read (one launch, no ordering hazard) and also stored.
  const int64_t s0 = nnz - nslack;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * NT) {
    const int64_t k = map[i];
    ATnz[i] = k >= s0 ? -1.0 : AV[k];
    if (i >= s0) AV[i] = -1.0;
  }
}

// ------------------------------------------------------------------ SpMV (cuda_wrapper.jl:43-94)
// y[r] = alpha * sum_q v[q] x[c[q]] + beta * y[r], entries of row r in storage order (G lanes per
// row stride the row, then a fixed butterfly: the order is fixed, so results are reproducible).
// vmap: optional indirection into the caller's live values (transposed operator).
template <int G>
__global__ __launch_bounds__(NT) void k_spmv_rows(int32_t nrows, const int64_t* __restrict__ rp,
                                                  const int32_t* __restrict__ ci, const double* __restrict__ v,
                                                  const int64_t* __restrict__ vmap, const double* __restrict__ x,
                                                  double* __restrict__ y, double alpha, double beta) {
  const int gl = threadIdx.x & (G - 1);
  for (int64_t r = (blockIdx.x * (int64_t)NT + threadIdx.x) / G; r < nrows; r += (int64_t)gridDim.x * (NT / G)) {
    double s = 0.0;
    const int64_t q1 = rp[r + 1];
    for (int64_t q = rp[r] + gl; q < q1; q += G) s += (vmap ? v[vmap[q]] : v[q]) * x[ci[q]];
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, G);
    if (gl == 0) y[r] = beta == 0.0 ? alpha * s : alpha * s + beta * y[r];
  }
}

// int32 row pointers of the caller's CSR ('N' operator reads the caller's arrays live)
template <int G>
__global__ __launch_bounds__(NT) void k_spmv_rows32(int32_t nrows, const int32_t* __restrict__ rp,
                                                    const int32_t* __restrict__ ci, const double* __restrict__ v,
                                                    const double* __restrict__ x, double* __restrict__ y,
                                                    double alpha, double beta) {
  const int gl = threadIdx.x & (G - 1);
  for (int64_t r = (blockIdx.x * (int64_t)NT + threadIdx.x) / G; r < nrows; r += (int64_t)gridDim.x * (NT / G)) {
    double s = 0.0;
    const int32_t q1 = rp[r + 1];
    for (int32_t q = rp[r] + gl; q < q1; q += G) s += v[q] * x[ci[q]];
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, G);
    if (gl == 0) y[r] = beta == 0.0 ? alpha * s : alpha * s + beta * y[r];
  }
}

// ------------------------------------------------------------------ coo_to_csr (utils.jl:158-201)
// also validates the indices: an entry outside [0, nrows) x [0, ncols) sets *bad (its key is clamped
// into the sort range, and the caller reports the error after the launch sequence)
__global__ __launch_bounds__(NT) void k_coo_keys(int64_t nnz, const int32_t* __restrict__ Ai,
                                                 const int32_t* __restrict__ Aj, int32_t nrows, int32_t ncols,
                                                 int sort_cols, uint64_t* __restrict__ key, int64_t* __restrict__ val,
                                                 int32_t* __restrict__ bad) {
  for (int64_t k = blockIdx.x * (int64_t)NT + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * NT) {
    int32_t i = Ai[k], j = Aj[k];
    if (i < 0 || i >= nrows || j < 0 || j >= ncols) {
      *bad = 1;
      i = 0;
      j = 0;
    }
    key[k] = sort_cols ? (uint64_t)i * (uint64_t)ncols + (uint64_t)j : (uint64_t)i;
    val[k] = k;
  }
}

__global__ __launch_bounds__(NT) void k_coo_scatter(int64_t nnz, const int64_t* __restrict__ perm,
                                                    const int32_t* __restrict__ Aj, const double* __restrict__ Ax,
                                                    int32_t* __restrict__ Bj, double* __restrict__ Bx) {
  for (int64_t q = blockIdx.x * (int64_t)NT + threadIdx.x; q < nnz; q += (int64_t)gridDim.x * NT) {
    const int64_t k = perm[q];
    Bj[q] = Aj[k];
    Bx[q] = Ax[k];
  }
}

// Bp[i] = first sorted position whose row is >= i (binary search over the sorted keys)
__global__ __launch_bounds__(NT) void k_coo_rowptr(int32_t nrows, int64_t nnz, const uint64_t* __restrict__ key,
                                                   uint64_t scale, int32_t* __restrict__ Bp) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i <= nrows; i += (int64_t)gridDim.x * NT) {
    const uint64_t target = (uint64_t)i * scale;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (key[mid] < target) lo = mid + 1; else hi = mid;
    }
    Bp[i] = (int32_t)lo;
  }
}

// ------------------------------------------------------------------ assemble_normal_system! (utils.jl:276-308)
// C entry c = (row j, column i), j >= i: Cx[c] = sum_k (Jx[i,k] * D[k]) * Jx[j,k], the merge-join of
// rows i and j of J over ascending column indices (cuda_wrapper.jl:108-139); the CPU loop sums the
// same products in row j's storage order, which is the same order for sorted rows.  One wave per
// column i of C: the wave's lanes take its entries.
__global__ __launch_bounds__(NT) void k_normal_merge(int32_t nrows, const int32_t* __restrict__ Jp,
                                                     const int32_t* __restrict__ Jj, const double* __restrict__ Jx,
                                                     const int32_t* __restrict__ Cp, const int32_t* __restrict__ Cj,
                                                     double* __restrict__ Cx, const double* __restrict__ Dx) {
#pragma clang fp contract(off)  // (a * d) * b then + acc, as the CPU loop rounds it (no FMA)
  const int lane = threadIdx.x & 63;
  for (int64_t i = (blockIdx.x * (int64_t)NT + threadIdx.x) >> 6; i < nrows; i += (int64_t)gridDim.x * (NT / 64)) {
    const int32_t a0 = Jp[i], a1 = Jp[i + 1];
    for (int32_t c = Cp[i] + lane; c < Cp[i + 1]; c += 64) {
      const int32_t j = Cj[c];
      int32_t p1 = a0, p2 = Jp[j];
      const int32_t p2e = Jp[j + 1];
      double acc = 0.0;
      while (p1 < a1 && p2 < p2e) {
        const int32_t k1 = Jj[p1], k2 = Jj[p2];
        if (k1 == k2) {
          acc += (Jx[p1] * Dx[k1]) * Jx[p2];
          ++p1;
          ++p2;
        } else if (k1 < k2) {
          ++p1;
        } else {
          ++p2;
        }
      }
      Cx[c] = acc;
    }
  }
}

// ------------------------------------------------------------------ fill_structure! (MadIPMCUDAExt.jl:15-32)
__global__ __launch_bounds__(NT) void k_fill_structure(int32_t nrows, const int32_t* __restrict__ Ap,
                                                       const int32_t* __restrict__ Aj, int32_t* __restrict__ rows,
                                                       int32_t* __restrict__ cols) {
  const int lane = threadIdx.x & 63;
  for (int64_t i = (blockIdx.x * (int64_t)NT + threadIdx.x) >> 6; i < nrows; i += (int64_t)gridDim.x * (NT / 64))
    for (int32_t c = Ap[i] + lane; c < Ap[i + 1]; c += 64) {
      rows[c] = (int32_t)i;
      cols[c] = Aj[c];
    }
}

// ------------------------------------------------------------------ QP evaluators (MadIPMCUDAExt.jl:34-45)
constexpr int DOT_BLOCKS = 256;
// partials of (c.x, v.x) per block, then one block sums them in fixed order
__global__ __launch_bounds__(NT) void k_dot2(int64_t n, const double* __restrict__ a, const double* __restrict__ b,
                                             const double* __restrict__ x, double* __restrict__ part) {
  double s0 = 0.0, s1 = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    s0 += a[i] * x[i];
    s1 += b[i] * x[i];
  }
  __shared__ double sh[2][NT / 64];
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_down(s0, o, 64);
    s1 += __shfl_down(s1, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = s0;
    sh[1][threadIdx.x >> 6] = s1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int w = 0; w < NT / 64; ++w) s += sh[threadIdx.x][w];
    part[threadIdx.x * DOT_BLOCKS + blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(NT) void k_dot2_final(const double* __restrict__ part, double c0, double* __restrict__ out) {
  __shared__ double sh[2][NT / 64];
  double s0 = threadIdx.x < DOT_BLOCKS ? part[threadIdx.x] : 0.0;
  double s1 = threadIdx.x < DOT_BLOCKS ? part[DOT_BLOCKS + threadIdx.x] : 0.0;
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_down(s0, o, 64);
    s1 += __shfl_down(s1, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = s0;
    sh[1][threadIdx.x >> 6] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < NT / 64; ++w) {
      a += sh[0][w];
      b += sh[1][w];
    }
    out[0] = c0 + a + b / 2;  // qp.data.c0 + dot(c, x) + dot(v, x) / 2
  }
}

__global__ __launch_bounds__(NT) void k_axpy1(int64_t n, const double* __restrict__ c, double* __restrict__ g) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) g[i] += c[i];
}

}  // namespace
}  // namespace madipm

using namespace madipm;

// ------------------------------------------------------------------ handles
struct madipm_transfer {
  int64_t nsrc = 0, ndest = 0;
  DBuf<int64_t> ptr, idx;
};

struct madipm_spmv {
  int32_t m = 0, n = 0;       // size(A)
  int32_t orows = 0;          // rows of op(A)
  int64_t nnzA = 0;
  char transa = 'N';
  bool symmetric = false;
  // 'N' (non-symmetric): the caller's arrays, read live
  const int32_t *rp32 = nullptr, *ci32 = nullptr;
  const double* v_live = nullptr;
  // owned operator (symmetric copy, or the transposed plan over the caller's live values)
  DBuf<int64_t> rp, vmap;
  DBuf<int32_t> ci;
  DBuf<double> v;
  int group = 8;
};

#define KKT_API_BEGIN try {
#define KKT_API_END                                           \
  }                                                           \
  catch (const madipm::Error& e) {                            \
    set_last_error(e.what());                                 \
    return e.code < 0 ? e.code : -1;                          \
  }                                                           \
  catch (const std::exception& e) {                           \
    set_last_error(std::string("exception: ") + e.what());    \
    return -1;                                                \
  }

static int spmv_group(double mean_row) {
  if (mean_row <= 3) return 2;
  if (mean_row <= 6) return 4;
  if (mean_row <= 12) return 8;
  if (mean_row <= 24) return 16;
  if (mean_row <= 48) return 32;
  return 64;
}

template <class RP>
static void launch_rows(int G, int32_t nrows, const RP* rp, const int32_t* ci, const double* v, const int64_t* vmap,
                        const double* x, double* y, double alpha, double beta, hipStream_t s);

template <>
void launch_rows<int64_t>(int G, int32_t nrows, const int64_t* rp, const int32_t* ci, const double* v,
                          const int64_t* vmap, const double* x, double* y, double alpha, double beta, hipStream_t s) {
  const unsigned grid = grid_for((int64_t)nrows * G);
  switch (G) {
    case 2: k_spmv_rows<2><<<grid, NT, 0, s>>>(nrows, rp, ci, v, vmap, x, y, alpha, beta); break;
    case 4: k_spmv_rows<4><<<grid, NT, 0, s>>>(nrows, rp, ci, v, vmap, x, y, alpha, beta); break;
    case 8: k_spmv_rows<8><<<grid, NT, 0, s>>>(nrows, rp, ci, v, vmap, x, y, alpha, beta); break;
    case 16: k_spmv_rows<16><<<grid, NT, 0, s>>>(nrows, rp, ci, v, vmap, x, y, alpha, beta); break;
    case 32: k_spmv_rows<32><<<grid, NT, 0, s>>>(nrows, rp, ci, v, vmap, x, y, alpha, beta); break;
    default: k_spmv_rows<64><<<grid, NT, 0, s>>>(nrows, rp, ci, v, vmap, x, y, alpha, beta); break;
  }
}

template <>
void launch_rows<int32_t>(int G, int32_t nrows, const int32_t* rp, const int32_t* ci, const double* v,
                          const int64_t*, const double* x, double* y, double alpha, double beta, hipStream_t s) {
  const unsigned grid = grid_for((int64_t)nrows * G);
  switch (G) {
    case 2: k_spmv_rows32<2><<<grid, NT, 0, s>>>(nrows, rp, ci, v, x, y, alpha, beta); break;
    case 4: k_spmv_rows32<4><<<grid, NT, 0, s>>>(nrows, rp, ci, v, x, y, alpha, beta); break;
    case 8: k_spmv_rows32<8><<<grid, NT, 0, s>>>(nrows, rp, ci, v, x, y, alpha, beta); break;
    case 16: k_spmv_rows32<16><<<grid, NT, 0, s>>>(nrows, rp, ci, v, x, y, alpha, beta); break;
    case 32: k_spmv_rows32<32><<<grid, NT, 0, s>>>(nrows, rp, ci, v, x, y, alpha, beta); break;
    default: k_spmv_rows32<64><<<grid, NT, 0, s>>>(nrows, rp, ci, v, x, y, alpha, beta); break;
  }
}

extern "C" {

// ---------------------------------------------------------------- transfer!
int madipm_transfer_create(int64_t nsrc, const int64_t* map, int32_t map_on_device, int64_t ndest,
                           madipm_transfer_t* out) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(out && (nsrc == 0 || map) && nsrc >= 0 && ndest >= 0, "madipm_transfer_create: bad argument");
  std::vector<int64_t> h = to_host(map, nsrc, map_on_device != 0);
  std::vector<int64_t> ptr(ndest + 1, 0), idx(nsrc);
  for (int64_t k = 0; k < nsrc; ++k) {
    MADIPM_REQUIRE(h[k] >= 0 && h[k] < ndest, "madipm_transfer_create: map entry out of range");
    ptr[h[k] + 1]++;
  }
  for (int64_t e = 0; e < ndest; ++e) ptr[e + 1] += ptr[e];
  std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
  for (int64_t k = 0; k < nsrc; ++k) idx[fill[h[k]]++] = k;  // ascending k within a destination
  auto t = new struct madipm_transfer();
  t->nsrc = nsrc;
  t->ndest = ndest;
  t->ptr.upload(ptr);
  t->idx.upload(idx);
  MADIPM_HIP(hipDeviceSynchronize());
  *out = t;
  return 0;
  KKT_API_END
}

int madipm_transfer(madipm_transfer_t t, double* d_dest, const double* d_src, madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(t && (t->ndest == 0 || d_dest) && (t->nsrc == 0 || d_src), "madipm_transfer: bad argument");
  if (t->ndest == 0) return 0;
  auto s = (hipStream_t)stream;
  k_transfer<<<grid_for(t->ndest), NT, 0, s>>>(t->ndest, t->ptr, t->idx, d_src, d_dest);
  MADIPM_HIP(hipGetLastError());
  return 0;
  KKT_API_END
}

void madipm_transfer_destroy(madipm_transfer_t t) { delete t; }

// ---------------------------------------------------------------- compress_jacobian!
int madipm_compress_jacobian(double* d_AV, int64_t nnz, int32_t n_slack, const int64_t* d_csr_map, double* d_ATnz,
                             madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(nnz >= 0 && n_slack >= 0 && n_slack <= nnz, "madipm_compress_jacobian: bad sizes");
  if (nnz == 0) return 0;
  MADIPM_REQUIRE(d_AV && d_csr_map && d_ATnz, "madipm_compress_jacobian: null pointer");
  k_compress_jac<<<grid_for(nnz), NT, 0, (hipStream_t)stream>>>(d_AV, nnz, n_slack, d_csr_map, d_ATnz);
  MADIPM_HIP(hipGetLastError());
  return 0;
  KKT_API_END
}

// ---------------------------------------------------------------- MadIPMOperator
int madipm_spmv_create(int32_t m, int32_t n, int64_t nnz, const int32_t* d_rowptr, const int32_t* d_colval,
                       const double* d_nzval, char transa, int32_t symmetric, madipm_spmv_t* out) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(out && m >= 0 && n >= 0 && nnz >= 0, "madipm_spmv_create: bad argument");
  MADIPM_REQUIRE(transa == 'N' || transa == 'T', "madipm_spmv_create: transa must be 'N' or 'T'");
  MADIPM_REQUIRE(!symmetric || m == n, "madipm_spmv_create: a symmetric operator must be square");
  MADIPM_REQUIRE(d_rowptr && (nnz == 0 || (d_colval && d_nzval)), "madipm_spmv_create: null pointer");
  auto op = std::make_unique<madipm_spmv>();
  op->m = m;
  op->n = n;
  op->nnzA = nnz;
  op->transa = transa;
  op->symmetric = symmetric && nnz > 0;  // bool = symmetric && (nnz(A) > 0), cuda_wrapper.jl:66
  op->orows = transa == 'N' ? m : n;
  std::vector<int32_t> rp = to_host(d_rowptr, (int64_t)m + 1, true);
  MADIPM_REQUIRE(rp[0] == 0 && rp[m] == nnz, "madipm_spmv_create: rowptr does not match nnz");
  if (op->symmetric) {
    // mat = tril(A, -1) + A' (cuda_wrapper.jl:67): a copy, with each (i, j) combined in one entry
    // and columns ascending, as SparseArrays' sum produces it
    std::vector<int32_t> ci = to_host(d_colval, nnz, true);
    std::vector<double> v = to_host(d_nzval, nnz, true);
    std::vector<int64_t> cnt(m + 1, 0);
    for (int32_t i = 0; i < m; ++i)
      for (int64_t q = rp[i]; q < rp[i + 1]; ++q) {
        const int32_t j = ci[q];
        MADIPM_REQUIRE(j >= 0 && j < n, "madipm_spmv_create: column index out of range");
        if (i > j) cnt[i + 1]++;
        cnt[j + 1]++;
      }
    for (int32_t i = 0; i < m; ++i) cnt[i + 1] += cnt[i];
    std::vector<int32_t> tj(cnt[m]);
    std::vector<double> tv(cnt[m]);
    std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
    // tril(A, -1) part first, then A' (the order of the two terms in the sum)
    for (int32_t i = 0; i < m; ++i)
      for (int64_t q = rp[i]; q < rp[i + 1]; ++q)
        if (i > ci[q]) { tj[fill[i]] = ci[q]; tv[fill[i]++] = v[q]; }
    for (int32_t i = 0; i < m; ++i)
      for (int64_t q = rp[i]; q < rp[i + 1]; ++q) { tj[fill[ci[q]]] = i; tv[fill[ci[q]]++] = v[q]; }
    std::vector<int64_t> orp(m + 1, 0);
    std::vector<int32_t> oj;
    std::vector<double> ov;
    oj.reserve(tj.size());
    ov.reserve(tj.size());
    std::vector<int64_t> ord;
    for (int32_t i = 0; i < m; ++i) {
      ord.resize(cnt[i + 1] - cnt[i]);
      std::iota(ord.begin(), ord.end(), cnt[i]);
      std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return tj[a] < tj[b]; });
      for (size_t t = 0; t < ord.size(); ++t) {
        if (!oj.empty() && (int64_t)oj.size() > orp[i] && oj.back() == tj[ord[t]])
          ov.back() += tv[ord[t]];
        else {
          oj.push_back(tj[ord[t]]);
          ov.push_back(tv[ord[t]]);
        }
      }
      orp[i + 1] = (int64_t)oj.size();
    }
    op->rp.upload(orp);
    op->ci.upload(oj);
    op->v.upload(ov);
    op->group = spmv_group(m ? (double)oj.size() / m : 1.0);
  } else if (transa == 'T') {
    // y = A' x: the transposed structure (rows of A', i.e. columns of A, ascending row of A within
    // each) with a position map into the caller's values, which are read live at every apply
    std::vector<int32_t> ci = to_host(d_colval, nnz, true);
    std::vector<int64_t> cp(n + 1, 0), map(nnz);
    std::vector<int32_t> ri(nnz);
    for (int64_t q = 0; q < nnz; ++q) {
      MADIPM_REQUIRE(ci[q] >= 0 && ci[q] < n, "madipm_spmv_create: column index out of range");
      cp[ci[q] + 1]++;
    }
    for (int32_t j = 0; j < n; ++j) cp[j + 1] += cp[j];
    std::vector<int64_t> fill(cp.begin(), cp.end() - 1);
    for (int32_t i = 0; i < m; ++i)
      for (int64_t q = rp[i]; q < rp[i + 1]; ++q) {
        ri[fill[ci[q]]] = i;
        map[fill[ci[q]]++] = q;
      }
    op->rp.upload(cp);
    op->ci.upload(ri);
    op->vmap.upload(map);
    op->v_live = d_nzval;
    op->group = spmv_group(n ? (double)nnz / n : 1.0);
  } else {
    op->rp32 = d_rowptr;
    op->ci32 = d_colval;
    op->v_live = d_nzval;
    op->group = spmv_group(m ? (double)nnz / m : 1.0);
  }
  MADIPM_HIP(hipDeviceSynchronize());
  *out = op.release();
  return 0;
  KKT_API_END
}

int madipm_spmv_size(madipm_spmv_t op, int32_t* m, int32_t* n, int64_t* nnz) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(op, "null handle");
  if (m) *m = op->m;
  if (n) *n = op->n;
  if (nnz) *nnz = op->nnzA;  // SparseArrays.nnz(A::MadIPMOperator) = nnz(A.A)
  return 0;
  KKT_API_END
}

int madipm_spmv_apply(madipm_spmv_t op, const double* d_x, double* d_y, double alpha, double beta,
                      madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(op && (op->orows == 0 || d_y), "madipm_spmv_apply: bad argument");
  if (op->orows == 0) return 0;
  auto s = (hipStream_t)stream;
  if (op->rp32)
    launch_rows<int32_t>(op->group, op->orows, op->rp32, op->ci32, op->v_live, nullptr, d_x, d_y, alpha, beta, s);
  else if (op->symmetric)
    launch_rows<int64_t>(op->group, op->orows, op->rp.p, op->ci.p, op->v.p, nullptr, d_x, d_y, alpha, beta, s);
  else
    launch_rows<int64_t>(op->group, op->orows, op->rp.p, op->ci.p, op->v_live, op->vmap.p, d_x, d_y, alpha, beta, s);
  MADIPM_HIP(hipGetLastError());
  return 0;
  KKT_API_END
}

void madipm_spmv_destroy(madipm_spmv_t op) { delete op; }

// ---------------------------------------------------------------- coo_to_csr
int madipm_coo_to_csr(int32_t n_rows, int32_t n_cols, int64_t nnz, const int32_t* d_Ai, const int32_t* d_Aj,
                      const double* d_Ax, int32_t* d_rowptr, int32_t* d_colval, double* d_nzval, int32_t sort_cols,
                      madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(n_rows >= 0 && n_cols >= 0 && nnz >= 0 && nnz < (int64_t)INT32_MAX, "madipm_coo_to_csr: bad sizes");
  MADIPM_REQUIRE(d_rowptr && (nnz == 0 || (d_Ai && d_Aj && d_Ax && d_colval && d_nzval)),
                 "madipm_coo_to_csr: null pointer");
  auto s = (hipStream_t)stream;
  DBuf<uint64_t> k_in(std::max<int64_t>(1, nnz)), k_out(std::max<int64_t>(1, nnz));
  DBuf<int64_t> v_in(std::max<int64_t>(1, nnz)), v_out(std::max<int64_t>(1, nnz));
  const uint64_t scale = sort_cols ? (uint64_t)std::max(1, n_cols) : 1;
  DBuf<int32_t> bad(1);
  bad.zero(s);
  if (nnz > 0) {
    k_coo_keys<<<grid_for(nnz), NT, 0, s>>>(nnz, d_Ai, d_Aj, n_rows, std::max(1, n_cols), sort_cols, k_in, v_in,
                                            bad.p);
    // LSD radix sort is stable: equal keys keep the input order (utils.jl's counting sort order)
    const uint64_t maxkey = ((uint64_t)std::max(1, n_rows)) * scale;
    int end_bit = 1;
    while (end_bit < 64 && (1ull << end_bit) <= maxkey) ++end_bit;
    size_t tmp_bytes = 0;
    MADIPM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k_in.p, k_out.p, v_in.p, v_out.p, (int)nnz, 0,
                                                  end_bit, s));
    DBuf<uint8_t> tmp(std::max<size_t>(1, tmp_bytes));
    MADIPM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tmp_bytes, k_in.p, k_out.p, v_in.p, v_out.p, (int)nnz, 0,
                                                  end_bit, s));
    k_coo_scatter<<<grid_for(nnz), NT, 0, s>>>(nnz, v_out, d_Aj, d_Ax, d_colval, d_nzval);
  }
  k_coo_rowptr<<<grid_for((int64_t)n_rows + 1), NT, 0, s>>>(n_rows, nnz, k_out, scale, d_rowptr);
  MADIPM_HIP(hipGetLastError());
  MADIPM_HIP(hipStreamSynchronize(s));  // the temporaries are released on return
  int32_t hbad = 0;
  MADIPM_HIP(hipMemcpy(&hbad, bad.p, sizeof(int32_t), hipMemcpyDeviceToHost));
  MADIPM_REQUIRE(hbad == 0, "madipm_coo_to_csr: a row or column index is out of range (outputs are invalid)");
  return 0;
  KKT_API_END
}

// ---------------------------------------------------------------- build_normal_system (host)
int madipm_build_normal_system(int32_t n_rows, int32_t n_cols, const int32_t* Jtp, const int32_t* Jtj, int32_t* Cp,
                               int32_t* Cj, int64_t cap, int64_t* nnz_out) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(n_rows >= 0 && n_cols >= 0 && Jtp && Cp && nnz_out, "madipm_build_normal_system: bad argument");
  const int64_t nz = Jtp[n_rows];
  // columns of J -> their rows (ascending)
  std::vector<int64_t> cp(n_cols + 1, 0);
  for (int64_t q = 0; q < nz; ++q) {
    MADIPM_REQUIRE(Jtj[q] >= 0 && Jtj[q] < n_cols, "madipm_build_normal_system: column index out of range");
    cp[Jtj[q] + 1]++;
  }
  for (int32_t k = 0; k < n_cols; ++k) cp[k + 1] += cp[k];
  std::vector<int32_t> rows(nz);
  std::vector<int64_t> fill(cp.begin(), cp.end() - 1);
  for (int32_t i = 0; i < n_rows; ++i)
    for (int32_t q = Jtp[i]; q < Jtp[i + 1]; ++q) rows[fill[Jtj[q]]++] = i;
  // column i of tril(J J'): the rows j >= i sharing a column with row i, ascending (utils.jl:226-235)
  std::vector<int32_t> mark(n_rows, -1), lst;
  int64_t total = 0;
  Cp[0] = 0;
  for (int32_t i = 0; i < n_rows; ++i) {
    lst.clear();
    for (int32_t q = Jtp[i]; q < Jtp[i + 1]; ++q) {
      const int32_t k = Jtj[q];
      // rows of column k are ascending: start at the first row >= i
      const int32_t* b = rows.data() + cp[k];
      const int32_t* e = rows.data() + cp[k + 1];
      for (const int32_t* r = std::lower_bound(b, e, i); r != e; ++r)
        if (mark[*r] != i) {
          mark[*r] = i;
          lst.push_back(*r);
        }
    }
    std::sort(lst.begin(), lst.end());
    if (Cj && total + (int64_t)lst.size() <= cap) std::copy(lst.begin(), lst.end(), Cj + total);
    total += (int64_t)lst.size();
    MADIPM_REQUIRE(total < (int64_t)INT32_MAX, "madipm_build_normal_system: nnz exceeds int32");
    Cp[i + 1] = (int32_t)total;
  }
  *nnz_out = total;
  if (Cj && total > cap) {
    set_last_error("madipm_build_normal_system: cap < nnz (" + std::to_string(total) + "): Cj not filled");
    return -4;
  }
  return 0;
  KKT_API_END
}

// ---------------------------------------------------------------- assemble_normal_system!
int madipm_assemble_normal_system(int32_t n_rows, int32_t n_cols, const int32_t* d_Jtp, const int32_t* d_Jtj,
                                  const double* d_Jtx, const int32_t* d_Cp, const int32_t* d_Cj, double* d_Cx,
                                  const double* d_Dx, madipm_stream_t stream) {
  KKT_API_BEGIN
  (void)n_cols;
  MADIPM_REQUIRE(n_rows >= 0 && d_Jtp && d_Cp, "madipm_assemble_normal_system: bad argument");
  if (n_rows == 0) return 0;
  k_normal_merge<<<grid_for((int64_t)n_rows * 64), NT, 0, (hipStream_t)stream>>>(n_rows, d_Jtp, d_Jtj, d_Jtx, d_Cp,
                                                                                  d_Cj, d_Cx, d_Dx);
  MADIPM_HIP(hipGetLastError());
  return 0;
  KKT_API_END
}

// ---------------------------------------------------------------- fill_structure!
int madipm_csr_fill_structure(int32_t n_rows, const int32_t* d_Ap, const int32_t* d_Aj, int32_t* d_rows,
                              int32_t* d_cols, madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(n_rows >= 0 && d_Ap, "madipm_csr_fill_structure: bad argument");
  if (n_rows == 0) return 0;
  k_fill_structure<<<grid_for((int64_t)n_rows * 64), NT, 0, (hipStream_t)stream>>>(n_rows, d_Ap, d_Aj, d_rows, d_cols);
  MADIPM_HIP(hipGetLastError());
  return 0;
  KKT_API_END
}

// ---------------------------------------------------------------- QP evaluators
int madipm_qp_obj(madipm_spmv_t H, const double* d_c, double c0, const double* d_x, double* d_v, int32_t n,
                  double* d_work, double* h_obj, madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(H && H->orows == n && d_work, "madipm_qp_obj: bad argument");
  auto s = (hipStream_t)stream;
  int rc = madipm_spmv_apply(H, d_x, d_v, 1.0, 0.0, stream);  // mul!(qp.data.v, qp.data.H, x)
  if (rc) return rc;
  k_dot2<<<DOT_BLOCKS, NT, 0, s>>>(n, d_c, d_v, d_x, d_work);
  k_dot2_final<<<1, NT, 0, s>>>(d_work, c0, d_work + 2 * DOT_BLOCKS);
  MADIPM_HIP(hipGetLastError());
  if (h_obj) {
    MADIPM_HIP(hipMemcpyAsync(h_obj, d_work + 2 * DOT_BLOCKS, sizeof(double), hipMemcpyDeviceToHost, s));
    MADIPM_HIP(hipStreamSynchronize(s));
  }
  return 0;
  KKT_API_END
}

int madipm_qp_grad(madipm_spmv_t H, const double* d_c, const double* d_x, double* d_g, int32_t n,
                   madipm_stream_t stream) {
  KKT_API_BEGIN
  MADIPM_REQUIRE(H && H->orows == n, "madipm_qp_grad: bad argument");
  int rc = madipm_spmv_apply(H, d_x, d_g, 1.0, 0.0, stream);  // mul!(g, qp.data.H, x)
  if (rc) return rc;
  if (n > 0) k_axpy1<<<grid_for(n), NT, 0, (hipStream_t)stream>>>(n, d_c, d_g);  // g .+= qp.data.c
  MADIPM_HIP(hipGetLastError());
  return 0;
  KKT_API_END
}

}  // extern "C"
