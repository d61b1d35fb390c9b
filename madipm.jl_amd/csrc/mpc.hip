// Native MPC driver + fused IPM vector kernels (gfx950).
//
// Restates MadIPM's per-iteration path on the GPU (file:line relative to the reference root):
//   update_termination_criteria!  src/solver.jl:194-222  -> k_term + k_final(TERM)
//   set_aug_diagonal_reg! (K2)    src/kernels.jl:124-136 -> k_diag (also writes the K2 diagonal)
//   factorize_regularized_system! src/linear_solver.jl:6-17 -> LDLSolver::factorize_async (+retry)
//   set_predictive_rhs! / set_correction_rhs! / reduce_rhs!  src/kernels.jl:21-58 -> k_rhs
//   solve_system! + finish_aug_solve! + residual (mul!, _kktmul!)  src/linear_solver.jl:19-44 -> k_residual
//   get_fraction_to_boundary_step (max-ratio test)  src/kernels.jl:226-289 -> k_alpha (argmin)
//   get_(affine_)complementarity_measure, update_barrier!  src/kernels.jl:155-220 -> k_mu
//   update_step! (Adaptive/Conservative/MehrotraAdaptive)  src/kernels.jl:291-358 -> k_alpha/k_mu FINAL
//   apply_step! + adjust_boundary!  src/solver.jl:308-317 -> k_apply
//   evaluate_model!  src/solver.jl:319-326 -> k_eval (SpMV H x, J x, J^T y, objective)
//   init_starting_point!  src/solver.jl:6-125 -> k_init_kkt, k_rhs(INIT_*), k_zinit, k_zshift1/2
// Reductions are two-pass (per-block partials, then one finalising block in fixed order), so every
// scalar is bitwise reproducible run to run; all scalars stay on the device and the host reads one
// 200-byte state block per iteration (published by k_publish into coherent host memory; the host
// spins on its counter, overlapped with the factorisation and the speculated directions).
#include <algorithm>
#include <array>
#include <atomic>
#include <thread>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>

#include "mpc.hpp"

namespace madipm {

struct QPHost {
  int nx = 0, m = 0, n = 0, ns = 0;
  std::vector<double> c, lvar, uvar, lcon, ucon, x0, y0, Hv;
  std::vector<int32_t> Hr, Hc;
  // A's COO: the caller's arrays, read during construction only (no host copy: 8 GB for the dense QP)
  const int32_t* Ar = nullptr;
  const int32_t* Ac = nullptr;
  const double* Av = nullptr;
  int64_t nnzA = 0;
  double c0 = 0, sgn = 1;
  bool minimize = true;
  std::vector<int32_t> ind_ineq, ind_fixed, ind_lb, ind_ub;
  std::vector<uint8_t> fixed;
  bool has_ineq = false;
  std::vector<double> con_scale;
  double obj_scale = 1;
  std::vector<double> x, xl, xu, rhs, y;
};

namespace {

constexpr int NT = 256;
constexpr int NPART = 16;
constexpr int MAXB = 2048;  // partial-reduction blocks (part_ holds NPART x MAXB, value-major)
// partial k of block b: value-major so k_final's loads of one value are coalesced
__device__ __forceinline__ int pidx(int b, int k) { return k * MAXB + b; }
constexpr double INF = std::numeric_limits<double>::infinity();

struct DCsr {
  const int64_t* rp;
  const int32_t* ci;
  const double* v;
};

struct DV {
  int n, m, nx, nlb, nub;
  double *x, *xl, *xu, *zl, *zu, *f, *jacl, *c, *y, *rhs;
  double *pr_diag, *l_diag, *u_diag, *l_lower, *u_lower;
  double *d, *p, *corr_lb, *corr_ub;
  double* Kx;
  const int64_t* diag_pos;
  const double *Hdiag, *cs, *gfix, *cfix;
  const int32_t *ind_lb, *ind_ub, *lbpos, *ubpos;
  const uint8_t* fixed;
  DCsr H, J, JT;
  double* part;
  DevState* st;
  // KKT formulation (madipm_options.kkt_system): K2 / K2.5 (scaled) / normal equations
  int kkt;
  double* sk;               // K2.5: primal scaling s_i = sqrt(dist_l * dist_u)
  const int32_t *Krow, *Kcol;
  const double* K0;         // K2.5: unscaled K2 values (off-diagonal entries are constant)
  int64_t nnzK;
  double* Dinv;             // normal: 1 ./ pr_diag
  double* bufm;             // normal: right-hand side / solution of the m x m system
  const int64_t* cpp;       // normal: C entry e = sum over products [cpp[e], cpp[e+1])
  const int2* cprod;        //   product = (position of A_ik, position of A_jk) in J's values
  double* Cx;               //   values of C = A Sigma^{-1} A^T (lower CSC)
  int64_t nnzC;
};

enum { KKT_K2 = 0, KKT_K25 = 1, KKT_NORMAL = 2 };

enum { OP_SUM = 0, OP_MAX = 1, OP_MIN = 2 };

__device__ __forceinline__ double nmax(double a, double b) { return ((b > a) | (b != b)) ? b : a; }
__device__ __forceinline__ double comb(double a, double b, int op) {
  return op == OP_SUM ? a + b : (op == OP_MAX ? nmax(a, b) : fmin(a, b));
}
__device__ __forceinline__ double csr_dot(const DCsr& A, int row, const double* __restrict__ x) {
  double s = 0.0;
  for (int64_t q = A.rp[row]; q < A.rp[row + 1]; ++q) s += A.v[q] * x[A.ci[q]];
  return s;
}

// Wave reductions with the pairing of the `for (o = 32; o; o >>= 1) a = op(a, __shfl_down(a, o))` tree
// (lane i combines lane i + o; lane 0 ends with the same value bit for bit), without the LDS crossbar:
// o = 32 / 16 by the gfx950 half-row swaps (v_permlane32_swap / v_permlane16_swap: the swapped-in half
// is lane i + o for the lanes the tree reads), o = 8, 4, 2, 1 by DPP row_shl:o inside each 16-lane row.
// (ds_bpermute costs an LDS round trip per step: k_final's level-1 tree took ~2 us, MADIPM_FINAL_DEBUG.)
template <int O>
__device__ __forceinline__ int lane_down_i32(int v) {
  if constexpr (O == 32) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (int)p[1];
  } else if constexpr (O == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (int)p[1];
  } else {
    return __builtin_amdgcn_update_dpp(v, v, 0x100 + O, 0xf, 0xf, false);  // row_shl:O
  }
}
template <int O>
__device__ __forceinline__ double lane_down(double v) {
  return __hiloint2double(lane_down_i32<O>(__double2hiint(v)), lane_down_i32<O>(__double2loint(v)));
}
template <int OP>
__device__ __forceinline__ double wave_reduce(double a) {
  a = comb(a, lane_down<32>(a), OP);
  a = comb(a, lane_down<16>(a), OP);
  a = comb(a, lane_down<8>(a), OP);
  a = comb(a, lane_down<4>(a), OP);
  a = comb(a, lane_down<2>(a), OP);
  return comb(a, lane_down<1>(a), OP);
}
template <int O>
__device__ __forceinline__ void argmin_step(double& a, int& b);
__device__ __forceinline__ double wave_reduce_op(double a, int op) {
  return op == OP_SUM ? wave_reduce<OP_SUM>(a) : (op == OP_MAX ? wave_reduce<OP_MAX>(a) : wave_reduce<OP_MIN>(a));
}

template <int NV>
__device__ void block_partials(double (&v)[NV], const int (&ops)[NV], double* part, int base = 0, int bid = -1) {
  __shared__ double sh[NV][NT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double a = wave_reduce_op(v[k], ops[k]);
    if (lane == 0) sh[k][wv] = a;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int k = threadIdx.x;
    double a = sh[k][0];
    for (int w = 1; w < NT / 64; ++w) a = comb(a, sh[k][w], ops[k]);
    part[pidx(bid >= 0 ? bid : (int)blockIdx.x, base + k)] = a;
  }
}

// (value, index) argmin in the order of the reference's left fold (kernels.jl:226-272:
// mapreduce(...; init = (1.0, 0)) with `elem1[1] < elem2[1] ? elem1 : elem2`): a later element
// replaces the accumulator unless the accumulator is strictly smaller, so among equal ratios the
// LAST index wins.  As a total order, (value ascending, index descending): associative, so any
// combine tree gives the fold's answer.  The init element is index -1 (below every real index).
__device__ __forceinline__ void amin_upd(double& v, int& ix, double nv, int ni) {
  const bool take = (nv < v) | ((nv == v) & (ni > ix));  // no short circuit: selects, not branches
  v = take ? nv : v;
  ix = take ? ni : ix;
}

template <int O>
__device__ __forceinline__ void argmin_step(double& a, int& b) {
  const double a2 = lane_down<O>(a);
  const int b2 = lane_down_i32<O>(b);
  amin_upd(a, b, a2, b2);
}
__device__ __forceinline__ void wave_argmin(double& a, int& b) {
  argmin_step<32>(a, b);
  argmin_step<16>(a, b);
  argmin_step<8>(a, b);
  argmin_step<4>(a, b);
  argmin_step<2>(a, b);
  argmin_step<1>(a, b);
}

#define GRID_LOOP(i, N) for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (N); i += (int64_t)gridDim.x * blockDim.x)

// SpMV rows in groups of G lanes (G | 64): the group's lanes stride the row's entries (coalesced),
// then a G-wide butterfly sums them (every lane of the group holds the row sum).  G is chosen per
// problem from the mean row length (MPCSolver::spmv_group).
#define GROUP_LOOP(i, N, G) \
  for (int64_t i = (blockIdx.x * (int64_t)NT + threadIdx.x) / (G); i < (N); i += (int64_t)gridDim.x * (NT / (G)))
// the same loops over a sub-grid of nblk blocks (block bid of it): kernels whose blocks split into roles
#define GROUP_LOOP_B(i, N, G, bid, nblk) \
  for (int64_t i = ((bid) * (int64_t)NT + threadIdx.x) / (G); i < (N); i += (int64_t)(nblk) * (NT / (G)))
#define GRID_LOOP_B(i, N, bid, nblk) \
  for (int64_t i = (bid) * (int64_t)blockDim.x + threadIdx.x; i < (N); i += (int64_t)(nblk) * blockDim.x)

template <int G>
__device__ __forceinline__ double gdot(const DCsr& A, int64_t row, const double* __restrict__ x) {
  const int gl = threadIdx.x & (G - 1);
  double s = 0.0;
  const int64_t q1 = A.rp[row + 1];
  // two entries per lane and trip, both issued before either is summed (clamped index, the second
  // masked): the gathers of consecutive trips no longer wait for each other; same summation order
  for (int64_t q = A.rp[row] + gl; q < q1; q += 2 * G) {
    const int64_t qb = min(q + G, q1 - 1);
    const double va = A.v[q], vb = A.v[qb];
    const double xa = x[A.ci[q]], xb = x[A.ci[qb]];
    s = fma(va, xa, s);
    s = fma((q + G < q1) ? vb : 0.0, xb, s);
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, G);
  return s;
}

// gdot<G>(A, ra, xa) and gdot<G>(B, rb, xb) at once (a primal row's H and J^T parts): both rows'
// extents, then each trip's entries and gathers of both, issued before either is summed — one chain
// of dependent loads instead of two back to back.  Each sum in gdot's own order (same bits).
template <int G>
__device__ __forceinline__ void gdot2(const DCsr& A, int64_t ra, const double* __restrict__ xa, const DCsr& B,
                                      int64_t rb, const double* __restrict__ xb, double& sa, double& sb) {
  const int gl = threadIdx.x & (G - 1);
  const int64_t a1 = A.rp[ra + 1], b1 = B.rp[rb + 1];
  int64_t qa = A.rp[ra] + gl, qb = B.rp[rb] + gl;
  sa = 0.0;
  sb = 0.0;
  while (qa < a1 || qb < b1) {
    const bool ta = qa < a1, tb = qb < b1;
    double va = 0.0, va2 = 0.0, ya = 0.0, ya2 = 0.0, vb = 0.0, vb2 = 0.0, yb = 0.0, yb2 = 0.0;
    if (ta) {
      const int64_t q2 = min(qa + G, a1 - 1);
      va = A.v[qa];
      va2 = A.v[q2];
      ya = xa[A.ci[qa]];
      ya2 = xa[A.ci[q2]];
    }
    if (tb) {
      const int64_t q2 = min(qb + G, b1 - 1);
      vb = B.v[qb];
      vb2 = B.v[q2];
      yb = xb[B.ci[qb]];
      yb2 = xb[B.ci[q2]];
    }
    if (ta) {
      sa = fma(va, ya, sa);
      sa = fma((qa + G < a1) ? va2 : 0.0, ya2, sa);
      qa += 2 * G;
    }
    if (tb) {
      sb = fma(vb, yb, sb);
      sb = fma((qb + G < b1) ? vb2 : 0.0, yb2, sb);
      qb += 2 * G;
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) {
    sa += __shfl_xor(sa, o, G);
    sb += __shfl_xor(sb, o, G);
  }
}

// ------------------------------------------------------------------ KKT diagonal (kernels.jl:124-149)
// K2 (set_aug_diagonal! for SparseKKTSystem, kernels.jl:124-136): pr_diag into the K2 diagonal.
// K2.5 (kernels.jl:139-149 + MadNLP._set_aug_diagonal! [EXT]): the primal block is scaled
// symmetrically by S = diag(s), s_i = sqrt((x - xl)(xu - x)) (a missing bound contributes 1), so the
// diagonal is s^2 (dw + H_ii) + zl (xu - x) + zu (x - xl) — bounded as x approaches a bound.
// Normal equations (NormalKKTSystem.build_kkt!, normalkkt.jl:180-194): Dinv = 1 ./ pr_diag.
// l_diag / u_diag keep the K2 sign convention (xl - x, x - xu) in every mode: they feed the
// unreduced operator of the residual, which is the same for the three formulations.
__device__ __forceinline__ void diag_entry(const DV& D, int64_t i, double dw, double dc) {
  if (i < D.n) {
    double pr = dw;
    const int kl = D.lbpos[i], ku = D.ubpos[i];
    const double x = D.x[i];
    double dl = 1.0, du = 1.0, zlv = 0.0, zuv = 0.0;
    if (kl >= 0) {
      const double ld = D.xl[i] - x, zl = D.zl[i];
      D.l_diag[kl] = ld;
      D.l_lower[kl] = zl;
      pr -= zl / ld;
      dl = -ld;
      zlv = zl;
    }
    if (ku >= 0) {
      const double ud = x - D.xu[i], zu = D.zu[i];
      D.u_diag[ku] = ud;
      D.u_lower[ku] = zu;
      pr -= zu / ud;
      du = -ud;
      zuv = zu;
    }
    D.pr_diag[i] = pr;
    if (D.kkt == KKT_NORMAL) {
      D.Dinv[i] = 1.0 / pr;
    } else if (D.kkt == KKT_K25) {
      const double s2 = dl * du;
      D.sk[i] = sqrt(s2);
      D.Kx[D.diag_pos[i]] = s2 * (dw + D.Hdiag[i]) + zlv * du + zuv * dl;
    } else {
      D.Kx[D.diag_pos[i]] = pr + D.Hdiag[i];
    }
  } else if (D.kkt != KKT_NORMAL) {
    D.Kx[D.diag_pos[i]] = dc;
  }
}

// rs != nullptr: the factorisation that follows starts here (LinSolver::ext_reset)
__global__ __launch_bounds__(NT) void k_diag(DV D, double dw, double dc, LDLStatus* rs) {
  if (rs && blockIdx.x == 0 && threadIdx.x == 0) ldl_status_start(rs);
  GRID_LOOP(i, D.n + D.m) diag_entry(D, i, dw, dc);
}

// MadNLP.initialize!(kkt) + init_starting_point! lines 16-18 (l_diag = u_diag = 1, l/u_lower = 0,
// pr_diag = dw; K2.5 scaling factor 1)
__global__ __launch_bounds__(NT) void k_init_kkt(DV D, double dw, double dc, LDLStatus* rs) {
  if (rs && blockIdx.x == 0 && threadIdx.x == 0) ldl_status_start(rs);
  GRID_LOOP(i, D.n + D.m) {
    if (i < D.n) {
      const int kl = D.lbpos[i], ku = D.ubpos[i];
      if (kl >= 0) {
        D.l_diag[kl] = 1.0;
        D.l_lower[kl] = 0.0;
      }
      if (ku >= 0) {
        D.u_diag[ku] = 1.0;
        D.u_lower[ku] = 0.0;
      }
      D.pr_diag[i] = dw;
      if (D.kkt == KKT_NORMAL) {
        D.Dinv[i] = 1.0 / dw;
      } else {
        if (D.kkt == KKT_K25) D.sk[i] = 1.0;
        D.Kx[D.diag_pos[i]] = dw + D.Hdiag[i];
      }
    } else if (D.kkt != KKT_NORMAL) {
      D.Kx[D.diag_pos[i]] = dc;
    }
  }
}

// K2.5: off-diagonal entries K[e] = s_row s_col K0[e] (s = 1 on the dual block)
__global__ __launch_bounds__(NT) void k_k25_scale(DV D) {
  GRID_LOOP(e, D.nnzK) {
    const int r = D.Krow[e], c = D.Kcol[e];
    if (r == c) continue;
    const double sr = r < D.n ? D.sk[r] : 1.0, sc = c < D.n ? D.sk[c] : 1.0;
    D.Kx[e] = sr * sc * D.K0[e];
  }
}

// K2.5: dx = S (S^{-1} dx) after the scaled solve
__global__ __launch_bounds__(NT) void k_k25_unscale(DV D) {
  GRID_LOOP(i, D.n) D.d[i] *= D.sk[i];
}

// NormalKKTSystem.build_kkt! / assemble_normal_system! (normalkkt.jl:180-194, utils.jl:276-308):
// C_ij = sum_k A_ik Sigma_k^{-1} A_jk over the precomputed product list of entry (i, j) — one
// thread per entry of tril(C), fixed summation order, no atomics.
__global__ __launch_bounds__(NT) void k_normal_asm(DV D) {
  GRID_LOOP(e, D.nnzC) {
    double v = 0.0;
    const int64_t p1 = D.cpp[e + 1];
    for (int64_t p = D.cpp[e]; p < p1; ++p) {
      const int2 ab = D.cprod[p];
      v += D.J.v[ab.x] * D.Dinv[D.J.ci[ab.x]] * D.J.v[ab.y];
    }
    D.Cx[e] = v;
  }
}

// MadNLP.solve!(kkt::NormalKKTSystem, w) (normalkkt.jl:196-219), after reduce_rhs! (done by k_rhs):
// r2 = A Sigma^{-1} r1 - r2 (one thread per row of A)
template <int G>
__global__ __launch_bounds__(NT) void k_normal_rhs(DV D) {
  GROUP_LOOP(i, D.m, G) {
    const int gl = threadIdx.x & (G - 1);
    double s = 0.0;
    for (int64_t q = D.J.rp[i] + gl; q < D.J.rp[i + 1]; q += G) {
      const int k = D.J.ci[q];
      s += D.J.v[q] * (D.d[k] / D.pr_diag[k]);
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, G);
    if (gl == 0) D.bufm[i] = s - D.d[D.n + i];
  }
}

// ... dy = C^{-1} r2 (LDL^T solve on bufm), then dx = Sigma^{-1} (r1 - A^T dy), wy = dy
template <int G>
__global__ __launch_bounds__(NT) void k_normal_back(DV D) {
  GROUP_LOOP(i, D.n + D.m, G) {
    if (i < D.n) {
      const double s = gdot<G>(D.JT, i, D.bufm);
      if ((threadIdx.x & (G - 1)) == 0) D.d[i] = (D.d[i] - s) / D.pr_diag[i];
    } else if ((threadIdx.x & (G - 1)) == 0) {
      D.d[i] = D.bufm[i - D.n];
    }
  }
}

enum { RHS_INIT_PRIMAL = 0, RHS_INIT_DUAL = 1, RHS_PRED = 2, RHS_CORR = 3, RHS_GONDZIO = 4 };

// set_*_rhs! (kernels.jl:1-58) fused with reduce_rhs! [EXT]: writes the unreduced p and the
// reduced right-hand side d[0:n+m] handed to the LDL^T solve.
// reset: 1 = start of an iteration's directions (max_res_ratio), 2 = also clear the NaN flag (redo)
// publish the device state to the host mirror: payload with system-scope stores, drained and
// released, then the counter (the host spins on the counter, MPCSolver::wait_state)
static_assert(sizeof(DevState) % 8 == 0 && sizeof(DevState) <= 64 * 8, "k_publish: one word per lane");
__device__ __forceinline__ void publish_state(const DevState* __restrict__ st, DevState* host, uint32_t* hseq,
                                              uint32_t seq, bool fresh = false) {  // called by one whole wave
  // fresh: the state was just stored by lane 0 of this wave: read it back from L2 (agent-scope loads)
  const int i = threadIdx.x;
  if (i < (int)(sizeof(DevState) / 8)) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(st) + i;
    const uint64_t v = fresh ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
    __hip_atomic_store(reinterpret_cast<uint64_t*>(host) + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (i == 0) __hip_atomic_store(hseq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// FIN_MU_PRED folded into the corrector's k_rhs: every block reduces k_mu's nb partials (slots 0..3)
// in the same fixed order, so all blocks agree on mu bit for bit; block 0 records it in the state
struct MuFold {
  int nb;                         // 0: mu from the state (FIN_MU_PRED ran)
  double cnt, has_ineq, mu_min;   // nlb + nub, has_inequalities, mu_min (FIN_MU_PRED's parameters)
};

// host != nullptr: wave 0 of block 0 first publishes the state (k_publish's work: the speculated
// predictor's k_rhs is the first launch after the factorisation, one launch less per iteration)
// t1 != nullptr: the factorisation before this launch ended (LinSolver::lazy_inertia)
__global__ __launch_bounds__(NT) void k_rhs(DV D, int mode, double mu_g, int reset, DevState* host, uint32_t* hseq,
                                            uint32_t seq, MuFold mf, LDLStatus* t1) {
  if (t1 && blockIdx.x == 0 && threadIdx.x == 0) ldl_status_end(t1);
  const int n = D.n, m = D.m, nlb = D.nlb;
  double mu = (mode == RHS_CORR) ? D.st->mu : mu_g;
  if (mf.nb > 0) {  // prediction_step! + update_barrier! (kernels.jl:176-220), as k_final(FIN_MU_PRED)
    __shared__ double shm[4][NT / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b = threadIdx.x; b < mf.nb; b += NT)
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += D.part[pidx(b, k)];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = wave_reduce<OP_SUM>(a[k]);
      if (lane == 0) shm[k][wv] = a[k];
    }
    __syncthreads();
    double r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r[k] = shm[k][0];
      for (int w = 1; w < NT / 64; ++w) r[k] += shm[k][w];
    }
    const double mu_aff = mf.cnt == 0 ? 0.0 : (r[2] + r[3]) / mf.cnt;
    const double mu_curr = mf.cnt == 0 ? 0.0 : (r[0] + r[1]) / mf.cnt;
    double sigma = 1.0;
    if (mf.has_ineq != 0.0) {
      const double q = mu_aff / mu_curr;
      sigma = fmin(fmax(q * q * q, 1e-6), 10.0);
    }
    mu = fmax(mf.mu_min, sigma * mu_curr);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      D.st->mu_aff = mu_aff;
      D.st->mu_curr = mu_curr;
      D.st->mu = mu;
    }
  }
  if (host && blockIdx.x == 0 && threadIdx.x < 64) publish_state(D.st, host, hseq, seq);
  if (reset && blockIdx.x == 0 && threadIdx.x == 0) {
    D.st->max_res_ratio = 0.0;
    if (reset == 2) D.st->nan_flag = 0;
  }
  // every operand of the row loaded first and unconditionally (clamped indices; the bound blocks'
  // entries right after the bound positions), the mode / bound tests applied afterwards: behind
  // `if (kl >= 0)` the loads were dependent round trips of their own
  const int nub = D.nub;
  GRID_LOOP(i, n + m) {
    if (i < n) {
      const int kl = D.lbpos[i], ku = D.ubpos[i];
      const double f = D.f[i], zl = D.zl[i], zu = D.zu[i], jl = D.jacl[i];
      const double x = D.x[i], xl = D.xl[i], xu = D.xu[i], di = D.d[i];
      const int kl0 = kl >= 0 ? kl : 0, ku0 = ku >= 0 ? ku : 0;
      const double ldg = D.l_diag[kl0], udg = D.u_diag[ku0], clb = D.corr_lb[kl0], cub = D.corr_ub[ku0];
      const double dzl = D.d[nlb > 0 ? n + m + kl0 : 0], dzu = D.d[nub > 0 ? n + m + nlb + ku0 : 0];
      double px;
      if (mode == RHS_INIT_PRIMAL)
        px = 0.0;
      else if (mode == RHS_INIT_DUAL)
        px = -f;
      else
        px = -f + zl - zu - jl;
      double dr = px;
      const bool full = mode >= RHS_PRED;
      if (kl >= 0) {
        double pz = 0.0;
        if (full) {
          pz = (xl - x) * zl;
          if (mode == RHS_CORR) {
            const double corr = di * dzl;
            D.corr_lb[kl] = corr;
            pz = pz + mu - corr;
          } else if (mode == RHS_GONDZIO) {
            pz = pz + mu - clb;
          }
        }
        D.p[n + m + kl] = pz;
        dr -= pz / ldg;
      }
      if (ku >= 0) {
        double pz = 0.0;
        if (full) {
          pz = (xu - x) * zu;
          if (mode == RHS_CORR) {
            const double corr = di * dzu;
            D.corr_ub[ku] = corr;
            pz = pz - mu - corr;
          } else if (mode == RHS_GONDZIO) {
            pz = pz - mu - cub;
          }
        }
        D.p[n + m + nlb + ku] = pz;
        dr -= pz / udg;
      }
      D.p[i] = px;
      D.d[i] = (D.kkt == KKT_K25) ? dr * D.sk[i] : dr;  // K2.5: right-hand side S r1
    } else {
      const double py = (mode == RHS_INIT_DUAL) ? 0.0 : -D.c[i - n];
      D.p[i] = py;
      D.d[i] = py;
    }
  }
}

// finish_aug_solve! [EXT] + residual w = p - K d (mul!/_kktmul! [EXT], linear_solver.jl:29-35)
enum { ALPHA_PRED = 0, ALPHA_CONSERVATIVE = 1, ALPHA_ADAPTIVE = 2, ALPHA_MEHROTRA = 3, ALPHA_GONDZIO = 4 };
// k_alpha may write its partials from slot PART_ALPHA (4 values, 4 indices) so that the residual's
// finaliser finalises both (one k_final less per direction).  Measured and reverted: the step test
// inside k_residual itself — its division-heavy tail then runs on one lane per SpMV lane group
// (k_residual 20.9 -> 32.2 us per launch, more than the two launches it saved).
constexpr int PART_ALPHA = 8;

__device__ __forceinline__ double alpha_tau(const DV& D, int mode, double tau_param) {
  double tau = 1.0;
  if (mode == ALPHA_CONSERVATIVE || mode == ALPHA_GONDZIO) tau = tau_param;
  if (mode == ALPHA_ADAPTIVE) tau = fmax(1.0 - D.st->mu, tau_param);
  return tau;
}

// block argmin of (v[k], ix[k]), k < 4, into part slots base + k (values) and base + 4 + k (indices)
__device__ void block_argmin4(const double (&v)[4], const int (&ix)[4], double* part, int base, int bid) {
  __shared__ double sv[4][NT / 64];
  __shared__ int si[4][NT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double a = v[k];
    int b = ix[k];
    wave_argmin(a, b);
    if (lane == 0) {
      sv[k][wv] = a;
      si[k][wv] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    double a = sv[k][0];
    int b = si[k][0];
    for (int w = 1; w < NT / 64; ++w) amin_upd(a, b, sv[k][w], si[k][w]);
    part[pidx(bid, base + k)] = a;
    part[pidx(bid, base + 4 + k)] = (double)b;
  }
}

template <bool FROM_P>
__device__ void alpha_body(const DV& D, int mode, double tau_param, int base, int bid, int nblk);

// nres < gridDim.x: blocks [nres, gridDim.x) run the step test of mode amode (alpha_body, partials
// from slot PART_ALPHA) beside the nres residual blocks — one launch for both
template <int G>
__global__ __launch_bounds__(NT) void k_residual(DV D, double dw, double dc, int nres, int amode, double atau) {
  const int n = D.n, m = D.m, nlb = D.nlb;
  if ((int)blockIdx.x >= nres) {
    alpha_body<true>(D, amode, atau, PART_ALPHA, (int)blockIdx.x - nres, (int)gridDim.x - nres);
    return;
  }
  const bool lead = (threadIdx.x & (G - 1)) == 0;
  double wmax = 0.0, pmax = 0.0, dxmax = 0.0;
  GROUP_LOOP_B(i, n + m, G, (int)blockIdx.x, nres) {
    // the row's own entries and its bound blocks do not depend on the dot products: loaded first,
    // unconditionally (clamped indices; every lane of the group, one cache line), so their latency
    // overlaps the gathers — behind `if (!lead)` / `if (kl >= 0)` they were two more round trips
    const double dxi = D.d[i], pi = D.p[i];
    const int kl = (i < n) ? D.lbpos[i] : -1, ku = (i < n) ? D.ubpos[i] : -1;
    const int kl0 = kl >= 0 ? kl : 0, ku0 = ku >= 0 ? ku : 0;
    const double pl = D.p[kl >= 0 ? n + m + kl : i], llo = D.l_lower[kl0], ldi = D.l_diag[kl0];
    const double pu = D.p[ku >= 0 ? n + m + nlb + ku : i], ulo = D.u_lower[ku0], udi = D.u_diag[ku0];
    if (i < n) {
      double hd, jd;
      gdot2<G>(D.H, i, D.d, D.JT, i, D.d + n, hd, jd);
      const double hj = hd + jd;
      if (!lead) continue;
      const double dx = dxi;
      double kv = hj + dw * dx;
      if (kl >= 0) {
        const double dzl = (-pl + llo * dx) / ldi;
        D.d[n + m + kl] = dzl;
        kv -= dzl;
        const double wl = pl - (dx * llo - dzl * ldi);
        wmax = nmax(wmax, fabs(wl));
        pmax = nmax(pmax, fabs(pl));
      }
      if (ku >= 0) {
        const double dzu = (pu - ulo * dx) / udi;
        D.d[n + m + nlb + ku] = dzu;
        kv += dzu;
        const double wu = pu - (dx * ulo + dzu * udi);
        wmax = nmax(wmax, fabs(wu));
        pmax = nmax(pmax, fabs(pu));
      }
      wmax = nmax(wmax, fabs(pi - kv));
      pmax = nmax(pmax, fabs(pi));
      dxmax = nmax(dxmax, fabs(dx));
    } else {
      const double jd = gdot<G>(D.J, i - n, D.d);
      if (!lead) continue;
      const double kv = jd + dc * dxi;
      wmax = nmax(wmax, fabs(pi - kv));
      pmax = nmax(pmax, fabs(pi));
    }
  }
  double v[3] = {wmax, pmax, dxmax};
  const int ops[3] = {OP_MAX, OP_MAX, OP_MAX};
  block_partials<3>(v, ops, D.part, 0, (int)blockIdx.x);
}

// get_alpha_max_primal / get_alpha_max_dual (kernels.jl:226-272): min-ratio with argmin
// from_p: dz formed here from the reduced rhs p and dx, exactly as k_residual's finish_aug_solve
// forms it (the step-test blocks of a k_residual launch run beside the residual blocks that store it).
// The reduced-rhs operands (p, l_lower, l_diag, u_lower, u_diag) exist only in the FROM_P instance:
// madipm_update_step's standalone DV leaves them null.
template <bool FROM_P>
__device__ void alpha_body(const DV& D, int mode, double tau_param, int base, int bid, int nblk) {
  constexpr bool from_p = FROM_P;
  const int n = D.n, m = D.m, nlb = D.nlb, nub = D.nub;
  const double tau = alpha_tau(D, mode, tau_param);
  double v[4] = {INF, INF, INF, INF};
  int ix[4] = {-1, -1, -1, -1};
  // every operand loaded unconditionally (clamped indices) right after the bound's index, the tests
  // applied as selects: behind `if (dx < 0)` etc. the loads were dependent round trips of their own
  GRID_LOOP_B(t, (nlb > nub ? nlb : nub), bid, nblk) {
    const int tl = t < nlb ? (int)t : 0, tu = t < nub ? (int)t : 0;
    const int il = nlb > 0 ? D.ind_lb[tl] : 0, iu = nub > 0 ? D.ind_ub[tu] : 0;
    const double dxl = D.d[il], xl_x = D.x[il], xl_l = D.xl[il], zl = D.zl[il];
    const double pl = from_p ? D.p[nlb > 0 ? n + m + tl : 0] : D.d[nlb > 0 ? n + m + tl : 0];
    const double lo = from_p ? D.l_lower[tl] : 0.0, ldg = from_p ? D.l_diag[tl] : 1.0;
    const double dxu = D.d[iu], xu_x = D.x[iu], xu_u = D.xu[iu], zu = D.zu[iu];
    const int qu = nub > 0 ? n + m + nlb + tu : 0;  // in range
    const double pu = from_p ? D.p[qu] : D.d[qu];
    const double uo = from_p ? D.u_lower[tu] : 0.0, udg = from_p ? D.u_diag[tu] : 1.0;
    if (t < nlb) {
      const double dx = dxl;
      if (dx < 0) amin_upd(v[0], ix[0], (-xl_x + xl_l) * tau / dx, (int)t);
      const double dz = from_p ? (-pl + lo * dx) / ldg : pl;
      if (dz < 0) amin_upd(v[2], ix[2], (-zl) * tau / dz, (int)t);
    }
    if (t < nub) {
      const double dx = dxu;
      if (dx > 0) amin_upd(v[1], ix[1], (-xu_x + xu_u) * tau / dx, (int)t);
      const double dz = from_p ? (pu - uo * dx) / udg : pu;
      if (dz < 0 && zu + dz < 0) amin_upd(v[3], ix[3], (-zu) * tau / dz, (int)t);
    }
  }
  block_argmin4(v, ix, D.part, base, bid);
}

__global__ __launch_bounds__(NT) void k_alpha(DV D, int mode, double tau_param, int base) {
  alpha_body<false>(D, mode, tau_param, base, blockIdx.x, gridDim.x);
}

enum { MU_PRED = 0, MU_FULL = 1, MU_GONDZIO = 2 };

// complementarity sums (kernels.jl:155-208); step lengths from the device state (use_state) or args
__global__ __launch_bounds__(NT) void k_mu(DV D, int use_state, double ap_arg, double ad_arg) {
  const int n = D.n, m = D.m, nlb = D.nlb, nub = D.nub;
  const double ap = use_state ? D.st->alpha_aff_p : ap_arg;
  const double ad = use_state ? D.st->alpha_aff_d : ad_arg;
  double cl = 0, cu = 0, al = 0, au = 0;
  GRID_LOOP(t, (nlb > nub ? nlb : nub)) {
    if (t < nlb) {
      const int i = D.ind_lb[t];
      const double x = D.x[i], xl = D.xl[i], zl = D.zl[i];
      cl += (x - xl) * zl;
      al += ((x + ap * D.d[i]) - xl) * (zl + ad * D.d[n + m + t]);
    }
    if (t < nub) {
      const int i = D.ind_ub[t];
      const double x = D.x[i], xu = D.xu[i], zu = D.zu[i];
      cu += (xu - x) * zu;
      au += (xu - (x + ap * D.d[i])) * (zu + ad * D.d[n + m + nlb + t]);
    }
  }
  double v[4] = {cl, cu, al, au};
  const int ops[4] = {OP_SUM, OP_SUM, OP_SUM, OP_SUM};
  block_partials<4>(v, ops, D.part);
}

// apply_step! + adjust_boundary! [EXT] (solver.jl:308-317)
__global__ __launch_bounds__(NT) void k_apply(DV D) {
  if (D.st->nan_flag) return;  // SolveException raised in this iteration's directions: no step
  const int n = D.n, m = D.m, nlb = D.nlb;
  const double ap = D.st->alpha_p, ad = D.st->alpha_d, mu = D.st->mu;
  const double eps = 2.220446049250313e-16;
  const double c1 = eps * mu, c2 = 1.8189894035458617e-12;  // eps^(3/4)
  GRID_LOOP(i, n + m) {
    if (i < n) {
      const double x = D.x[i] + ap * D.d[i];
      D.x[i] = x;
      const int kl = D.lbpos[i], ku = D.ubpos[i];
      if (kl >= 0) {
        D.zl[i] += ad * D.d[n + m + kl];
        const double xl = D.xl[i];
        if (x - xl < c1) D.xl[i] = xl - c2 * fmax(1.0, fabs(x));
      }
      if (ku >= 0) {
        D.zu[i] += ad * D.d[n + m + nlb + ku];
        const double xu = D.xu[i];
        if (xu - x < c1) D.xu[i] = xu + c2 * fmax(1.0, fabs(x));
      }
    } else {
      D.y[i - n] += ad * D.d[i];
    }
  }
}

// evaluate_model! (solver.jl:319-326): obj, grad f = Hx + c, cons c = Jx - rhs, jacl = J^T y
template <int G>
__global__ __launch_bounds__(NT) void k_eval(DV D, int slot) {
  const int n = D.n;
  const bool lead = (threadIdx.x & (G - 1)) == 0;
  double op = 0.0;
  GROUP_LOOP(i, n + D.m, G) {
    if (i < n) {
      double hx, jy;
      gdot2<G>(D.H, i, D.x, D.JT, i, D.y, hx, jy);
      if (!lead) continue;
      const double x = D.x[i];
      const double g = D.cs[i] + D.gfix[i];
      D.f[i] = D.fixed[i] ? 0.0 : hx + g;
      D.jacl[i] = jy;
      op += x * g + 0.5 * x * hx;
    } else {
      const int64_t j = i - n;
      const double jx = gdot<G>(D.J, j, D.x);
      if (lead) D.c[j] = jx - D.rhs[j] + D.cfix[j];
    }
  }
  double v[1] = {op};
  const int ops[1] = {OP_SUM};
  block_partials<1>(v, ops, D.part, slot);
}

// jtprod!(jacl, kkt, y)
__global__ __launch_bounds__(NT) void k_jtprod(DV D) {
  GRID_LOOP(i, D.n) D.jacl[i] = csr_dot(D.JT, (int)i, D.y);
}

// update_termination_criteria! pieces (solver.jl:194-204; dual_objective kernels.jl:408-417;
// get_optimality_gap kernels.jl:419-430; get_inf_pr/get_inf_du [EXT])
// diag != 0: also k_diag's work for the next factorisation (same grid, same iterate reads; the
// regularisation is decided on the host before this launch), one launch less per iteration
__global__ __launch_bounds__(NT) void k_term(DV D, int diag, double dw, double dc) {
  const int n = D.n;
  double du = 0, gap = 0, pr = 0, sy = 0, sl = 0, su = 0;
  GRID_LOOP(i, n + D.m) {
    if (diag) diag_entry(D, i, dw, dc);
    if (i < n) {
      du = nmax(du, fabs(D.f[i] - D.zl[i] + D.zu[i] + D.jacl[i]));
      const int kl = D.lbpos[i], ku = D.ubpos[i];
      if (kl >= 0) {
        gap = nmax(gap, fabs((D.x[i] - D.xl[i]) * D.zl[i]));
        sl += D.zl[i] * D.xl[i];
      }
      if (ku >= 0) {
        gap = nmax(gap, fabs((D.xu[i] - D.x[i]) * D.zu[i]));
        su += D.zu[i] * D.xu[i];
      }
    } else {
      const int j = (int)(i - n);
      pr = nmax(pr, fabs(D.c[j]));
      sy += D.y[j] * D.rhs[j];
    }
  }
  double v[6] = {du, gap, pr, sy, sl, su};
  const int ops[6] = {OP_MAX, OP_MAX, OP_MAX, OP_SUM, OP_SUM, OP_SUM};
  block_partials<6>(v, ops, D.part);
}

// init_starting_point! Step 3 (solver.jl:37-78): z from r = A^T y + f, then min-reductions
__global__ __launch_bounds__(NT) void k_zinit(DV D) {
  const int n = D.n;
  double mxl = 0, mxu = 0, mzl = 0, mzu = 0;  // minimum(...; init=0.0)
  GRID_LOOP(i, n) {
    const double res = csr_dot(D.JT, (int)i, D.y) + D.f[i];
    const double l = D.xl[i], u = D.xu[i];
    const bool fl = isfinite(l), fu = isfinite(u);
    const double zl = (fl && fu) ? 0.5 * res : (fl ? res : D.zl[i]);
    const double zu = (fl && fu) ? -0.5 * res : (fu ? -res : D.zu[i]);
    D.zl[i] = zl;
    D.zu[i] = zu;
    const double x = D.x[i];
    if (D.lbpos[i] >= 0) {
      mxl = fmin(mxl, x - l);
      mzl = fmin(mzl, zl);
    }
    if (D.ubpos[i] >= 0) {
      mxu = fmin(mxu, u - x);
      mzu = fmin(mzu, zu);
    }
  }
  double v[4] = {mxl, mxu, mzl, mzu};
  const int ops[4] = {OP_MIN, OP_MIN, OP_MIN, OP_MIN};
  block_partials<4>(v, ops, D.part);
}

// solver.jl:80-99: first shift, then the sums defining mu, delta_x2, delta_s2
__global__ __launch_bounds__(NT) void k_zshift1(DV D) {
  const int n = D.n;
  const double dx = D.st->delta_x, ds = D.st->delta_s;
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  GRID_LOOP(i, n) {
    const bool lb = D.lbpos[i] >= 0, ub = D.ubpos[i] >= 0;
    double x = D.x[i];
    if (lb) x = x + dx;
    if (ub) x = x - dx;
    D.x[i] = x;
    if (lb) {
      const double zl = D.zl[i] + 1.0 + ds;
      D.zl[i] = zl;
      const double l = D.xl[i];
      s[0] += x * zl;
      s[1] += l * zl;
      s[4] += zl;
      s[6] += x - l;
    }
    if (ub) {
      const double zu = D.zu[i] + 1.0 + ds;
      D.zu[i] = zu;
      const double u = D.xu[i];
      s[2] += u * zu;
      s[3] += x * zu;
      s[5] += zu;
      s[7] += u - x;
    }
  }
  const int ops[8] = {OP_SUM, OP_SUM, OP_SUM, OP_SUM, OP_SUM, OP_SUM, OP_SUM, OP_SUM};
  block_partials<8>(s, ops, D.part);
}

// solver.jl:96-123: second shift, Ipopt projection, interior assertions (violation count)
__global__ __launch_bounds__(NT) void k_zshift2(DV D, double kappa) {
  const int n = D.n;
  const double dx2 = D.st->delta_x2, ds2 = D.st->delta_s2;
  double viol = 0;
  GRID_LOOP(i, n) {
    const bool lb = D.lbpos[i] >= 0, ub = D.ubpos[i] >= 0;
    double x = D.x[i];
    if (lb) x = x + dx2;
    if (ub) x = x - dx2;
    if (lb) D.zl[i] = D.zl[i] + ds2;
    if (ub) D.zu[i] = D.zu[i] + ds2;
    const double l = D.xl[i], u = D.xu[i];
    if (x < l) {
      x = l + fmin(kappa * fmax(1.0, l), kappa * (u - l));
    } else if (u < x) {
      x = u - fmin(kappa * fmax(1.0, u), kappa * (u - l));
    }
    D.x[i] = x;
    if (lb && !(D.zl[i] > 0.0 && x > l)) viol += 1;
    if (ub && !(D.zu[i] > 0.0 && x < u)) viol += 1;
  }
  double v[1] = {viol};
  const int ops[1] = {OP_SUM};
  block_partials<1>(v, ops, D.part);
}

__global__ void k_set_mu(DevState* st, double mu) {
  st->mu = mu;
  st->alpha_p = st->alpha_d = 0.0;
  st->nan_flag = 0;
  st->max_res_ratio = 0.0;
  st->dx_inf = 0.0;
}

enum {
  FIN_RESID = 0,
  FIN_ALPHA = 1,
  FIN_MU_PRED = 2,
  FIN_MU_FULL = 3,
  FIN_EVAL = 4,
  FIN_TERM = 5,
  FIN_ZINIT = 6,
  FIN_ZSHIFT1 = 7,
  FIN_ZSHIFT2 = 8,
  FIN_MU_GONDZIO = 9
};

struct FinParams {
  int nb;          // number of partial blocks
  int alpha_mode;  // for FIN_ALPHA (and FIN_RESID with nb_alpha > 0)
  double a, b, c;  // kind-specific parameters
  int nb_alpha;    // FIN_RESID: > 0 -> also finalise k_alpha's nb_alpha partials (slots PART_ALPHA..)
  int nb_eval;     // FIN_TERM: > 0 -> also finalise evaluate_model!'s objective (k_eval's nb_eval
                   // partials in slot PART_EVAL, the previous iteration's; P.c = its constant)
  LDLStatus* rs;   // != nullptr: a factorisation follows this launch (LinSolver::ext_reset)
  int64_t* dbg = nullptr;  // diagnostics (MADIPM_FINAL_DEBUG): thread 0's wall clock at entry / reduced / end
  DevState* host = nullptr;  // != nullptr: wave 0 of the last workgroup publishes the state (sequence seq)
  uint32_t* hseq = nullptr;
  uint32_t seq = 0;
};
constexpr int PART_EVAL = 6;

// k_final combines the producers' block partials (nb <= MAXB per slot) in two levels inside ONE launch:
// FG workgroups of FT threads, thread t of workgroup g owning block g FT + t; each workgroup reduces its
// FT blocks (wave shuffles, then wave 0 before wave 1) and stores one partial per value write-through
// (sc1), and the last workgroup to take a ticket combines the FG partials in workgroup order and runs
// the scalar logic.  Fixed combine order: bitwise reproducible.  One workgroup reading every partial was
// bound by a single CU's memory parallelism (~1 us per 16-KB slot, 11 us for the residual + step test:
// MADIPM_FINAL_DEBUG stamps); spread over FG CUs each reads ~1/FG of it in one round trip.
// (Finalising inside the producing kernel instead — block 0 polling per-block flags, or a ticket —
// measured slower on ex10: the in-launch hand-off costs more than this launch.)
constexpr int FG = 16, FT = 128;  // workgroups, threads per workgroup (one partial block per thread)
static_assert(MAXB == FG * FT, "k_final: one partial block per thread");
constexpr int NL2 = 24;  // level-2 value slots: 8 generic + 4 alpha values + 4 alpha indices + eval

__device__ __forceinline__ double ld_sc1(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// the step test's result (fraction-to-boundary ratios and their argmins) into the state
__device__ void fin_alpha_store(const DV& D, const FinParams& P, double (&a)[4], int (&ii)[4]) {
  DevState* st = D.st;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // mapreduce init (1.0, 0) is the fold's first element: an element whose ratio is exactly 1.0
    // comes later and replaces it (the index is the element's); larger ratios keep (1.0, init)
    if (!(a[k] <= 1.0)) {
      a[k] = 1.0;
      ii[k] = -1;
    }
  }
  st->a_xl = a[0];
  st->a_xu = a[1];
  st->a_zl = a[2];
  st->a_zu = a[3];
  st->i_xl = ii[0];
  st->i_xu = ii[1];
  st->i_zl = ii[2];
  st->i_zu = ii[3];
  const double ap = fmin(a[0], a[1]), ad = fmin(a[2], a[3]);
  if (P.alpha_mode == ALPHA_PRED) {
    st->alpha_aff_p = ap;
    st->alpha_aff_d = ad;
  } else if (P.alpha_mode == ALPHA_CONSERVATIVE || P.alpha_mode == ALPHA_ADAPTIVE) {
    st->alpha_p = ap;
    st->alpha_d = ad;
  } else {  // MEHROTRA / GONDZIO: keep in the aff slots for the follow-up pass
    st->alpha_aff_p = ap;
    st->alpha_aff_d = ad;
  }
}

// value slots and combine operation of each finaliser kind (compile time: the k_final instance's
// combines are branch-free)
constexpr int fin_nv(int kind) {
  return kind == FIN_RESID ? 3
         : kind == FIN_TERM ? 6
         : (kind == FIN_MU_PRED || kind == FIN_MU_FULL || kind == FIN_MU_GONDZIO || kind == FIN_ZINIT) ? 4
         : kind == FIN_ZSHIFT1 ? 8
         : (kind == FIN_EVAL || kind == FIN_ZSHIFT2) ? 1
                                                     : 0;
}
__host__ __device__ constexpr int fin_op(int kind, int k) {
  return (kind == FIN_RESID || (kind == FIN_TERM && k < 3)) ? OP_MAX : (kind == FIN_ZINIT ? OP_MIN : OP_SUM);
}

// the scalar logic of each finaliser kind on the reduced values res[] (thread 0 of the last workgroup)
__device__ void fin_tail(const DV& D, int kind, const FinParams& P, const double* res) {
  DevState* st = D.st;
  switch (kind) {
    case FIN_RESID: {
      const double ratio = res[0] / fmax(1.0, res[1]);  // linear_solver.jl:35
      st->res_ratio = ratio;
      st->max_res_ratio = nmax(st->max_res_ratio, ratio);
      st->dx_inf = res[2];
      if (ratio != ratio || (P.a > 0 && ratio > P.a)) st->nan_flag = 1;  // SolveException
      break;
    }
    case FIN_MU_PRED: {  // prediction_step! + update_barrier! (kernels.jl:176-220)
      const double cnt = P.a;  // nlb + nub
      const double mu_aff = cnt == 0 ? 0.0 : (res[2] + res[3]) / cnt;
      const double mu_curr = cnt == 0 ? 0.0 : (res[0] + res[1]) / cnt;
      double sigma = 1.0;
      if (P.b != 0.0) {  // has_inequalities
        const double q = mu_aff / mu_curr;
        sigma = fmin(fmax(q * q * q, 1e-6), 10.0);
      }
      st->mu_aff = mu_aff;
      st->mu_curr = mu_curr;
      st->mu = fmax(P.c, sigma * mu_curr);
      break;
    }
    case FIN_MU_FULL: {  // MehrotraAdaptiveStep (kernels.jl:309-358)
      const double cnt = P.a, gamma_f = P.b;
      const double gamma_a = 1.0 / (1.0 - gamma_f);
      double mu_full = cnt == 0 ? 0.0 : (res[2] + res[3]) / cnt;
      mu_full /= gamma_a;
      const double max_p = st->alpha_aff_p, max_d = st->alpha_aff_d;
      const int n = D.n, m = D.m, nlb = D.nlb;
      double ap = 1.0, ad = 1.0;
      if (max_p < 1.0) {
        if (st->a_xl <= st->a_xu) {
          const int k = st->i_xl, i = D.ind_lb[k];
          const double tmp = mu_full / (D.zl[i] + max_d * D.d[n + m + k]);
          ap = (D.x[i] - D.xl[i] - tmp) / (-D.d[i]);
        } else {
          const int k = st->i_xu, i = D.ind_ub[k];
          const double tmp = mu_full / (D.zu[i] + max_d * D.d[n + m + nlb + k]);
          ap = (D.xu[i] - D.x[i] - tmp) / (D.d[i]);
        }
      }
      if (max_d < 1.0) {
        if (st->a_zl <= st->a_zu) {
          const int k = st->i_zl, i = D.ind_lb[k];
          const double tmp = mu_full / (D.x[i] + max_p * D.d[i] - D.xl[i]);
          ad = -(D.zl[i] - tmp) / D.d[n + m + k];
        } else {
          const int k = st->i_zu, i = D.ind_ub[k];
          const double tmp = mu_full / (D.xu[i] - D.x[i] - max_p * D.d[i]);
          ad = -(D.zu[i] - tmp) / D.d[n + m + nlb + k];
        }
      }
      st->alpha_p = fmax(ap, gamma_f * max_p);
      st->alpha_d = fmax(ad, gamma_f * max_d);
      break;
    }
    case FIN_MU_GONDZIO: {
      const double cnt = P.a;
      st->mu_aff = cnt == 0 ? 0.0 : (res[2] + res[3]) / cnt;
      break;
    }
    case FIN_EVAL: st->obj_val = P.a + res[0]; break;
    case FIN_TERM:
      st->inf_du_raw = res[0];
      st->inf_compl_raw = res[1];
      st->inf_pr_raw = res[2];
      st->dobj = -res[3] + res[4] - res[5];
      break;
    case FIN_ZINIT:
      st->delta_x = fmax(fmax(0.0, -1.5 * res[0]), -1.5 * res[1]);
      st->delta_s = fmax(fmax(0.0, -1.5 * res[2]), -1.5 * res[3]);
      break;
    case FIN_ZSHIFT1: {
      double mu = 0.0;
      if (D.nlb > 0) mu += res[0] - res[1];
      if (D.nub > 0) mu += res[2] - res[3];
      st->delta_x2 = mu / (2 * (res[4] + res[5]));
      st->delta_s2 = mu / (2 * (res[6] + res[7]));
      break;
    }
    case FIN_ZSHIFT2: st->init_viol = res[0]; break;
  }
}

// Instantiated per (finaliser kind KIND, fused step test AL, fused objective EV) so that a thread holds
// exactly the partials of its launch and every combine is a compile-time operation (launch_final
// picks the instance).  Level-2 partials and the
// ticket live past the NPART x MAXB partials (part_): L2 = part + NPART MAXB, NL2 x FG doubles, then the
// ticket counter (reset by the last workgroup).
// NG == 1 (producers of at most FT1 blocks, MPCSolver::maxb_): ONE workgroup of FT1 threads reduces
// every partial in one round trip — no level-2 partials, no ticket.
template <int KIND, bool AL, bool EV, int NG = FG, int NTH = FT>
__global__ __launch_bounds__(NTH) void k_final(DV D, int kind, FinParams P) {
  constexpr int NV = fin_nv(KIND);
  __shared__ double res[NL2];
  __shared__ int s_last;
  DevState* st = D.st;
  double* L2 = D.part + NPART * MAXB;
  int32_t* ticket = reinterpret_cast<int32_t*>(L2 + NL2 * FG);
  const int g = blockIdx.x, b = g * NTH + threadIdx.x;
  if (P.dbg && threadIdx.x == 0 && g == 0) {
    P.dbg[0] = (int64_t)wall_clock64();
    P.dbg[3] = kind | (AL && NV > 0 ? 16 : 0) | (EV ? 32 : 0);
  }
  // every load first (unconditional: each slot holds MAXB partials, stale past nb), then the pins
  // (waits) and the selections — a predicated load compiles to a branch with a wait inside
  constexpr int NA = AL ? 8 : 0;
  double q[NV > 0 ? NV : 1], aq[AL ? 8 : 1], eq = 0.0;
#pragma unroll
  for (int k = 0; k < NV; ++k) q[k] = D.part[pidx(b, k)];
#pragma unroll
  for (int k = 0; k < NA; ++k) aq[k] = D.part[pidx(b, (NV > 0 ? PART_ALPHA : 0) + k)];
  if (EV) eq = D.part[pidx(b, PART_EVAL)];
#pragma unroll
  for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(q[k]));
#pragma unroll
  for (int k = 0; k < NA; ++k) asm volatile("" : "+v"(aq[k]));
  if (EV) asm volatile("" : "+v"(eq));
  if (P.dbg && threadIdx.x == 0 && g == 0) P.dbg[4] = (int64_t)wall_clock64();  // loads returned
  // level 1: this workgroup's blocks — every value's shuffle tree in lockstep (one latency chain for all
  // of them, not one per value), then the waves in order
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double w1[NV > 0 ? NV : 1], av[4];
  int ai[4];
#pragma unroll
  for (int k = 0; k < NV; ++k) w1[k] = b < P.nb ? q[k] : 0.0;
  const int nba = NV > 0 ? P.nb_alpha : P.nb;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    av[k] = (AL && b < nba) ? aq[k] : INF;
    ai[k] = (AL && b < nba) ? (int)aq[AL ? 4 + k : 0] : -1;
  }
  double e1 = (EV && b < P.nb_eval) ? eq : 0.0;
  // every value's tree in lockstep (one latency chain for all of them), the __shfl_down pairing
  auto stage = [&](auto otag) {
    constexpr int O = decltype(otag)::value;
#pragma unroll
    for (int k = 0; k < NV; ++k) w1[k] = comb(w1[k], lane_down<O>(w1[k]), fin_op(KIND, k));
    if (AL)
#pragma unroll
      for (int k = 0; k < 4; ++k) argmin_step<O>(av[k], ai[k]);
    if (EV) e1 += lane_down<O>(e1);
  };
  stage(std::integral_constant<int, 32>{});
  stage(std::integral_constant<int, 16>{});
  stage(std::integral_constant<int, 8>{});
  stage(std::integral_constant<int, 4>{});
  stage(std::integral_constant<int, 2>{});
  stage(std::integral_constant<int, 1>{});
  __shared__ double shv[NL2][NTH / 64];
  __shared__ int shx[4][NTH / 64];
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) shv[k][wv] = w1[k];
    if (AL)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        shv[8 + k][wv] = av[k];
        shx[k][wv] = ai[k];
      }
    if (EV) shv[16][wv] = e1;
  }
  __syncthreads();
  if constexpr (NG == 1) {  // the waves in order, straight into res[]
    const int t = threadIdx.x;
    if (t < NV) {
      double a = shv[t][0];
#pragma unroll
      for (int w = 1; w < NTH / 64; ++w) a = comb(a, shv[t][w], fin_op(KIND, t));
      res[t] = a;
    } else if (AL && t >= 8 && t < 12) {
      double a = shv[t][0];
      int ix = shx[t - 8][0];
#pragma unroll
      for (int w = 1; w < NTH / 64; ++w) amin_upd(a, ix, shv[t][w], shx[t - 8][w]);
      res[t] = a;
      res[t + 4] = (double)ix;
    } else if (EV && t == 16) {
      double a = shv[16][0];
#pragma unroll
      for (int w = 1; w < NTH / 64; ++w) a += shv[16][w];
      res[16] = a;
    }
    if (P.dbg && t == 0) P.dbg[5] = P.dbg[6] = (int64_t)wall_clock64();
    __syncthreads();
  } else {
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double a = shv[k][0];
#pragma unroll
      for (int w = 1; w < FT / 64; ++w) a = comb(a, shv[k][w], fin_op(KIND, k));
      st_sc1(L2 + k * FG + g, a);
    }
    if (AL)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        double a = shv[8 + k][0];
        int ix = shx[k][0];
#pragma unroll
        for (int w = 1; w < FT / 64; ++w) amin_upd(a, ix, shv[8 + k][w], shx[k][w]);
        st_sc1(L2 + (8 + k) * FG + g, a);
        st_sc1(L2 + (12 + k) * FG + g, (double)ix);
      }
    if (EV) {
      double a = shv[16][0];
#pragma unroll
      for (int w = 1; w < FT / 64; ++w) a += shv[16][w];
      st_sc1(L2 + 16 * FG + g, a);
    }
    if (P.dbg && g == 0) P.dbg[5] = (int64_t)wall_clock64();  // level 1 reduced
    // release: this workgroup's level-2 partials are visible before its ticket; the last
    // workgroup's acquire (below) pairs with every earlier release on the ticket's RMW chain
    s_last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == FG - 1;
    if (P.dbg && s_last) P.dbg[6] = (int64_t)wall_clock64();  // last ticket taken
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every thread of the last workgroup: see the partials
  // level 2 (last workgroup): every level-2 partial loaded at once (one per thread, sc1), then thread k
  // combines value slot k over the workgroups in order
  const int t = threadIdx.x;
  __shared__ double l2s[NL2 * FG];
  constexpr int NUSE = AL ? (EV ? 17 : 16) : (EV ? 17 : NV);  // slots in use: 0..NV-1, 8..15 (alpha), 16 (eval)
  static_assert(NUSE * FG <= 3 * FT, "level 2: at most three loads per thread");
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int e = t + h * FT;
    if (e < NUSE * FG) l2s[e] = ld_sc1(L2 + e);
  }
  __syncthreads();
  if (t < NV) {
    double a = l2s[t * FG];
#pragma unroll
    for (int w = 1; w < FG; ++w) a = comb(a, l2s[t * FG + w], fin_op(KIND, t));
    res[t] = a;
  } else if (AL && t >= 8 && t < 12) {
    double a = l2s[t * FG];
    int ix = (int)l2s[(t + 4) * FG];
#pragma unroll
    for (int w = 1; w < FG; ++w) amin_upd(a, ix, l2s[t * FG + w], (int)l2s[(t + 4) * FG + w]);
    res[t] = a;
    res[t + 4] = (double)ix;
  } else if (EV && t == 16) {
    double a = l2s[16 * FG];
#pragma unroll
    for (int w = 1; w < FG; ++w) a += l2s[16 * FG + w];
    res[16] = a;
  }
  __syncthreads();
  }  // NG > 1
  const int t = threadIdx.x;
  if (t >= 64) return;
  if (t == 0) {
    if (NG > 1) *ticket = 0;  // every workgroup has taken its ticket: reset for the next launch
    if (P.dbg) P.dbg[1] = (int64_t)wall_clock64();
    if (AL) {
      double a[4];
      int ii[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = res[8 + k];
        ii[k] = (int)res[12 + k];
      }
      fin_alpha_store(D, P, a, ii);
    }
    if (EV) st->obj_val = P.c + res[16];  // FIN_TERM: the previous iteration's FIN_EVAL, deferred here
    if (NV > 0) {
      if (P.rs) ldl_status_start(P.rs);
      fin_tail(D, kind, P, res);
    }
    if (P.dbg) {
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      P.dbg[2] = (int64_t)wall_clock64();
    }
  }
  if (P.host) {  // publish the state right here (the termination test's, before the factorisation):
    // lane 0's state stores drained to L2, the wave reads them back past L1 and publishes
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    publish_state(st, P.host, P.hseq, P.seq, true);
  }
}

// the k_final instance of a finaliser launch (slots, fused step test, fused objective)
constexpr int FT1 = 1024;  // the single-workgroup finaliser's threads (one partial block each)
void launch_final(const DV& D, int kind, const FinParams& P, hipStream_t s) {
  // one workgroup when every producer launch had at most FT1 blocks (maxb_ <= FT1), else FG of them
  const bool one = std::max(P.nb, std::max(P.nb_alpha, P.nb_eval)) <= FT1;
#define LF(K, AL, EV)                                                 \
  do {                                                                \
    if (one)                                                          \
      k_final<K, AL, EV, 1, FT1><<<1, FT1, 0, s>>>(D, kind, P);       \
    else                                                              \
      k_final<K, AL, EV><<<FG, FT, 0, s>>>(D, kind, P);               \
  } while (0)
  switch (kind) {
    case FIN_ALPHA: LF(FIN_ALPHA, true, false); break;
    case FIN_RESID:
      if (P.nb_alpha > 0)
        LF(FIN_RESID, true, false);
      else
        LF(FIN_RESID, false, false);
      break;
    case FIN_MU_PRED: LF(FIN_MU_PRED, false, false); break;
    case FIN_MU_FULL: LF(FIN_MU_FULL, false, false); break;
    case FIN_MU_GONDZIO: LF(FIN_MU_GONDZIO, false, false); break;
    case FIN_ZINIT: LF(FIN_ZINIT, false, false); break;
    case FIN_EVAL: LF(FIN_EVAL, false, false); break;
    case FIN_ZSHIFT2: LF(FIN_ZSHIFT2, false, false); break;
    case FIN_TERM:
      if (P.nb_eval > 0)
        LF(FIN_TERM, false, true);
      else
        LF(FIN_TERM, false, false);
      break;
    case FIN_ZSHIFT1: LF(FIN_ZSHIFT1, false, false); break;
    default: throw Error("k_final: unknown finaliser kind", -2);
  }
#undef LF
}

__global__ void k_publish(const DevState* __restrict__ st, DevState* host, uint32_t* hseq, uint32_t seq) {
  publish_state(st, host, hseq, seq);
}

__global__ void k_copy(double* __restrict__ dst, const double* __restrict__ src, int64_t n) {
  GRID_LOOP(i, n) dst[i] = src[i];
}
// get_solution's constraint values: one wave per row of J (CSR), the columns < nx (A's; the slack
// columns left out), a fixed-order wave sum, + cfix (the fixed columns' terms)
__global__ __launch_bounds__(NT) void k_cons(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                             const double* __restrict__ v, const double* __restrict__ x,
                                             const double* __restrict__ cfix, int m, int nx, double* __restrict__ out) {
  const int row = blockIdx.x * (NT / 64) + threadIdx.x / 64, l = threadIdx.x & 63;
  if (row >= m) return;
  double a = 0.0;
  for (int64_t p = rp[row] + l; p < rp[row + 1]; p += 64) {
    const int c = ci[p];
    if (c < nx) a = fma(v[p], x[c], a);
  }
  a = wave_reduce<OP_SUM>(a);
  if (l == 0) out[row] = a + cfix[row];
}
__global__ void k_axpy_x(DV D) {
  GRID_LOOP(i, D.n) D.x[i] += D.d[i];
}
__global__ void k_copy_y(DV D) {
  GRID_LOOP(j, D.m) D.y[j] = D.d[D.n + j];
}
// Gondzio: set_extra_correction! (kernels.jl:74-122)
__global__ void k_extra_corr(DV D, double ap, double ad, double tmin, double tmax) {
  const int n = D.n, m = D.m, nlb = D.nlb, nub = D.nub;
  GRID_LOOP(t, (nlb > nub ? nlb : nub)) {
    if (t < nlb) {
      const int i = D.ind_lb[t];
      const double xx = D.x[i] + ap * D.d[i] - D.xl[i];
      const double zz = D.zl[i] + ad * D.d[n + m + t];
      const double v = xx * zz;
      const double del = v < tmin ? tmin - v : (v > tmax ? tmax - v : 0.0);
      D.corr_lb[t] = D.corr_lb[t] - del;
    }
    if (t < nub) {
      const int i = D.ind_ub[t];
      const double xx = D.xu[i] - ap * D.d[i] - D.x[i];
      const double zz = D.zu[i] + ad * D.d[n + m + nlb + t];
      const double v = xx * zz;
      const double del = v < tmin ? tmin - v : (v > tmax ? tmax - v : 0.0);
      D.corr_ub[t] = D.corr_ub[t] + del;
    }
  }
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// ======================================================================= host side

MPCSolver::~MPCSolver() {
  if (fdbg_.p) {  // MADIPM_FINAL_DEBUG: per finaliser kind, thread 0's mean time to the reduced values / to the end
    std::vector<int64_t> h((size_t)8 * kFinDbg);
    (void)hipStreamSynchronize(stream_);
    (void)hipMemcpy(h.data(), fdbg_.p, h.size() * 8, hipMemcpyDeviceToHost);
    std::map<int64_t, std::array<double, 6>> acc;
    for (int64_t q = 0; q < std::min<int64_t>(fdbg_n_, kFinDbg); ++q) {
      const int64_t* e = &h[8 * q];
      auto& a = acc[e[3]];
      a[0] += 1;
      a[1] += (e[4] - e[0]) * 1e-2;  // 100 MHz ticks -> us
      a[2] += (e[5] - e[0]) * 1e-2;
      a[3] += (e[6] - e[0]) * 1e-2;
      a[4] += (e[1] - e[0]) * 1e-2;
      a[5] += (e[2] - e[0]) * 1e-2;
    }
    for (auto& kv : acc) {
      const double n = kv.second[0];
      std::fprintf(stderr,
                   "k_final kind %2lld (alpha %d eval %d): %6.0f launches  wg0 loads %6.2f  wg0 level-1 %6.2f  last ticket "
                   "%6.2f  reduced %6.2f  end %6.2f us\n",
                   (long long)(kv.first & 15), (int)((kv.first >> 4) & 1), (int)((kv.first >> 5) & 1), n,
                   kv.second[1] / n, kv.second[2] / n, kv.second[3] / n, kv.second[4] / n, kv.second[5] / n);
    }
  }
  if (hst_) (void)hipHostFree(hst_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

int MPCSolver::blocks(int64_t n) const {
  int64_t b = (n + NT - 1) / NT;
  return (int)std::max<int64_t>(1, std::min<int64_t>(maxb_, b));
}

// GROUP_LOOP SpMV kernels: one row per lane group (spmv_g_ lanes), so a group walks one row instead
// of a dependent chain of rows (the row loads are latency-bound)
int MPCSolver::spmv_blocks(int64_t rows) const { return blocks(rows * spmv_g_); }

// ---- host construction helpers, threaded for the dense-QP config (5e8 entries in A): every O(nnz) pass
// runs on analysis_threads() host threads over contiguous input chunks, with per-thread counts and
// offsets in thread order, so the result is the one-thread result bit for bit (r3: 38 s of analysis_s
// on the box, mostly single-threaded passes and growing vectors over the 5e8 entries).
template <class F>
static void par_range(int64_t n, F f, int64_t grain = (int64_t)1 << 20) {
  const int T = (int)std::min<int64_t>(analysis_threads(), std::max<int64_t>(1, n / grain));
  if (T <= 1) {
    f(0, (int64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(f, t, n * t / T, n * (t + 1) / T);
  for (auto& x : th) x.join();
}
static int par_threads(int64_t n, int64_t grain = (int64_t)1 << 20) {
  return (int)std::min<int64_t>(analysis_threads(), std::max<int64_t>(1, n / grain));
}

// CSR (sorted by (row, col), duplicates summed in input order) of the COO (r, c, v): a stable counting
// sort by row — per-thread row counts over input chunks, offsets in thread order — then each row's
// run sorted by column only when it is not already (O(nnz) for the usual column- or row-major input;
// a comparison sort of 1e9 dense-QP entries took minutes) and duplicates merged
// entry k of the COO: row R(k), column C(k), value V(k) (accessors: the scaled Jacobian is read
// straight from the caller's A, no COO copy); the CSR arrays are filled in full by the threads
template <class R, class C, class V>
static void csr_from_coo(int nrow, int64_t nnz, R r, C c, V v, std::vector<int64_t>& rp, hvec<int32_t>& ci,
                         hvec<double>& cv) {
  // per-thread row counts cost T (nrow + 1) int64: bound T so that they stay within the entries' own
  // size (a tall sparse matrix with millions of rows would otherwise take gigabytes of scratch)
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(par_threads(nnz), nnz / (4 * ((int64_t)nrow + 1))));
  std::vector<std::vector<int64_t>> cnt(T, std::vector<int64_t>(nrow + 1, 0));
  auto chunk = [&](int t) { return std::make_pair(nnz * t / T, nnz * (t + 1) / T); };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        auto [k0, k1] = chunk(t);
        int64_t* cn = cnt[t].data();
        for (int64_t k = k0; k < k1; ++k) cn[r(k)]++;
      });
    for (auto& x : th) x.join();
  }
  std::vector<int64_t> start(nrow + 1, 0);
  for (int i = 0; i < nrow; ++i) {
    int64_t acc = start[i];
    for (int t = 0; t < T; ++t) {
      const int64_t c_ = cnt[t][i];
      cnt[t][i] = acc;  // this thread's first slot in row i
      acc += c_;
    }
    start[i + 1] = acc;
  }
  hvec<int32_t> tc(nnz);
  hvec<double> tv(nnz);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        auto [k0, k1] = chunk(t);
        int64_t* off = cnt[t].data();
        for (int64_t k = k0; k < k1; ++k) {
          const int64_t q = off[r(k)]++;
          tc[q] = c(k);
          tv[q] = v(k);
        }
      });
    for (auto& x : th) x.join();
  }
  // per row: sort if needed (stable: duplicates keep input order), count the distinct columns
  std::vector<int64_t> uniq(nrow + 1, 0);
  par_range(nrow, [&](int, int64_t i0, int64_t i1) {
    std::vector<std::pair<int32_t, double>> buf;
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t b = start[i], e = start[i + 1];
      bool sorted = true;
      for (int64_t q = b; q + 1 < e && sorted; ++q) sorted = tc[q] <= tc[q + 1];
      if (!sorted) {
        buf.clear();
        for (int64_t q = b; q < e; ++q) buf.emplace_back(tc[q], tv[q]);
        std::stable_sort(buf.begin(), buf.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        for (int64_t q = b; q < e; ++q) tc[q] = buf[q - b].first, tv[q] = buf[q - b].second;
      }
      int64_t u = 0;
      for (int64_t q = b; q < e; ++q) u += (q == b || tc[q] != tc[q - 1]);
      uniq[i + 1] = u;
    }
  }, 4096);
  for (int i = 0; i < nrow; ++i) uniq[i + 1] += uniq[i];
  if (uniq[nrow] == nnz) {  // no duplicates: the sorted runs are the CSR
    rp = std::move(start);
    ci = std::move(tc);
    cv = std::move(tv);
    return;
  }
  rp = uniq;
  ci.resize(uniq[nrow]);
  cv.resize(uniq[nrow]);
  par_range(nrow, [&](int, int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      int64_t o = rp[i] - 1;
      for (int64_t q = start[i]; q < start[i + 1]; ++q) {
        if (q == start[i] || tc[q] != tc[q - 1]) {
          ++o;
          ci[o] = tc[q];
          cv[o] = tv[q];
        } else {
          cv[o] += tv[q];
        }
      }
    }
  }, 4096);
}
static void csr_from_coo(int nrow, const std::vector<int32_t>& r, const std::vector<int32_t>& c,
                         const std::vector<double>& v, std::vector<int64_t>& rp, hvec<int32_t>& ci, hvec<double>& cv) {
  const int32_t *rr = r.data(), *cc = c.data();
  const double* vv = v.data();
  csr_from_coo(
      nrow, (int64_t)r.size(), [=](int64_t k) { return rr[k]; }, [=](int64_t k) { return cc[k]; },
      [=](int64_t k) { return vv[k]; }, rp, ci, cv);
}

MPCSolver::MPCSolver(const madipm_qp& qp, const madipm_options& opt, Comm* comm) : opt_(opt), comm_(comm) {
  const double t0 = now();
  PhaseClock clk("MPCSolver");
  MADIPM_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  clk("stream");
  // state mirror + publication counter on their own line: coherent host memory, written by k_publish
  constexpr size_t seq_off = (sizeof(DevState) + 63) / 64 * 64;
  MADIPM_HIP(hipHostMalloc((void**)&hst_, seq_off + 64, hipHostMallocCoherent));
  std::memset((void*)hst_, 0, seq_off + 64);
  hseq_ = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(hst_) + seq_off);
  clk("host state");
  setup_host(qp);
  clk("setup_host (its locals freed)");
  t_init_ = now() - t0;
}

// The linear solver: one LDL^T, or a sharded one — across processes (comm, RCCL) or as a group of
// shards on this device (ldl.nshards > 1, ShardGroup)
std::unique_ptr<LinSolver> MPCSolver::make_linsolver(int n, const int64_t* cp, const int32_t* ri,
                                                     const SymbolicOptions& so) {
  if (comm_ && comm_->size > 1) {
    SymbolicOptions o = so;
    o.nshards = comm_->size;
    o.shard = comm_->rank;
    return std::make_unique<LDLSolver>(n, cp, ri, o, opt_.ldl.pivot_tol, nullptr, comm_);
  }
  if (opt_.ldl.nshards > 1)
    return std::make_unique<ShardGroup>(opt_.ldl.nshards, n, cp, ri, so, opt_.ldl.pivot_tol);
  return std::make_unique<LDLSolver>(n, cp, ri, so, opt_.ldl.pivot_tol);
}

// Host-side construction: MPCSolver(...) (structure.jl:79-178), MadNLP.initialize!/set_scaling!
// [EXT] and the K2 pattern of SparseKKTSystem [EXT].
void MPCSolver::setup_host(const madipm_qp& q) {
  PhaseClock clk("setup_host");
  H_ = std::make_unique<QPHost>();
  QPHost& P = *H_;
  MADIPM_REQUIRE(q.nvar >= 0 && q.ncon >= 0, "negative dimensions");
  P.nx = q.nvar;
  P.m = q.ncon;
  const int nx = P.nx, m = P.m;
  auto cp = [](const double* a, int64_t n, double dflt = 0.0) {
    std::vector<double> v(n, dflt);
    if (a) std::copy(a, a + n, v.begin());
    return v;
  };
  P.c = cp(q.c, nx);
  P.lvar = cp(q.lvar, nx, -INF);
  P.uvar = cp(q.uvar, nx, INF);
  P.lcon = cp(q.lcon, m, -INF);
  P.ucon = cp(q.ucon, m, INF);
  P.x0 = cp(q.x0, nx);
  P.y0 = cp(q.y0, m);
  P.c0 = q.c0;
  P.minimize = q.minimize != 0;
  P.sgn = P.minimize ? 1.0 : -1.0;
  P.Hr.assign(q.Hrows, q.Hrows + q.nnzh);
  P.Hc.assign(q.Hcols, q.Hcols + q.nnzh);
  P.Hv.assign(q.Hvals, q.Hvals + q.nnzh);
  P.Ar = q.Arows;
  P.Ac = q.Acols;
  P.Av = q.Avals;
  P.nnzA = q.nnzj;
  for (int64_t k = 0; k < q.nnzh; ++k)
    MADIPM_REQUIRE(P.Hr[k] >= P.Hc[k] && P.Hr[k] < nx && P.Hc[k] >= 0, "H must be lower-triangular COO in range");
  {
    std::atomic<bool> bad{false};
    par_range(q.nnzj, [&](int, int64_t a, int64_t b) {
      bool ok = true;
      for (int64_t k = a; k < b; ++k) ok &= P.Ar[k] >= 0 && P.Ar[k] < m && P.Ac[k] >= 0 && P.Ac[k] < nx;
      if (!ok) bad = true;
    });
    MADIPM_REQUIRE(!bad, "A index out of range");
  }
  clk("copy + validate");
  // ---- index sets: MadNLP.get_index_constraints (EnforceEquality, MakeParameter) [EXT]
  for (int i = 0; i < m; ++i)
    if (P.lcon[i] != P.ucon[i]) P.ind_ineq.push_back(i);
  P.ns = (int)P.ind_ineq.size();
  const int n = nx + P.ns;
  P.n = n;
  P.xl.resize(n);
  P.xu.resize(n);
  for (int i = 0; i < nx; ++i) {
    P.xl[i] = P.lvar[i];
    P.xu[i] = P.uvar[i];
  }
  for (int k = 0; k < P.ns; ++k) {
    P.xl[nx + k] = P.lcon[P.ind_ineq[k]];
    P.xu[nx + k] = P.ucon[P.ind_ineq[k]];
  }
  P.fixed.assign(n, 0);
  for (int i = 0; i < n; ++i) {
    if (P.xl[i] == P.xu[i]) {
      P.ind_fixed.push_back(i);
      P.fixed[i] = 1;
    } else {
      if (P.xl[i] != -INF) P.ind_lb.push_back(i);
      if (P.xu[i] != INF) P.ind_ub.push_back(i);
    }
  }
  // structure.jl:172-173 field swap => update_barrier! tests nlb + nub > 0
  P.has_ineq = (P.ind_lb.size() + P.ind_ub.size()) > 0;
  // ---- MadNLP.initialize!(cb, ...) [EXT]
  P.x.assign(n, 0.0);
  for (int i = 0; i < nx; ++i) P.x[i] = P.x0[i];
  for (int i : P.ind_fixed) P.x[i] = P.xl[i];
  P.y = P.y0;
  P.rhs.assign(m, 0.0);
  for (int i = 0; i < m; ++i) P.rhs[i] = (P.lcon[i] == P.ucon[i]) ? P.lcon[i] : 0.0;
  const double tol = opt_.bound_relax_factor;
  for (int i = 0; i < n; ++i) {
    if (P.fixed[i]) continue;
    if (std::isfinite(P.xl[i])) P.xl[i] = P.xl[i] - tol * std::max(1.0, std::fabs(P.xl[i]));
    if (std::isfinite(P.xu[i])) P.xu[i] = P.xu[i] + tol * std::max(1.0, std::fabs(P.xu[i]));
  }
  if (P.ns) {
    std::vector<double> ax(m, 0.0);
    for (int64_t k = 0; k < P.nnzA; ++k) ax[P.Ar[k]] += P.Av[k] * P.x[P.Ac[k]];
    for (int k = 0; k < P.ns; ++k) P.x[nx + k] = ax[P.ind_ineq[k]];
  }
  // initialize_variables! (Ipopt bound push) [EXT]
  const double bp = opt_.bound_push, bf = opt_.bound_fac;
  for (int i = 0; i < n; ++i) {
    if (P.fixed[i]) continue;
    const double l = P.xl[i], u = P.xu[i];
    double lo = -INF, hi = INF;
    if (std::isfinite(l)) {
      double pl = bp * std::max(1.0, std::fabs(l));
      if (std::isfinite(u)) pl = std::min(pl, bf * (u - l));
      lo = l + pl;
    }
    if (std::isfinite(u)) {
      double pu = bp * std::max(1.0, std::fabs(u));
      if (std::isfinite(l)) pu = std::min(pu, bf * (u - l));
      hi = u - pu;
    }
    P.x[i] = std::min(std::max(P.x[i], lo), hi);
  }
  // ---- set_scaling!(..., 100) [EXT] (solver.jl:148-159)
  P.obj_scale = 1.0;
  P.con_scale.assign(m, 1.0);
  if (opt_.scaling) {
    std::vector<double> g(nx);
    for (int i = 0; i < nx; ++i) g[i] = P.sgn * P.c[i];
    for (size_t k = 0; k < P.Hv.size(); ++k) {
      const int r = P.Hr[k], c = P.Hc[k];
      const double v = P.sgn * P.Hv[k];
      g[r] += v * P.x[c];
      if (r != c) g[c] += v * P.x[r];
    }
    double gmax = 0;
    for (double v : g) gmax = std::max(gmax, std::fabs(v));
    P.obj_scale = gmax > 0 ? std::min(1.0, 100.0 / gmax) : 1.0;
    std::vector<double> rowmax(m, 0.0);
    {  // per-thread row maxima, then their maximum (order-free)
      const int64_t nz = P.nnzA;
      // at most nz / (4 m) threads: their m-long maxima stay within the entries' own size
      const int64_t tc = std::max<int64_t>(1, std::min<int64_t>(par_threads(nz), nz / (4 * std::max(m, 1))));
      std::vector<std::vector<double>> rm(tc, std::vector<double>(m, 0.0));
      par_range(nz, [&](int t, int64_t a, int64_t b) {
        double* x = rm[t].data();
        for (int64_t k = a; k < b; ++k) x[P.Ar[k]] = std::max(x[P.Ar[k]], std::fabs(P.Av[k]));
      }, std::max<int64_t>((int64_t)1 << 20, (nz + tc - 1) / tc));
      for (const auto& x : rm)
        for (int i = 0; i < m; ++i) rowmax[i] = std::max(rowmax[i], x[i]);
    }
    for (int i = 0; i < m; ++i) P.con_scale[i] = std::min(1.0, 100.0 / rowmax[i]);
    for (int k = 0; k < P.ns; ++k) {
      const double cs = P.con_scale[P.ind_ineq[k]];
      P.xl[nx + k] *= cs;
      P.xu[nx + k] *= cs;
      P.x[nx + k] *= cs;
    }
    for (int i = 0; i < m; ++i) P.rhs[i] *= P.con_scale[i];
  }
  obj_scale_ = P.obj_scale;
  clk("initialize + scaling");

  // ---- device problem data
  nx_ = nx;
  ns_ = P.ns;
  n_ = n;
  m_ = m;
  nlb_ = (int)P.ind_lb.size();
  nub_ = (int)P.ind_ub.size();
  L_ = (int64_t)n + m + nlb_ + nub_;
  // scaled Hessian (full symmetric CSR over n; MakeParameter zeroes fixed rows/cols), diagonal apart
  std::vector<int32_t> hr, hc;
  std::vector<double> hv, Hdiag(n, 0.0);
  std::vector<double> gfix(n, 0.0), cfix(m, 0.0);
  double const_fixed = 0.0;
  for (size_t k = 0; k < P.Hv.size(); ++k) {
    const int r = P.Hr[k], c = P.Hc[k];
    const double v = P.obj_scale * P.sgn * P.Hv[k];
    const bool fr = P.fixed[r], fc = P.fixed[c];
    if (fr && fc) {
      const_fixed += (r == c ? 0.5 : 1.0) * v * P.x[r] * P.x[c];
      continue;
    }
    if (fr || fc) {  // cross term with a fixed variable -> constant gradient shift
      if (!fr) gfix[r] += v * P.x[c];
      if (!fc) gfix[c] += v * P.x[r];
      continue;
    }
    if (r == c) {
      Hdiag[r] += v;
      hr.push_back(r);
      hc.push_back(c);
      hv.push_back(v);
    } else {
      hr.push_back(r);
      hc.push_back(c);
      hv.push_back(v);
      hr.push_back(c);
      hc.push_back(r);
      hv.push_back(v);
    }
  }
  std::vector<int64_t> Hrp;
  hvec<int32_t> Hci;
  hvec<double> Hcv;
  csr_from_coo(n, hr, hc, hv, Hrp, Hci, Hcv);
  // scaled Jacobian with slack columns (m x n); fixed columns zeroed (their term -> cfix).  Without a
  // fixed column every entry is kept in input order and read straight from the caller's A
  std::vector<int32_t> jr, jc;
  std::vector<double> jv;
  bool anyfix = false;
  for (int i = 0; i < nx && !anyfix; ++i) anyfix = P.fixed[i];
  {
    const int64_t nz = P.nnzA;
    if (anyfix) {  // cfix sums in input order: the sequential pass
      for (int64_t k = 0; k < nz; ++k) {
        const int r = P.Ar[k], c = P.Ac[k];
        const double v = P.con_scale[r] * P.Av[k];
        if (P.fixed[c]) {
          cfix[r] += v * P.x[c];
          continue;
        }
        jr.push_back(r);
        jc.push_back(c);
        jv.push_back(v);
      }
      for (int k = 0; k < P.ns; ++k) {
        jr.push_back(P.ind_ineq[k]);
        jc.push_back(nx + k);
        jv.push_back(-1.0);
      }
    }
  }
  clk("H CSR + J COO");
  std::vector<int64_t> Jrp, JTrp;
  hvec<int32_t> Jci, JTci;
  hvec<double> Jcv, JTcv;
  if (anyfix) {
    csr_from_coo(m, jr, jc, jv, Jrp, Jci, Jcv);
    csr_from_coo(n, jc, jr, jv, JTrp, JTci, JTcv);
    std::vector<int32_t>().swap(jr);
    std::vector<int32_t>().swap(jc);
    std::vector<double>().swap(jv);
  } else {  // entries k < nnzA: A's (scaled); then one -1 per slack column
    const int64_t na = P.nnzA, nj = na + P.ns;
    const int32_t *Ar = P.Ar, *Ac = P.Ac, *ineq = P.ind_ineq.data();
    const double *Av = P.Av, *cs = P.con_scale.data();
    auto row = [=](int64_t k) { return k < na ? Ar[k] : ineq[k - na]; };
    auto col = [=](int64_t k) { return k < na ? Ac[k] : (int32_t)(nx + (k - na)); };
    auto val = [=](int64_t k) { return k < na ? cs[Ar[k]] * Av[k] : -1.0; };
    csr_from_coo(m, nj, row, col, val, Jrp, Jci, Jcv);
    csr_from_coo(n, nj, col, row, val, JTrp, JTci, JTcv);
  }
  clk("J, J^T CSR");
  std::vector<double> cs(n, 0.0);
  for (int i = 0; i < nx; ++i) cs[i] = P.obj_scale * P.sgn * P.c[i];
  c0s_ = P.obj_scale * (P.sgn * P.c0) + const_fixed;
  // K2 lower CSC: diag(n+m) + H strictly-lower + J at rows n+r  (SparseKKTSystem [EXT]), built by
  // columns: column j < n = [j; H's rows i > j (row j of the symmetric CSR H, ascending); n + the rows r
  // of column j of J (row j of J^T's CSR, ascending)], column j >= n = [j]
  std::vector<int64_t> Kcp(n + m + 1, 0);
  hvec<int32_t> Kri;
  hvec<double> Kv;
  {
    std::vector<int64_t> hup(n, 0);  // per column: H entries below the diagonal
    for (int i = 0; i < n; ++i)
      for (int64_t q = Hrp[i]; q < Hrp[i + 1]; ++q) hup[i] += Hci[q] > i;
    for (int j = 0; j < n + m; ++j) Kcp[j + 1] = Kcp[j] + 1 + (j < n ? hup[j] + (JTrp[j + 1] - JTrp[j]) : 0);
    Kri.resize(Kcp[n + m]);
    Kv.resize(Kcp[n + m]);
    par_range(n + m, [&](int, int64_t j0, int64_t j1) {
      for (int64_t j = j0; j < j1; ++j) {
        int64_t o = Kcp[j];
        Kri[o] = (int32_t)j;
        Kv[o++] = 0.0;
        if (j >= n) continue;
        for (int64_t q = Hrp[j]; q < Hrp[j + 1]; ++q)
          if (Hci[q] > j) {
            Kri[o] = Hci[q];
            Kv[o++] = Hcv[q];
          }
        for (int64_t q = JTrp[j]; q < JTrp[j + 1]; ++q) {
          Kri[o] = n + JTci[q];
          Kv[o++] = JTcv[q];
        }
      }
    }, 1024);
  }
  nnzK_ = (int64_t)Kri.size();
  clk("K2 CSC");
  if (const char* e = std::getenv("MADIPM_SPEC_NEAR")) spec_near_ = std::max(0.0, std::atof(e));
  if (const char* e = std::getenv("MADIPM_FINAL_DEBUG"); e && e[0] == '1') {
    fdbg_.alloc(8 * kFinDbg);
    MADIPM_HIP(hipMemset(fdbg_.p, 0, 8 * kFinDbg * sizeof(int64_t)));
  }
  {  // SpMV lane-group width: ~2 entries per lane on an average row of [H A^T; A]
    const double avg = (double)(Hci.size() + 2 * Jci.size()) / std::max(1, n + m);
    spmv_g_ = 4;
    while (spmv_g_ < 64 && spmv_g_ * 2 < avg) spmv_g_ *= 2;
  }
  std::vector<int64_t> diag_pos(Kcp.begin(), Kcp.end() - 1);  // the diagonal leads every column

  // ---- KKT formulation + LDL^T symbolic analysis + device plan (linear-solver constructor)
  kkt_ = opt_.kkt_system;
  MADIPM_REQUIRE(kkt_ == KKT_K2 || kkt_ == KKT_K25 || kkt_ == KKT_NORMAL, "unknown kkt_system");
  SymbolicOptions so;
  so.ordering = opt_.ldl.ordering;
  so.dense_alpha = opt_.ldl.dense_alpha;
  so.relax = opt_.ldl.relax;
  so.small_front_max = opt_.ldl.small_front_max;
  std::vector<int64_t> Ccp, cpp;
  std::vector<int32_t> Cri, cprod;
  if (kkt_ == KKT_NORMAL) {
    // NormalKKTSystem constructor (normalkkt.jl:29-140): LP only; pattern of tril(A A^T) with A the
    // scaled Jacobian with slack columns (build_normal_system, utils.jl:209-274), plus the product
    // list of every entry for the assembly kernel (positions into J's CSR values).
    MADIPM_REQUIRE(q.nnzh == 0,
                   "The KKT system NormalKKTSystem supports only linear programs. "
                   "The problem has a positive number of nonzero in its Hessian.");
    std::vector<int64_t> colp(n + 1, 0);
    for (int32_t k : Jci) colp[k + 1]++;
    for (int k = 0; k < n; ++k) colp[k + 1] += colp[k];
    std::vector<int32_t> crow(Jci.size()), cpos(Jci.size());
    {
      std::vector<int64_t> fill(colp.begin(), colp.end() - 1);
      for (int i = 0; i < m; ++i)
        for (int64_t p = Jrp[i]; p < Jrp[i + 1]; ++p) {
          const int64_t t = fill[Jci[p]]++;
          crow[t] = i;
          cpos[t] = (int32_t)p;
        }
    }
    Ccp.assign(m + 1, 0);
    cpp.push_back(0);
    struct Prod {
      int32_t j, a, b;
    };
    std::vector<Prod> pr;
    for (int i = 0; i < m; ++i) {
      pr.clear();
      for (int64_t p = Jrp[i]; p < Jrp[i + 1]; ++p) {
        const int k = Jci[p];
        for (int64_t t = colp[k]; t < colp[k + 1]; ++t)
          if (crow[t] >= i) pr.push_back({crow[t], (int32_t)p, cpos[t]});
      }
      std::stable_sort(pr.begin(), pr.end(), [](const Prod& x, const Prod& y) { return x.j < y.j; });
      for (size_t t = 0; t < pr.size(); ++t) {
        if (t == 0 || pr[t].j != pr[t - 1].j) {
          if (t) cpp.push_back((int64_t)cprod.size() / 2);
          Cri.push_back(pr[t].j);
        }
        cprod.push_back(pr[t].a);
        cprod.push_back(pr[t].b);
      }
      if (!pr.empty()) {
        cpp.push_back((int64_t)cprod.size() / 2);
      } else {  // empty row of A: structurally singular C; keep the (zero) diagonal entry
        Cri.push_back(i);
        cpp.push_back((int64_t)cprod.size() / 2);
      }
      Ccp[i + 1] = (int64_t)Cri.size();
    }
    nnzC_ = (int64_t)Cri.size();
    ldl_ = make_linsolver(m, Ccp.data(), Cri.data(), so);
    ldl_->spd = true;  // Cholesky semantics (test/test_gpu.jl:11): a non-positive pivot fails
  } else {
    ldl_ = make_linsolver(n + m, Kcp.data(), Kri.data(), so);
  }

  clk("linear solver (analysis + plan)");
  // ---- uploads
  std::vector<int32_t> lbpos(n, -1), ubpos(n, -1);
  for (int k = 0; k < nlb_; ++k) lbpos[P.ind_lb[k]] = k;
  for (int k = 0; k < nub_; ++k) ubpos[P.ind_ub[k]] = k;
  hipStream_t s = stream_;
  auto up = [&](auto& buf, const auto& vec, size_t minlen = 1) {
    using T = typename std::decay_t<decltype(vec)>::value_type;
    buf.alloc(std::max(vec.size(), minlen));
    if (!vec.empty()) MADIPM_HIP(hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice, s));
  };
  up(x_, P.x);
  up(xl_, P.xl);
  up(xu_, P.xu);
  up(y_, P.y);
  up(rhs_, P.rhs);
  up(Hdiag_, Hdiag);
  up(cs_, cs);
  up(gfix_, gfix);
  up(cfix_, cfix);
  up(diag_pos_, diag_pos);
  up(Kx_, Kv);
  up(ind_lb_, P.ind_lb);
  up(ind_ub_, P.ind_ub);
  up(lbpos_, lbpos);
  up(ubpos_, ubpos);
  up(fixed_, P.fixed);
  up(Hrp_, Hrp);
  up(Hci_, Hci);
  up(Hv_, Hcv);
  up(Jrp_, Jrp);
  up(Jci_, Jci);
  up(Jv_, Jcv);
  up(JTrp_, JTrp);
  up(JTci_, JTci);
  up(JTv_, JTcv);
  auto zeros = [&](DBuf<double>& b, int64_t len) {
    b.alloc(std::max<int64_t>(len, 1));
    b.zero(s);
  };
  zeros(zl_, n);
  zeros(zu_, n);
  zeros(f_, n);
  zeros(jacl_, n);
  zeros(c_, m);
  zeros(pr_diag_, n);
  zeros(l_diag_, nlb_);
  zeros(u_diag_, nub_);
  zeros(l_lower_, nlb_);
  zeros(u_lower_, nub_);
  zeros(d_, L_);
  zeros(p_, L_);
  zeros(dsave_, L_);
  zeros(corr_lb_, nlb_);
  zeros(corr_ub_, nub_);
  if (kkt_ == KKT_NORMAL) {
    up(cpp_, cpp);
    up(cprod_, cprod, 2);
    zeros(Cx_, nnzC_);
    zeros(Dinv_, n);
    zeros(bufm_, m);
  } else if (kkt_ == KKT_K25) {
    hvec<int32_t> kcol(Kri.size());
    par_range(n + m, [&](int, int64_t j0, int64_t j1) {
      for (int64_t j = j0; j < j1; ++j)
        for (int64_t q = Kcp[j]; q < Kcp[j + 1]; ++q) kcol[q] = (int32_t)j;
    }, 1024);
    up(Krow_, Kri);
    up(Kcol_, kcol);
    up(K0_, Kv);
    zeros(sk_, n);
  }
  part_.alloc(MAXB * NPART + NL2 * FG + 8);  // + k_final's level-2 partials and ticket
  MADIPM_HIP(hipMemset(part_.p, 0, (MAXB * NPART + NL2 * FG + 8) * sizeof(double)));
  st_.alloc(1);
  if (ldl_->external_status(&st_.p->ldl_status, &hst_->ldl_status)) {  // carried by read_state()
    // the MPC's own kernels start / end each factorisation: no k_status_init, no k_inertia (K2, K2.5:
    // the pivot check needs no inertia; the normal equations' Cholesky check keeps k_inertia)
    ldl_->ext_reset = true;
    ldl_->lazy_inertia = !ldl_->spd;
  }
  st_.zero(s);
  MADIPM_HIP(hipStreamSynchronize(s));
  clk("uploads");
  // norm_b (solver.jl:173) on host
  norm_b_ = 0;
  for (double v : P.rhs) norm_b_ = std::max(norm_b_, std::fabs(v));
  // the host copies of J, J^T and K2 (dense QP: ~18 GB) are released on a thread of their own: their
  // page-table teardown took 2.1 s of the construction on the box (r6) with nothing waiting for it
  free_async(std::move(Jci), std::move(JTci), std::move(Jcv), std::move(JTcv), std::move(Kri), std::move(Kv),
             std::move(Hci), std::move(Hcv));
}

// Launch helpers (the DV view is rebuilt from member buffers; cheap, host-only)
#define DV_ARGS                                                                                         \
  DV D;                                                                                                 \
  D.n = n_;                                                                                             \
  D.m = m_;                                                                                             \
  D.nx = nx_;                                                                                           \
  D.nlb = nlb_;                                                                                         \
  D.nub = nub_;                                                                                         \
  D.x = x_;                                                                                             \
  D.xl = xl_;                                                                                           \
  D.xu = xu_;                                                                                           \
  D.zl = zl_;                                                                                           \
  D.zu = zu_;                                                                                           \
  D.f = f_;                                                                                             \
  D.jacl = jacl_;                                                                                       \
  D.c = c_;                                                                                             \
  D.y = y_;                                                                                             \
  D.rhs = rhs_;                                                                                         \
  D.pr_diag = pr_diag_;                                                                                 \
  D.l_diag = l_diag_;                                                                                   \
  D.u_diag = u_diag_;                                                                                   \
  D.l_lower = l_lower_;                                                                                 \
  D.u_lower = u_lower_;                                                                                 \
  D.d = d_;                                                                                             \
  D.p = p_;                                                                                             \
  D.corr_lb = corr_lb_;                                                                                 \
  D.corr_ub = corr_ub_;                                                                                 \
  D.Kx = Kx_;                                                                                           \
  D.diag_pos = diag_pos_;                                                                               \
  D.Hdiag = Hdiag_;                                                                                     \
  D.cs = cs_;                                                                                           \
  D.gfix = gfix_;                                                                                       \
  D.cfix = cfix_;                                                                                       \
  D.ind_lb = ind_lb_;                                                                                   \
  D.ind_ub = ind_ub_;                                                                                   \
  D.lbpos = lbpos_;                                                                                     \
  D.ubpos = ubpos_;                                                                                     \
  D.fixed = fixed_;                                                                                     \
  D.H = DCsr{Hrp_, Hci_, Hv_};                                                                          \
  D.J = DCsr{Jrp_, Jci_, Jv_};                                                                          \
  D.JT = DCsr{JTrp_, JTci_, JTv_};                                                                      \
  D.part = part_;                                                                                       \
  D.st = st_;                                                                                           \
  D.kkt = kkt_;                                                                                         \
  D.sk = sk_;                                                                                           \
  D.Krow = Krow_;                                                                                       \
  D.Kcol = Kcol_;                                                                                       \
  D.K0 = K0_;                                                                                           \
  D.nnzK = nnzK_;                                                                                       \
  D.Dinv = Dinv_;                                                                                       \
  D.bufm = bufm_;                                                                                       \
  D.cpp = cpp_;                                                                                         \
  D.cprod = reinterpret_cast<const int2*>(cprod_.p);                                                    \
  D.Cx = Cx_;                                                                                           \
  D.nnzC = nnzC_;

// launch a GROUP_LOOP SpMV kernel with the problem's lane-group width
#define SPMV_LAUNCH(kern, grid, strm, ...)                                        \
  do {                                                                            \
    switch (spmv_g_) {                                                            \
      case 4: kern<4><<<(grid), NT, 0, (strm)>>>(__VA_ARGS__); break;             \
      case 8: kern<8><<<(grid), NT, 0, (strm)>>>(__VA_ARGS__); break;             \
      case 16: kern<16><<<(grid), NT, 0, (strm)>>>(__VA_ARGS__); break;           \
      case 32: kern<32><<<(grid), NT, 0, (strm)>>>(__VA_ARGS__); break;           \
      default: kern<64><<<(grid), NT, 0, (strm)>>>(__VA_ARGS__); break;           \
    }                                                                             \
  } while (0)

void MPCSolver::kkt_diag(double dw, double dc) {
  DV_ARGS;
  k_diag<<<blocks(n_ + m_), NT, 0, stream_>>>(D, dw, dc, fact_reset());
}

// set_aug_diagonal_reg! + build_kkt! of the chosen formulation (values consumed by the LDL^T)
void MPCSolver::assemble_kkt(double dw, double dc, bool diag_done) {
  DV_ARGS;
  if (!diag_done) kkt_diag(dw, dc);
  if (kkt_ == KKT_K25) k_k25_scale<<<blocks(nnzK_), NT, 0, stream_>>>(D);
  if (kkt_ == KKT_NORMAL) k_normal_asm<<<blocks(nnzC_), NT, 0, stream_>>>(D);
}

const double* MPCSolver::kvals() const { return kkt_ == KKT_NORMAL ? Cx_.p : Kx_.p; }

// factorize! between two pooled timing events (cnt.linear_solver_time, MadNLP.factorize_wrapper!);
// the pool grows only when a solve needs more pairs than any earlier one did
void MPCSolver::timed_factorize() {
  ldl_->factorize_async(kvals(), stream_);
  // the next k_rhs stamps the factorisation's end (an asynchronous tail stamps its own)
  fact_end_pending_ = ldl_->lazy_inertia && !ldl_->tail_async();
}

// the status block the kernel right before a factorisation resets (LinSolver::ext_reset), or nullptr
LDLStatus* MPCSolver::fact_reset() const { return ldl_->ext_reset ? &st_.p->ldl_status : nullptr; }
// the status block the first kernel after a factorisation stamps (LinSolver::lazy_inertia), or nullptr
LDLStatus* MPCSolver::take_fact_end() {
  LDLStatus* p = fact_end_pending_ ? &st_.p->ldl_status : nullptr;
  fact_end_pending_ = false;
  return p;
}

void MPCSolver::factor_enqueue(double dw, double dc) {
  assemble_kkt(dw, dc);
  timed_factorize();
}

// MadNLP.solve!(kkt, d) between reduce_rhs! (k_rhs) and finish_aug_solve! (k_residual)
void MPCSolver::kkt_solve() {
  DV_ARGS;
  if (kkt_ == KKT_NORMAL) {
    SPMV_LAUNCH(k_normal_rhs, spmv_blocks(m_), stream_, D);
    ldl_->solve_async(bufm_.p, stream_);
    SPMV_LAUNCH(k_normal_back, spmv_blocks(n_ + m_), stream_, D);
  } else {
    ldl_->solve_async(d_.p, stream_);
    if (kkt_ == KKT_K25) k_k25_unscale<<<blocks(n_), NT, 0, stream_>>>(D);
  }
}

void MPCSolver::launch_reduce_final(int kind, int nb, int amode, int nb_eval, LDLStatus* rs, bool publish) {
  DV_ARGS;
  FinParams P{nb, 0, 0, 0, 0, 0, nb_eval, rs};
  if (publish) {
    P.host = hst_;
    P.hseq = hseq_;
    P.seq = ++pub_seq_;
  }
  if (nb_eval > 0) P.c = c0s_;
  if (amode >= 0) {
    P.alpha_mode = amode;
    P.nb_alpha = blocks(std::max(nlb_, nub_));
  }
  if (kind == FIN_MU_PRED) {
    P.a = (double)(nlb_ + nub_);
    P.b = H_->has_ineq ? 1.0 : 0.0;
    P.c = opt_.mu_min;
  } else if (kind == FIN_MU_FULL) {
    P.a = (double)(nlb_ + nub_);
    P.b = opt_.step_tau;
  } else if (kind == FIN_MU_GONDZIO) {
    P.a = (double)(nlb_ + nub_);
  } else if (kind == FIN_EVAL) {
    P.a = c0s_;
  } else if (kind == FIN_RESID) {
    P.a = opt_.check_residual ? opt_.tol_linear_solve : 0.0;
  }
  if (fdbg_.p) P.dbg = fdbg_.p + 8 * (fdbg_n_++ % kFinDbg);
  launch_final(D, kind, P, stream_);
}

// solve_system! (linear_solver.jl:19-44): rhs (mode) -> LDL^T solve -> finish + residual
void MPCSolver::solve_system(int mode, double mu, int reset, int amode, double atau, int mu_nb) {
  DV_ARGS;
  const int nb = blocks(n_ + m_), nbs = spmv_blocks(n_ + m_);
  DevState* host = nullptr;
  uint32_t seq = 0;
  bool late = false;  // published by the residual's finaliser instead: after the solve joined the
                      // factorisation's asynchronous tail, whose pivot check the state carries
  if (publish_next_ && ldl_->tail_async()) {
    late = true;
    publish_next_ = false;
  } else if (publish_next_) {  // read_state() folded into this launch
    host = hst_;
    seq = ++pub_seq_;
    publish_next_ = false;
  }
  MuFold mf{0, 0.0, 0.0, 0.0};
  if (mu_nb > 0) mf = MuFold{mu_nb, (double)(nlb_ + nub_), H_->has_ineq ? 1.0 : 0.0, opt_.mu_min};
  k_rhs<<<nb, NT, 0, stream_>>>(D, mode, mu, reset, host, hseq_, seq, mf, take_fact_end());
  kkt_solve();
  // amode >= 0: the step test of that mode on the new direction runs in the same launch (its own
  // blocks) and is finalised with the residual
  const int nbz = amode >= 0 ? blocks(std::max(nlb_, nub_)) : 0;
  SPMV_LAUNCH(k_residual, nbs + nbz, stream_, D, del_w_, del_c_, nbs, amode, atau);
  launch_reduce_final(FIN_RESID, nbs, amode, 0, nullptr, late);
}

// gondzio_correction_direction! (solver.jl:245-298): host-controlled loop, one read-back per solve
void MPCSolver::gondzio() {
  DV_ARGS;
  hipStream_t s = stream_;
  const double delta = 0.1, bmin = 0.1, bmax = 10.0, tau = 0.995;
  const int nbz = blocks(std::max(nlb_, nub_));
  auto ftb = [&](double& ap, double& ad) {  // get_fraction_to_boundary_step(solver, tau)
    k_alpha<<<nbz, NT, 0, s>>>(D, ALPHA_GONDZIO, tau, 0);
    FinParams P{nbz, ALPHA_GONDZIO, 0, 0, 0, 0, 0};
    launch_final(D, FIN_ALPHA, P, s);
    read_state();
    wait_state();
    ap = hst_->alpha_aff_p;
    ad = hst_->alpha_aff_d;
  };
  double ap, ad;
  ftb(ap, ad);
  for (int nc = 0; nc < opt_.max_ncorr; ++nc) {
    const double tap = std::min(ap + delta, 1.0), tad = std::min(ad + delta, 1.0);
    k_mu<<<nbz, NT, 0, s>>>(D, 0, tap, tad);
    launch_reduce_final(FIN_MU_GONDZIO, nbz);
    read_state();
    wait_state();
    const double ga = hst_->mu_aff, g = hst_->mu_curr;
    const double mu = (ga / g) * (ga / g) * ga;  // Eq. (12)
    k_extra_corr<<<nbz, NT, 0, s>>>(D, tap, tad, bmin * mu, bmax * mu);
    k_copy<<<blocks(L_), NT, 0, s>>>(dsave_, d_, L_);  // copyto!(dp, d.values) happens before the solve
    solve_system(RHS_GONDZIO, mu);
    double hap, had;
    ftb(hap, had);
    if (hap < 1.005 * ap || had < 1.005 * ad) {
      k_copy<<<blocks(L_), NT, 0, s>>>(d_, dsave_, L_);
      break;
    }
    ap = hap;
    ad = had;
  }
}

void MPCSolver::read_state() {
  k_publish<<<1, 64, 0, stream_>>>(st_, hst_, hseq_, ++pub_seq_);
  MADIPM_HIP(hipGetLastError());
}

// Host spin on the publication counter (no event record in the stream: each one costs a ~5 us
// bubble between kernels); bounded, and a failed stream surfaces as its HIP error.  The stream is
// queried only once a wait has lasted 2 ms: a query puts a marker into the stream, another ~6 us
// bubble at the point the host had enqueued to (r6_x: before the predictor's k_rhs and k_apply)
void MPCSolver::wait_state() {
  const double t0 = now();
  for (uint64_t spin = 0;; ++spin) {
    if (__atomic_load_n(hseq_, __ATOMIC_ACQUIRE) == pub_seq_) return;
    if ((spin & 1023) == 1023 && now() - t0 > 2e-3) {
      const hipError_t e = hipStreamQuery(stream_);
      if (e != hipSuccess && e != hipErrorNotReady) MADIPM_HIP(e);
      if (e == hipSuccess && __atomic_load_n(hseq_, __ATOMIC_ACQUIRE) != pub_seq_)
        throw Error("state publication lost (stream idle, counter not updated)", -5);
      if (now() - t0 > 600.0) throw Error("state publication: timed out", -5);
    }
  }
}

void MPCSolver::init_starting_point() {
  DV_ARGS;
  const int nb = blocks(n_ + m_), nbn = blocks(n_);
  hipStream_t s = stream_;
  k_init_kkt<<<nb, NT, 0, s>>>(D, del_w_, del_c_, fact_reset());
  if (kkt_ == KKT_NORMAL) k_normal_asm<<<blocks(nnzC_), NT, 0, s>>>(D);
  if (kkt_ == KKT_K25) k_k25_scale<<<blocks(nnzK_), NT, 0, s>>>(D);  // s = 1: K2.5 = K2
  timed_factorize();
  // init factorization: the reference does not retry here; a solve with an unfactorized LDL^T is a
  // step-computation failure (oracle/mpc.py solve_system)
  if (ldl_->status(s) != 0) {
    exception_ = MADIPM_EXC_UNFACTORIZED;
    throw Error("init_starting_point!: KKT factorization failed", -4);
  }
  // Step 1: least-squares primal correction
  k_rhs<<<nb, NT, 0, s>>>(D, RHS_INIT_PRIMAL, 0.0, 0, nullptr, nullptr, 0, MuFold{0, 0.0, 0.0, 0.0}, take_fact_end());
  kkt_solve();
  SPMV_LAUNCH(k_residual, nb, s, D, del_w_, del_c_, nb, -1, 1.0);
  launch_reduce_final(FIN_RESID, nb);
  k_axpy_x<<<nbn, NT, 0, s>>>(D);
  // Step 2: dual least squares
  k_rhs<<<nb, NT, 0, s>>>(D, RHS_INIT_DUAL, 0.0, 0, nullptr, nullptr, 0, MuFold{0, 0.0, 0.0, 0.0}, take_fact_end());
  kkt_solve();
  SPMV_LAUNCH(k_residual, nb, s, D, del_w_, del_c_, nb, -1, 1.0);
  launch_reduce_final(FIN_RESID, nb);
  k_copy_y<<<blocks(m_), NT, 0, s>>>(D);
  // Step 3: bound multipliers and shifts
  k_zinit<<<nbn, NT, 0, s>>>(D);
  launch_reduce_final(FIN_ZINIT, nbn);
  k_zshift1<<<nbn, NT, 0, s>>>(D);
  launch_reduce_final(FIN_ZSHIFT1, nbn);
  k_zshift2<<<nbn, NT, 0, s>>>(D, opt_.bound_fac);
  launch_reduce_final(FIN_ZSHIFT2, nbn);
  read_state();
  wait_state();
  if (hst_->nan_flag) {
    exception_ = MADIPM_EXC_SOLVE;
    throw Error("SolveException in init_starting_point!", -4);
  }
  MADIPM_REQUIRE(hst_->init_viol == 0.0, "init_starting_point!: interior assertion failed");
}

void MPCSolver::initialize() {
  DV_ARGS;
  hipStream_t s = stream_;
  {  // restart from the problem's initial point (solve! always restarts)
    const QPHost& P = *H_;
    MADIPM_HIP(hipMemcpyAsync(x_.p, P.x.data(), sizeof(double) * n_, hipMemcpyHostToDevice, s));
    MADIPM_HIP(hipMemcpyAsync(xl_.p, P.xl.data(), sizeof(double) * n_, hipMemcpyHostToDevice, s));
    MADIPM_HIP(hipMemcpyAsync(xu_.p, P.xu.data(), sizeof(double) * n_, hipMemcpyHostToDevice, s));
    if (m_) MADIPM_HIP(hipMemcpyAsync(y_.p, P.y.data(), sizeof(double) * m_, hipMemcpyHostToDevice, s));
    zl_.zero(s);
    zu_.zero(s);
    d_.zero(s);
    p_.zero(s);
  }
  fs0_ = ldl_->fact_seconds(s);
  // init_regularization! (kernels.jl:364-392)
  switch (opt_.regularization) {
    case 0: del_w_ = 1.0; del_c_ = 0.0; break;
    case 1: del_w_ = 1.0; del_c_ = opt_.delta_d; break;
    default:
      adapt_dp_ = opt_.delta_p;
      adapt_dd_ = opt_.delta_d;
      adapt_dmin_ = opt_.delta_min;
      del_w_ = 1.0;
      del_c_ = opt_.delta_d;
  }
  k_set_mu<<<1, 1, 0, s>>>(st_, 0.0);
  // callbacks at the initial point (solver.jl:166-170)
  const int nb = blocks(n_ + m_);
  SPMV_LAUNCH(k_eval, nb, s, D, 0);
  launch_reduce_final(FIN_EVAL, nb);
  // norm_c = ||primal(f)||_inf (solver.jl:174)
  std::vector<double> fh(n_);
  if (n_) MADIPM_HIP(hipMemcpyAsync(fh.data(), f_.p, sizeof(double) * n_, hipMemcpyDeviceToHost, s));
  MADIPM_HIP(hipStreamSynchronize(s));
  norm_c_ = 0;
  for (double v : fh) norm_c_ = std::max(norm_c_, std::fabs(v));
  init_starting_point();
  k_set_mu<<<1, 1, 0, s>>>(st_, opt_.mu_init);  // solver.jl:179
  k_jtprod<<<blocks(n_), NT, 0, s>>>(D);        // solver.jl:187
  best_compl_ = INF;
  status_ = MADIPM_REGULAR;
  k_ = 0;
  eval_pending_ = false;
}

void MPCSolver::initialize_public() {
  const double t0 = now();
  initialize();
  MADIPM_HIP(hipStreamSynchronize(stream_));
  t_init_ += now() - t0;
  initialized_ = true;
}

// prediction_step! (solver.jl:230-237) + mehrotra_correction_direction! (solver.jl:239-243)
void MPCSolver::directions(bool redo, bool fuse_step) {
  DV_ARGS;
  hipStream_t s = stream_;
  const int nbz = blocks(std::max(nlb_, nub_));
  // the affine step test (get_alpha_max_primal/dual with tau = 1) is finalised with the residual
  solve_system(RHS_PRED, 0.0, redo ? 2 : 1, ALPHA_PRED, 1.0);
  // mu_affine at (alpha_aff_p, alpha_aff_d) and mu_curr; the alphas never leave the device.  The
  // barrier update (FIN_MU_PRED) is finalised inside the corrector's k_rhs (no separate launch).
  k_mu<<<nbz, NT, 0, s>>>(D, 1, 0.0, 0.0);
  double tau = 1.0;
  const int amode = fuse_step ? step_alpha_mode(tau) : -1;
  solve_system(RHS_CORR, 0.0, 0, amode, tau, nbz);
}

// the step test update_step_size! runs for the configured rule (its mode and tau parameter)
int MPCSolver::step_alpha_mode(double& tau) const {
  if (opt_.step_rule == 2) {
    tau = 1.0;
    return ALPHA_MEHROTRA;
  }
  tau = opt_.step_tau;
  return opt_.step_rule == 0 ? ALPHA_CONSERVATIVE : ALPHA_ADAPTIVE;
}

// update_step_size! (solver.jl:304-307)
// fused: the corrector solve already ran the step test (directions(.., true))
void MPCSolver::step_size(bool fused) {
  DV_ARGS;
  hipStream_t s = stream_;
  const int nbz = blocks(std::max(nlb_, nub_));
  double tau = 1.0;
  const int mode = step_alpha_mode(tau);
  if (!fused) {
    k_alpha<<<nbz, NT, 0, s>>>(D, mode, tau, 0);
    FinParams P{nbz, mode, 0, 0, 0, 0, 0};
    launch_final(D, FIN_ALPHA, P, s);
  }
  if (opt_.step_rule == 2) {
    k_mu<<<nbz, NT, 0, s>>>(D, 1, 0.0, 0.0);
    launch_reduce_final(FIN_MU_FULL, nbz);
  }
}

int MPCSolver::solve(madipm_stats* stats) {
  DV_ARGS;
  hipStream_t s = stream_;
  trace_.clear();
  int status = MADIPM_REGULAR;
  exception_ = MADIPM_EXC_NONE;
  double tstart = now();
  try {
    if (!initialized_) initialize_public();
    initialized_ = false;
    tstart = now();  // solver.jl:181
    const int nb = blocks(n_ + m_);
    while (true) {
      // ---- update_termination_criteria! (+ speculative factorization of this iteration)
      const double del_w_print = del_w_;
      // factorize_system! = update_regularization! + factorize_regularized_system!
      double save_w = del_w_, save_c = del_c_;
      switch (opt_.regularization) {
        case 0: del_w_ = 0.0; del_c_ = 0.0; break;
        case 1: del_w_ = opt_.delta_p; del_c_ = opt_.delta_d; break;
        default:
          adapt_dp_ = std::max(adapt_dp_ / 10.0, adapt_dmin_);
          adapt_dd_ = std::min(adapt_dd_ / 10.0, -adapt_dmin_);
          del_w_ = adapt_dp_;
          del_c_ = adapt_dd_;
      }
      // first trial enqueued together with the state read-back: ONE sync per iteration.  At
      // k >= max_iter the termination test ends the solve whatever it finds: nothing to speculate.
      const bool last = k_ >= opt_.max_iter;
      k_term<<<nb, NT, 0, s>>>(D, last ? 0 : 1, del_w_, del_c_);
      // the termination test's state is published by its own finaliser: the host decides while the GPU
      // runs this iteration's (speculative) factorisation, and a converged solve enqueues no directions
      launch_reduce_final(FIN_TERM, nb, -1, eval_pending_ ? spmv_blocks(n_ + m_) : 0, last ? nullptr : fact_reset(),
                          true);
      eval_pending_ = false;
      // the factorisation is enqueued before the host reads the termination test (speculatively),
      // except when the previous iteration's residuals were within spec_near_ x tol: there the solve
      // is likely to stop now, and a converged test would leave the whole factorisation as waste
      // (~0.3 ms on ex10) where holding it back costs one host turn-around (~20 us) otherwise
      const bool hold = !last && spec_near_ > 0 && k_ > 0 &&
                        std::max(inf_pr_, std::max(inf_du_, inf_compl_)) <= spec_near_ * opt_.tol;
      if (!last && !hold) {
        assemble_kkt(del_w_, del_c_, true);
        timed_factorize();
      }
      wait_state();
      const DevState h = *hst_;
      last_ = h;
      if (h.nan_flag) {
        // SolveException in the previous iteration's solve_system! (linear_solver.jl:40-41): the
        // reference throws before apply_step!, so k_apply skipped the step on the device and the
        // iteration is not counted (cnt.k += 1 is inside apply_step!, solver.jl:316).  It throws the
        // TYPE MadNLP.SolveException, which is not `isa MadNLP.LinearSolverException`, so solve!'s
        // catch-all maps it to INTERNAL_ERROR (solver.jl:398-403)
        status = MADIPM_INTERNAL_ERROR;
        exception_ = MADIPM_EXC_SOLVE;
        if (k_ > 0) --k_;
        break;
      }
      const double dobj = h.dobj;
      inf_pr_ = h.inf_pr_raw / std::max(1.0, norm_b_);
      inf_du_ = h.inf_du_raw / std::max(1.0, norm_c_);
      inf_compl_ = h.inf_compl_raw / std::max(1.0, norm_c_);
      best_compl_ = std::min(best_compl_, inf_compl_);
      const double obj_val = h.obj_val;
      madipm_iter_trace tr{k_, obj_val / obj_scale_, inf_pr_, inf_du_, inf_compl_, h.mu, h.alpha_p, h.alpha_d,
                           del_w_print, k_ == 0 ? 0.0 : h.dx_inf, h.max_res_ratio};
      trace_.push_back(tr);
      if (opt_.print_level > 0) {
        if (k_ % 10 == 0) std::printf("iter    objective    inf_pr   inf_du lg(mu)  ||d||  lg(rg) alpha_du alpha_pr\n");
        char rg[16];
        if (del_w_print == 0)
          std::snprintf(rg, sizeof rg, "   - ");
        else
          std::snprintf(rg, sizeof rg, "%5.1f", std::log10(del_w_print));
        std::printf("%4d % 10.7e %6.2e %6.2e %5.1f %6.2e %s %6.2e %6.2e\n", k_, obj_val / obj_scale_, inf_pr_,
                    inf_du_, std::log10(h.mu), tr.dx_inf, rg, h.alpha_d, h.alpha_p);
      }
      if (std::max(inf_pr_, std::max(inf_du_, inf_compl_)) <= opt_.tol) {
        status = MADIPM_SOLVE_SUCCEEDED;
      } else if (inf_compl_ > opt_.divergence_tol * best_compl_ && dobj > std::max(10.0 * std::fabs(obj_val), 1.0)) {
        status = MADIPM_INFEASIBLE_PROBLEM_DETECTED;
      } else if (obj_val < -opt_.divergence_tol * std::max(std::max(10.0, std::fabs(dobj)), 1.0)) {
        status = MADIPM_DIVERGING_ITERATES;
      } else if (k_ >= opt_.max_iter) {
        status = MADIPM_MAXIMUM_ITERATIONS_EXCEEDED;
      } else if (now() - tstart >= opt_.max_wall_time) {
        status = MADIPM_MAXIMUM_WALLTIME_EXCEEDED;
      }
      if (status != MADIPM_REGULAR) {
        del_w_ = save_w;
        del_c_ = save_c;
        break;
      }
      // speculation: this iteration's directions (prediction_step!, mehrotra_correction_direction!,
      // update_step_size!) are enqueued BEFORE the host reads the factorisation status, so the GPU is
      // busy while the host decides; they write scratch vectors and step scalars only (the iterate is
      // updated by k_apply, enqueued after the decision) and are recomputed after a failed
      // factorisation's retries.  Gondzio's loop synchronises internally: not speculated.
      if (hold) {
        assemble_kkt(del_w_, del_c_, true);
        timed_factorize();
      }
      const bool spec = opt_.max_ncorr == 0;
      if (spec) {  // the state read-back (with the factorisation status) rides on the predictor's first launch
        publish_next_ = true;
        directions(false, true);
        step_size(true);
      } else {
        ldl_->join(s);  // the factorisation's asynchronous tail (its pivot check) before the read-back
        read_state();
      }
      wait_state();
      const int frc = ldl_->status(s, false);
      if (frc != 0) {  // remaining trials of factorize_regularized_system!
        bool ok = false;
        for (int trial = 1; trial < 3 && !ok; ++trial) {
          del_w_ *= 100.0;
          del_c_ *= 100.0;
          factor_enqueue(del_w_, del_c_);
          ok = ldl_->status(s) == 0;
        }
        if (!ok) {  // every trial failed: prediction_step!'s solve would use an unfactorized LDL^T,
          // which the linear solver refuses with an exception that is no LinearSolverException
          // (LDLFactorizations' ldiv! [EXT]) -> solve!'s catch-all: INTERNAL_ERROR (solver.jl:398-403)
          del_w_ *= 100.0;
          del_c_ *= 100.0;
          status = MADIPM_INTERNAL_ERROR;
          exception_ = MADIPM_EXC_UNFACTORIZED;
          break;
        }
        if (spec) {  // the speculated directions used the failed factor: recompute
          directions(true, true);
          step_size(true);
        }
      }
      if (!spec) {
        directions(false, false);
        gondzio();  // gondzio_correction_direction! (solver.jl:245-298)
        step_size(false);
      }
      // ---- apply_step! + evaluate_model!
      k_apply<<<nb, NT, 0, s>>>(D);
      ++k_;
      // evaluate_model!: its objective is finalised by the next iteration's FIN_TERM (one launch
      // less; nothing reads obj_val before the termination test)
      SPMV_LAUNCH(k_eval, spmv_blocks(n_ + m_), s, D, PART_EVAL);
      eval_pending_ = true;
      MADIPM_HIP(hipGetLastError());
    }
  } catch (const Error& e) {
    // init_starting_point!'s failures (code -4): the same two exceptions, caught by solve!'s
    // catch-all (solver.jl:398-403)
    if (e.code == -4)
      status = MADIPM_INTERNAL_ERROR;
    else
      throw;
  }
  MADIPM_HIP(hipStreamSynchronize(s));
  t_total_ = now() - tstart;
  status_ = status;
  t_linsol_ = ldl_->fact_seconds(s) - fs0_;
  if (stats) {
    // the state read at the last termination test (the speculated directions after it changed only
    // step scalars, never the iterate)
    if (trace_.empty()) {
      read_state();
      wait_state();
      last_ = *hst_;
    }
    stats->status = status;
    stats->iter = k_;
    double obj = last_.obj_val / obj_scale_;
    if (!H_->minimize) obj = -obj;
    stats->objective = obj;
    stats->dual_objective = last_.dobj / obj_scale_;
    stats->inf_pr = inf_pr_;
    stats->inf_du = inf_du_;
    stats->inf_compl = inf_compl_;
    stats->mu = last_.mu;
    stats->total_time = t_total_;
    stats->linear_solver_time = t_linsol_;
    stats->init_time = t_init_;
    stats->exception = exception_;
  }
  return status;
}

}  // namespace madipm

namespace madipm {

// update_solution! (src/utils.jl:150-156) + MadNLP.update! [EXT]: un-scaled primal/dual solution
void MPCSolver::get_solution(double* x, double* y, double* zl, double* zu, double* cons) {
  MADIPM_HIP(hipStreamSynchronize(stream_));
  const QPHost& P = *H_;
  std::vector<double> xh(n_), yh(m_), zlh(n_), zuh(n_);
  if (n_) {
    MADIPM_HIP(hipMemcpy(xh.data(), x_.p, sizeof(double) * n_, hipMemcpyDeviceToHost));
    MADIPM_HIP(hipMemcpy(zlh.data(), zl_.p, sizeof(double) * n_, hipMemcpyDeviceToHost));
    MADIPM_HIP(hipMemcpy(zuh.data(), zu_.p, sizeof(double) * n_, hipMemcpyDeviceToHost));
  }
  if (m_) MADIPM_HIP(hipMemcpy(yh.data(), y_.p, sizeof(double) * m_, hipMemcpyDeviceToHost));
  if (x) std::copy(xh.begin(), xh.begin() + nx_, x);
  if (zl)
    for (int i = 0; i < nx_; ++i) zl[i] = zlh[i] / obj_scale_;
  if (zu)
    for (int i = 0; i < nx_; ++i) zu[i] = zuh[i] / obj_scale_;
  if (y)
    for (int j = 0; j < m_; ++j) y[j] = yh[j] * P.con_scale[j] / obj_scale_;
  if (cons && m_) {  // A x = (J's columns < nx) x / con_scale + the fixed columns' part (cfix / con_scale)
    DBuf<double> ax;
    ax.alloc(m_);
    k_cons<<<(unsigned)((m_ + NT / 64 - 1) / (NT / 64)), NT, 0, stream_>>>(Jrp_, Jci_, Jv_, x_, cfix_, m_, nx_, ax);
    MADIPM_HIP(hipGetLastError());
    std::vector<double> h(m_);
    MADIPM_HIP(hipMemcpyAsync(h.data(), ax.p, sizeof(double) * m_, hipMemcpyDeviceToHost, stream_));
    MADIPM_HIP(hipStreamSynchronize(stream_));
    for (int j = 0; j < m_; ++j) cons[j] = h[j] / P.con_scale[j];
  }
}

}  // namespace madipm

namespace madipm {

// update_step! (kernels.jl:291-358) on caller-given bounded-coordinate vectors, through the solver's
// own step-test kernels (k_alpha + k_final(FIN_ALPHA), and k_mu + k_final(FIN_MU_FULL) for
// MehrotraAdaptiveStep).  The vectors are laid out as a problem with n = nlb + nub primal
// coordinates, the lower-bounded ones first, no constraints: ind_lb = [0, nlb), ind_ub = [nlb, n).
void update_step_standalone(int rule, double tau_param, double mu, int nlb, int nub, const double* const* v,
                            madipm_step_result* out, hipStream_t s) {
  const int n = nlb + nub;
  MADIPM_REQUIRE(nlb >= 0 && nub >= 0 && n > 0, "update_step: no bounded coordinate");
  MADIPM_REQUIRE(rule >= 0 && rule <= 2, "update_step: rule must be 0, 1 or 2");
  DBuf<double> x(n), xl(n), xu(n), zl(n), zu(n), d(n + nlb + nub), part((size_t)NPART * MAXB + NL2 * FG + 8);
  DBuf<int32_t> ilb(std::max(nlb, 1)), iub(std::max(nub, 1));
  DBuf<DevState> st(1);
  std::vector<int32_t> io(n);
  for (int i = 0; i < n; ++i) io[i] = i;
  ilb.upload(io.data(), nlb, s);
  iub.upload(io.data() + nlb, nub, s);
  MADIPM_HIP(hipMemsetAsync(part.p, 0, sizeof(double) * part.n, s));  // k_final's ticket starts at 0
  MADIPM_HIP(hipMemsetAsync(x.p, 0, sizeof(double) * n, s));
  MADIPM_HIP(hipMemsetAsync(xl.p, 0, sizeof(double) * n, s));
  MADIPM_HIP(hipMemsetAsync(xu.p, 0, sizeof(double) * n, s));
  MADIPM_HIP(hipMemsetAsync(zl.p, 0, sizeof(double) * n, s));
  MADIPM_HIP(hipMemsetAsync(zu.p, 0, sizeof(double) * n, s));
  auto cp = [&](double* dst, const double* src, int cnt) {
    if (cnt) MADIPM_HIP(hipMemcpyAsync(dst, src, sizeof(double) * cnt, hipMemcpyDeviceToDevice, s));
  };
  // v: x_lr, xl_r, zl_r, dx_lr, dzl, x_ur, xu_r, zu_r, dx_ur, dzu
  cp(x.p, v[0], nlb), cp(xl.p, v[1], nlb), cp(zl.p, v[2], nlb), cp(d.p, v[3], nlb), cp(d.p + n, v[4], nlb);
  cp(x.p + nlb, v[5], nub), cp(xu.p + nlb, v[6], nub), cp(zu.p + nlb, v[7], nub), cp(d.p + nlb, v[8], nub);
  cp(d.p + n + nlb, v[9], nub);
  DV D{};
  D.n = n;
  D.m = 0;
  D.nx = n;
  D.nlb = nlb;
  D.nub = nub;
  D.x = x.p, D.xl = xl.p, D.xu = xu.p, D.zl = zl.p, D.zu = zu.p, D.d = d.p;
  D.ind_lb = ilb.p, D.ind_ub = iub.p;
  D.part = part.p;
  D.st = st.p;
  k_set_mu<<<1, 1, 0, s>>>(st.p, mu);
  const int nbz = (int)std::max<int64_t>(1, std::min<int64_t>(MAXB, (std::max(nlb, nub) + NT - 1) / NT));
  const int mode = rule == 0 ? ALPHA_CONSERVATIVE : (rule == 1 ? ALPHA_ADAPTIVE : ALPHA_MEHROTRA);
  const double tau = rule == 2 ? 1.0 : tau_param;
  k_alpha<<<nbz, NT, 0, s>>>(D, mode, tau, 0);
  FinParams P{nbz, mode, 0, 0, 0, 0, 0};
  launch_final(D, FIN_ALPHA, P, s);
  if (rule == 2) {
    k_mu<<<nbz, NT, 0, s>>>(D, 1, 0.0, 0.0);
    FinParams Q{nbz, 0, (double)(nlb + nub), tau_param, 0, 0, 0};
    launch_final(D, FIN_MU_FULL, Q, s);
  }
  MADIPM_HIP(hipGetLastError());
  DevState h{};
  MADIPM_HIP(hipMemcpyAsync(&h, st.p, sizeof(DevState), hipMemcpyDeviceToHost, s));
  MADIPM_HIP(hipStreamSynchronize(s));
  out->alpha_p = h.alpha_p;
  out->alpha_d = h.alpha_d;
  out->alpha_xl = h.a_xl, out->alpha_xu = h.a_xu, out->alpha_zl = h.a_zl, out->alpha_zu = h.a_zu;
  out->i_xl = h.i_xl, out->i_xu = h.i_xu, out->i_zl = h.i_zl, out->i_zu = h.i_zu;
}

}  // namespace madipm
