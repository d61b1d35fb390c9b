/*
 * madipm_hip.h — C-ABI of libmadipm_hip.so, the MI355X (gfx950) hot path of MadIPM's
 * Mehrotra predictor-corrector (reference: klamike/MadIPM.jl v0.1.2).
 *
 * Conventions: 0-based indices, Float64 values, int32 row indices, int64 column pointers /
 * nonzero counts.  Every function returns 0 on success, a negative code on error (text in
 * madipm_last_error(), thread-local); madipm_ldl_factorize additionally returns k+1 > 0 when
 * pivot k (internal order) is zero / non-finite, which maps to MadIPM.is_factorized == false.
 * Device pointers are plain hipMalloc'd (or torch / AMDGPU.jl ROCArray) addresses; `stream` is a
 * hipStream_t (NULL = default stream).  No exceptions cross this boundary.
 *
 * Which reference interface each entry point replaces is cited per function (file:line relative
 * to the reference root).  INTEGRATION.md shows the Julia `ccall` binding a maintainer would add.
 */
#ifndef MADIPM_HIP_H
#define MADIPM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* madipm_stream_t; /* hipStream_t */

/* ------------------------------------------------------------------ library */
int madipm_version(void);                 /* MAJOR*10000 + MINOR*100 + PATCH */
const char* madipm_last_error(void);
int madipm_device_count(void);            /* hipGetDeviceCount; 0 when no GPU is present */
int madipm_set_device(int32_t dev);       /* hipSetDevice for the calling thread (one process per GPU),
                                            and the runtime's one-off device set-up done
                                            (context, first stream) */

/* ------------------------------------------------------------------ symbolic analysis (host)
 * Replaces the symbolic phase run by the linear-solver constructor `linear_solver(aug_com; opt)`
 * (src/KKT/normalkkt.jl:113-115; SparseKKTSystem constructor in MadNLP [EXT]) — SURVEY §8 a12. */
typedef struct madipm_ldl_opts {
  int32_t ordering;        /* 0 natural, 1 AMD, 2 user permutation, 3 nested dissection,
                              4 auto = AMD and ND, fewer flops wins (default) */
  double dense_alpha;      /* AMD dense-node threshold factor (default 10) */
  int32_t relax;           /* relaxed supernode amalgamation (default 1) */
  int32_t small_front_max; /* fronts with <= this many rows are factorised in LDS (default 128; up to 192 with packed LDS storage) */
  double pivot_tol;        /* |d| <= pivot_tol  =>  pivot failure (default 0: only 0 / NaN / Inf) */
  int32_t nshards;         /* > 1: subtree-sharded factorisation with nshards shards on THIS device
                              (single process, local all-reduce; SURVEY §8 e); default 1.  Across
                              GPUs use madipm_solver_create_dist / madipm_ldl_analyze_shard. */
  int32_t cholesky;        /* 1: Cholesky semantics — the matrix must be SPD, any pivot that is not > 0
                              fails the factorisation (is_factorized == false): the cuDSS CHOLESKY
                              configuration the reference pairs with NormalKKTSystem
                              (test/test_gpu.jl:11); default 0 (quasi-definite LDL^T)  [ABI 0.2] */
} madipm_ldl_opts;

typedef struct madipm_ldl_info {
  int64_t n;
  int64_t nnzK;            /* entries of the lower CSC input */
  int64_t nnzL;            /* exact nnz(L) incl. diagonal */
  int64_t nnzL_stored;     /* lower-trapezoid entries stored by the supernodes (incl. relaxed zeros) */
  double flops;            /* factorisation flops, sum_j (c_j-1)(c_j+2) */
  int32_t nsuper;          /* fronts */
  int32_t nlevels;         /* levels of the front tree (launch schedule depth) */
  int32_t max_front;       /* largest front order */
  int32_t nbig;            /* fronts handled by the global-memory blocked path */
  int64_t arena_bytes;     /* device bytes for factor + update blocks */
  int32_t lb_groups;       /* batched leaf-column groups (each absorbed by one SYRK into its parent) */
  int32_t lb_members;      /* single-column leaf fronts in those groups */
  int32_t fold_fronts;     /* tree fronts that fold their micro leaves (LDS product lists) */
  int32_t fold_leaves;     /* micro leaves folded by them */
  int64_t xch_fact;        /* sharded: doubles all-reduced per factorisation (top-front lower triangles
                              + 4 status slots per shard); 0 unsharded */
  int64_t xch_solve;       /* sharded: doubles all-reduced per solve (the top fronts' forward right-hand
                              sides); 0 unsharded */
  int64_t xch_gather;      /* sharded: doubles of the per-solve in-place all-gather of the shards'
                              subtree solution slices (nshards slices); 0 unsharded */
  int32_t tree_fronts;     /* fronts factorised by the dependency-driven tree launch (k_fact_tree) [ABI 0.2] */
  int32_t tree_medium;     /* of which medium fronts (192 < r <= 256: factorised in HBM, one 64-column
                              panel in LDS at a time) [ABI 0.2] */
  int32_t root_tail_async; /* 1: the elimination-tree roots after the tree launch are assembled and
                              factorised on a side stream, beside the next solve's forward leaves and
                              tree fronts (MADIPM_ROOT_ASYNC, default on) [ABI 0.2.3] */
  int32_t pad_;
} madipm_ldl_info;

void madipm_ldl_default_opts(madipm_ldl_opts* opts);

typedef struct madipm_symbolic* madipm_symbolic_t;
/* colptr[n+1] (int64), rowval[nnz] (int32): lower triangle (row >= col), unique entries. */
int madipm_symbolic_analyze(int32_t n, const int64_t* colptr, const int32_t* rowval,
                            const madipm_ldl_opts* opts, const int32_t* user_perm,
                            madipm_symbolic_t* out);
int madipm_symbolic_info(madipm_symbolic_t sym, madipm_ldl_info* info);
int madipm_symbolic_perm(madipm_symbolic_t sym, int32_t* perm /* n */);
/* first[nsuper+1], parent[nsuper], nrows[nsuper] (any may be NULL) */
int madipm_symbolic_supernodes(madipm_symbolic_t sym, int32_t* first, int32_t* parent, int32_t* nrows);
void madipm_symbolic_destroy(madipm_symbolic_t sym);
/* symbolic analysis of one shard of a subtree-sharded factorisation (see "subtree sharding" below),
 * and the partition: owner[nsuper] (-1 top, else shard) and the cost-model totals */
int madipm_symbolic_analyze_shard(int32_t n, const int64_t* colptr, const int32_t* rowval,
                                  const madipm_ldl_opts* opts, int32_t nshards, int32_t shard,
                                  const int32_t* user_perm, madipm_symbolic_t* out);
int madipm_symbolic_shard_info(madipm_symbolic_t sym, int32_t* owner, double* top_cost, double* shard_cost_max,
                               double* shard_cost_sum);

/* ------------------------------------------------------------------ LDL^T linear solver (device)
 * The MadNLP.AbstractLinearSolver the reference plugs in through `linear_solver=`
 * (src/utils.jl:72, src/structure.jl:117-123): LDLSolver (LDLFactorizations), CUDSSSolver with
 * cudss_algorithm=MadNLP.LDL (scripts/benchmarks_gpu.jl:41-42), Ma57Solver
 * (scripts/benchmarks_cpu.jl:36).  SURVEY §8 a11/a12/a14, boundary §8(b). */
typedef struct madipm_ldl* madipm_ldl_t;
/* Constructor `LS(aug_com; opt)`: symbolic analysis + device upload (src/KKT/normalkkt.jl:113-115). */
int madipm_ldl_analyze(int32_t n, const int64_t* colptr, const int32_t* rowval,
                       const madipm_ldl_opts* opts, const int32_t* user_perm, madipm_ldl_t* out);
int madipm_ldl_get_info(madipm_ldl_t ls, madipm_ldl_info* info);
/* MadNLP.factorize!(ls) (called via factorize_wrapper!, src/linear_solver.jl:10, src/solver.jl:21).
 * d_nzval: device values in the CSC order given to madipm_ldl_analyze.  Synchronises `stream`;
 * returns 0, or k+1 for the first failing pivot k (=> madipm_ldl_is_factorized() == 0). */
int madipm_ldl_factorize(madipm_ldl_t ls, const double* d_nzval, madipm_stream_t stream);
/* Asynchronous variant; the outcome is read by madipm_ldl_is_factorized / madipm_ldl_inertia. */
int madipm_ldl_factorize_async(madipm_ldl_t ls, const double* d_nzval, madipm_stream_t stream);
/* MadIPM.is_factorized(ls) (src/utils.jl:54-62): 1 when the last factorisation succeeded. */
int madipm_ldl_is_factorized(madipm_ldl_t ls);
/* MadNLP.solve!(ls, x) (src/linear_solver.jl:26 via MadNLP.solve!(kkt, d)): in place, nrhs
 * columns of length n stored contiguously. */
int madipm_ldl_solve(madipm_ldl_t ls, double* d_x, int32_t nrhs, madipm_stream_t stream);
/* MadNLP.inertia(ls) -> (pos, zero, neg); MadNLP.is_inertia(ls) is true. */
int madipm_ldl_inertia(madipm_ldl_t ls, int32_t* pos, int32_t* zero, int32_t* neg);
/* Diagonal D of the last factorisation, internal (permuted) order, copied to host memory. */
int madipm_ldl_get_d(madipm_ldl_t ls, double* h_d);
int madipm_ldl_perm(madipm_ldl_t ls, int32_t* perm /* n */);
void madipm_ldl_destroy(madipm_ldl_t ls);

/* ------------------------------------------------------------------ subtree sharding (SURVEY §8 e)
 * The north star's multi-GPU mode: the front tree is cut into independent subtrees dealt to
 * `nshards` shards (one per GPU) plus their common ancestors ("top" fronts), which every shard
 * factorises redundantly after ONE all-reduce (sum) of the top fronts' external contributions.
 * A solve needs two more: an all-reduce of the top fronts' forward right-hand sides and an all-gather
 * of the shards' subtree solution slices (the top solution is computed redundantly on every shard).
 * No reference counterpart (the reference is single-device: cuDSS / LDLFactorizations); these entry
 * points let a host binding drive the phases with its own collective (e.g. Julia + RCCL.jl):
 *   factorize: phase 1 -> all-reduce(xbuf, xlen) -> phase 2
 *   solve:     phase 1 -> all-reduce(xbuf, xlen) -> phase 2 -> all-gather(xbuf, xlen) -> phase 3
 * The solve's phase 2 returns the gather buffer: nshards slices of xlen / nshards doubles, this
 * shard's slice (at shard * xlen / nshards) filled and the others zero, so an in-place all-gather
 * (madipm_comm_allgather, ncclAllGather) or a sum all-reduce of the whole buffer completes it.
 * Phase 3 scatters the other shards' slices into x (xbuf = NULL, xlen = 0).
 * Shards must be created with the same pattern and options; every shard computes the same cut. */
int madipm_ldl_analyze_shard(int32_t n, const int64_t* colptr, const int32_t* rowval, const madipm_ldl_opts* opts,
                             int32_t nshards, int32_t shard, const int32_t* user_perm, madipm_ldl_t* out);
int madipm_ldl_factorize_phase(madipm_ldl_t ls, int32_t phase /* 1 | 2 */, const double* d_nzval,
                               madipm_stream_t stream, double** xbuf, int64_t* xlen);
int madipm_ldl_solve_phase(madipm_ldl_t ls, int32_t phase /* 1 | 2 | 3 */, double* d_x, madipm_stream_t stream,
                           double** xbuf, int64_t* xlen);
/* owner[s] of every front (-1 top, else shard), and the partition's cost model totals */
int madipm_ldl_shard_info(madipm_ldl_t ls, int32_t* owner, double* top_cost, double* shard_cost_max,
                          double* shard_cost_sum);
/* sum of nbuf device buffers of length n, written back to all of them (single-process shards) */
int madipm_local_allreduce(double* const* d_bufs, int32_t nbuf, int64_t n, madipm_stream_t stream);

/* RCCL communicator (one process per GPU): rank 0 makes the 128-byte id, the host broadcasts it. */
typedef struct madipm_comm* madipm_comm_t;
int madipm_comm_unique_id(void* id128);
int madipm_comm_create(int32_t nranks, int32_t rank, const void* id128, madipm_comm_t* out);
/* Host-staged communicator: each all-reduce synchronises the stream, copies the buffer to pinned host
 * memory, calls fn(host_buf, n, ctx) (which must sum it across ranks in place and return 0) and
 * copies it back.  For testing the multi-process protocol where RCCL cannot run (ranks sharing a GPU). */
typedef int (*madipm_allreduce_fn)(double* host_buf, int64_t n, void* ctx);
int madipm_comm_create_host(int32_t nranks, int32_t rank, madipm_allreduce_fn fn, void* ctx, madipm_comm_t* out);
/* in-place fp64 sum over the communicator's ranks, ordered on `stream` */
int madipm_comm_allreduce(madipm_comm_t comm, double* d_buf, int64_t n, madipm_stream_t stream);
/* in-place all-gather of nranks slices of nper doubles (rank r's slice at d_buf + r * nper, the other
 * slices zero on entry; a host-staged communicator sums the whole buffer), ordered on `stream` */
int madipm_comm_allgather(madipm_comm_t comm, double* d_buf, int64_t nper, madipm_stream_t stream);
void madipm_comm_destroy(madipm_comm_t comm);

/* Live per-kernel timing (no reference counterpart; measurement for bench.py's roofline).
 * Bit k of `mask` records HIP events around every launch of kernel kind k on the launch stream
 * (kinds: 0 k_asm_chunks, 1 k_assemble, 2 k_tiny_factor, 3 k_small_factor, 4 k_big_diag,
 * 5 k_big_trsm, 6 k_big_update, 7 k_inertia, 8 k_fwd_small, 9 k_fwd_gather, 10 k_fwd_big,
 * 11 k_bwd_below, 12 k_bwd_big, 13 k_bwd_small, 14 k_fwd_tiny, 15 k_bwd_tiny, 16 k_lb_build,
 * 17 k_lb_syrk, 18 k_lb_gemv, 19 k_fwd_tree, 20 k_bwd_tree, 21 k_fact_tree, 22 k_asm_update,
 * 23 k_big_dag [ABI 0.2.2]).  Setting a mask clears the statistics. */
#define MADIPM_NKERNELS 24
typedef struct madipm_kstat {
  char name[32];
  int64_t launches;
  double time_ms;          /* summed event time of the launches */
  double bytes;            /* staging-traffic model of those launches (what the kernel moves) */
  double flops;            /* algorithmic flops of those launches */
  double alg_bytes;        /* SURVEY 8(d)'s algorithmic bytes of those launches: 8 nnzL + 12 nnzK of the
                              columns they factorise, 8 nnzL of the columns a solve launch substitutes */
} madipm_kstat;
int madipm_ldl_set_timing(madipm_ldl_t ls, uint32_t mask);
/* synchronises the recorded events; out[MADIPM_NKERNELS] */
int madipm_ldl_kernel_stats(madipm_ldl_t ls, madipm_kstat* out);

/* ------------------------------------------------------------------ array-type overrides
 * The ROCArray counterparts of the methods MadIPM's CUDA extension overrides so that MPCSolver
 * runs on device arrays (ext/MadIPMCUDAExt/cuda_wrapper.jl, MadIPMCUDAExt.jl).  Device pointers,
 * 0-based, int32 indices as the reference's CuSparseMatrix{Float64,Int32}; every sum has a fixed
 * order (bitwise reproducible), and transfer / assemble_normal_system follow the reference CPU
 * loops' order and rounding exactly.  Asynchronous on `stream` unless stated. */

/* MadNLP.transfer!(dest::CSC, src::COO, map) (cuda_wrapper.jl:4-24, used by build_kkt!/
 * compress_hessian! :26-30): dest .= 0; dest[map[k]] += src[k] for k = 0..nsrc-1, sources of one
 * entry summed in ascending k.  The plan is built once from the map (host or device pointer). */
typedef struct madipm_transfer* madipm_transfer_t;
int madipm_transfer_create(int64_t nsrc, const int64_t* map, int32_t map_on_device, int64_t ndest,
                           madipm_transfer_t* out);
int madipm_transfer(madipm_transfer_t t, double* d_dest, const double* d_src, madipm_stream_t stream);
void madipm_transfer_destroy(madipm_transfer_t t);

/* compress_jacobian!(::NormalKKTSystem) (normalkkt.jl:163-172, cuda_wrapper.jl:32-41):
 * AV[nnz-n_slack .. nnz-1] = -1 (in place), then ATnz[i] = AV[csr_map[i]] for i < nnz. */
int madipm_compress_jacobian(double* d_AV, int64_t nnz, int32_t n_slack, const int64_t* d_csr_map,
                             double* d_ATnz, madipm_stream_t stream);

/* MadIPMOperator(A::CuSparseMatrixCSR; transa, symmetric) (cuda_wrapper.jl:43-83) and its mul!
 * (:85-94).  A is m x n CSR (rowptr m+1, colval/nzval nnz; device).  symmetric != 0 (and nnz > 0):
 * the operator is mat = tril(A,-1) + A', copied at creation like the reference's `mat`;
 * otherwise the caller's arrays are read live at every apply ('T' through a transposed index plan
 * built at creation).  apply: y = alpha op(A) x + beta y (y is not read when beta == 0); y has
 * m rows for 'N' / symmetric, n for 'T'.  size reports size(A) and nnz(A) (Base.size, nnz). */
typedef struct madipm_spmv* madipm_spmv_t;
int madipm_spmv_create(int32_t m, int32_t n, int64_t nnz, const int32_t* d_rowptr, const int32_t* d_colval,
                       const double* d_nzval, char transa, int32_t symmetric, madipm_spmv_t* out);
int madipm_spmv_apply(madipm_spmv_t op, const double* d_x, double* d_y, double alpha, double beta,
                      madipm_stream_t stream);
int madipm_spmv_size(madipm_spmv_t op, int32_t* m, int32_t* n, int64_t* nnz);
void madipm_spmv_destroy(madipm_spmv_t op);

/* MadIPM.coo_to_csr(n_rows, n_cols, Ai, Aj, Ax) (src/utils.jl:158-201; GPU cuda_wrapper.jl:96-106),
 * device arrays, 0-based.  Entries are grouped by row in input order (utils.jl's counting sort);
 * sort_cols != 0 orders each row by column (ties in input order), the layout cuSPARSE produces.
 * Duplicates are kept, as in the reference.  rowptr: n_rows+1.  Synchronises `stream`.
 * An index outside [0, n_rows) x [0, n_cols) is an error (negative return; outputs invalid). */
int madipm_coo_to_csr(int32_t n_rows, int32_t n_cols, int64_t nnz, const int32_t* d_Ai, const int32_t* d_Aj,
                      const double* d_Ax, int32_t* d_rowptr, int32_t* d_colval, double* d_nzval,
                      int32_t sort_cols, madipm_stream_t stream);

/* MadIPM.build_normal_system(n_rows, n_cols, Jtp, Jtj) (src/utils.jl:209-274; the GPU path runs it
 * on host copies too, normalkkt.jl:104): HOST arrays.  Pattern of tril(J J') for J in CSR:
 * column i of the lower CSC (Cp[n_rows+1], Cj) lists the rows j >= i sharing a column with row i,
 * ascending.  *nnz_out always receives the count; Cj (capacity cap) is filled when it is large
 * enough (-4 otherwise); pass Cj = NULL to size it. */
int madipm_build_normal_system(int32_t n_rows, int32_t n_cols, const int32_t* Jtp, const int32_t* Jtj,
                               int32_t* Cp, int32_t* Cj, int64_t cap, int64_t* nnz_out);

/* MadIPM.assemble_normal_system!(n_rows, n_cols, Jtp, Jtj, Jtx, Cp, Cj, Cx, Dx) (src/utils.jl:
 * 276-308; GPU cuda_wrapper.jl:108-156): Cx[c] = sum_k (Jx[i,k] Dx[k]) Jx[j,k] for entry c = (j,
 * column i), merge-joined over each row's ascending column indices (the GPU reference's
 * precondition, which coo_to_csr with sort_cols provides).  Device arrays. */
int madipm_assemble_normal_system(int32_t n_rows, int32_t n_cols, const int32_t* d_Jtp, const int32_t* d_Jtj,
                                  const double* d_Jtx, const int32_t* d_Cp, const int32_t* d_Cj, double* d_Cx,
                                  const double* d_Dx, madipm_stream_t stream);

/* fill_structure!(A::CSR, rows, cols) (MadIPMCUDAExt.jl:15-32; hess_structure!/jac_lin_structure!):
 * rows[c] = i, cols[c] = colval[c] for the entries c of row i. */
int madipm_csr_fill_structure(int32_t n_rows, const int32_t* d_Ap, const int32_t* d_Aj, int32_t* d_rows,
                              int32_t* d_cols, madipm_stream_t stream);

/* NLPModels.obj(qp, x) (MadIPMCUDAExt.jl:34-38): v = H x; obj = c0 + c'x + v'x/2 written to
 * d_work[512] (d_work: 513 doubles of scratch) and, when h_obj != NULL, to *h_obj (synchronises).
 * NLPModels.grad!(qp, x, g) (:40-45): g = H x + c.  H: a symmetric madipm_spmv_t of size n. */
int madipm_qp_obj(madipm_spmv_t H, const double* d_c, double c0, const double* d_x, double* d_v, int32_t n,
                  double* d_work, double* h_obj, madipm_stream_t stream);
int madipm_qp_grad(madipm_spmv_t H, const double* d_c, const double* d_x, double* d_g, int32_t n,
                   madipm_stream_t stream);

/* update_step! (src/kernels.jl:291-358) with get_alpha_max_primal / get_alpha_max_dual
 * (src/kernels.jl:226-272) on DEVICE vectors over the bounded coordinates (the reference's views
 * x_lr, xl_r, zl_r, dx_lr, dual_lb(d) and x_ur, xu_r, zu_r, dx_ur, dual_ub(d)); the same kernels the
 * native MPC loop runs.  rule: 0 ConservativeStep(tau), 1 AdaptiveStep(tau_min = tau; uses mu),
 * 2 MehrotraAdaptiveStep(gamma_f = tau).  The argmin follows the reference's left fold with
 * init (1.0, 0): the LAST index among equal ratios; index -1 = the init element (Julia's 0). */
typedef struct madipm_step_result {
  double alpha_p, alpha_d;                      /* solver.alpha_p / alpha_d after update_step! */
  double alpha_xl, alpha_xu, alpha_zl, alpha_zu; /* the four max-ratio values (tau of the rule) */
  int32_t i_xl, i_xu, i_zl, i_zu;               /* their argmin indices, 0-based */
} madipm_step_result;
int madipm_update_step(int32_t rule, double tau, double mu, int32_t nlb, int32_t nub,
                       const double* d_x_lr, const double* d_xl_r, const double* d_zl_r, const double* d_dx_lr,
                       const double* d_dzl, const double* d_x_ur, const double* d_xu_r, const double* d_zu_r,
                       const double* d_dx_ur, const double* d_dzu, madipm_step_result* out,
                       madipm_stream_t stream);

/* ------------------------------------------------------------------ native MPC solver
 * `MPCSolver(qp; kwargs...)` + `solve!(solver)` (src/structure.jl:79-178, src/solver.jl:362-418)
 * for a QuadraticModel with SparseKKTSystem (K2), run entirely on the GPU with the LDL^T above.
 * All problem arrays are HOST pointers (0-based COO; H = lower triangle). */
typedef struct madipm_qp {
  int32_t nvar, ncon;
  int64_t nnzh, nnzj;
  const double* c;
  double c0;
  const int32_t *Hrows, *Hcols;
  const double* Hvals;
  const int32_t *Arows, *Acols;
  const double* Avals;
  const double *lcon, *ucon, *lvar, *uvar;
  const double *x0, *y0; /* may be NULL (zeros) */
  int32_t minimize;
} madipm_qp;

/* IPMOptions (src/utils.jl:69-105) */
typedef struct madipm_options {
  double tol;                 /* 1e-8 */
  int32_t max_iter;           /* 3000 */
  double max_wall_time;       /* 1e6 */
  double divergence_tol;      /* 1e4 */
  int32_t scaling;            /* 1 */
  double bound_push, bound_fac, bound_relax_factor; /* 1e-2, 1e-2, 1e-12 */
  int32_t regularization;     /* 0 NoRegularization, 1 FixedRegularization, 2 AdaptiveRegularization */
  double delta_p, delta_d, delta_min; /* (1e-10, 1e-10, -) */
  int32_t step_rule;          /* 0 ConservativeStep(tau), 1 AdaptiveStep(tau_min), 2 MehrotraAdaptiveStep(gamma_f) */
  double step_tau;            /* 0.99 */
  int32_t max_ncorr;          /* 0 (Gondzio correctors) */
  double mu_init, mu_min;     /* 1e-1, 1e-12 */
  double tol_linear_solve;    /* 1e-8 */
  int32_t check_residual;     /* 0 */
  int32_t kkt_system;         /* 0 SparseKKTSystem (K2), 1 ScaledSparseKKTSystem (K2.5),
                                 2 NormalKKTSystem (src/KKT/normalkkt.jl; LPs only, Cholesky semantics) */
  int32_t print_level;        /* 0 silent, 1 iteration log to stdout */
  madipm_ldl_opts ldl;
} madipm_options;

/* MadNLP.Status values used by MadIPM */
enum {
  MADIPM_REGULAR = 0,
  MADIPM_SOLVE_SUCCEEDED = 1,
  MADIPM_INFEASIBLE_PROBLEM_DETECTED = 2,
  MADIPM_MAXIMUM_ITERATIONS_EXCEEDED = -1,
  MADIPM_MAXIMUM_WALLTIME_EXCEEDED = -2,
  MADIPM_DIVERGING_ITERATES = -3,
  MADIPM_ERROR_IN_STEP_COMPUTATION = -4,
  MADIPM_INTERNAL_ERROR = -5
};

typedef struct madipm_stats {
  int32_t status, iter;
  double objective;           /* un-scaled, sign-corrected (update_solution!, src/utils.jl:150-156) */
  double dual_objective;
  double inf_pr, inf_du, inf_compl, mu;
  double total_time;          /* MPC loop only, as cnt.total_time (src/solver.jl:181,407) */
  double linear_solver_time;  /* factorizations (GPU events) */
  double init_time;           /* symbolic analysis + initialize! */
  int32_t exception;          /* MADIPM_EXC_*: the exception solve!'s catch-all caught (status INTERNAL_ERROR);
                                 a binding with rethrow_error = true rethrows it (src/solver.jl:398-403) */
} madipm_stats;

/* Exceptions of the MPC loop.  Both end in solve!'s catch-all (src/solver.jl:398-403) as
 * INTERNAL_ERROR: linear_solver.jl:41 throws the TYPE MadNLP.SolveException, which is not
 * `isa MadNLP.LinearSolverException`, and the linear solver's own refusal to solve with an
 * unfactorized matrix (after factorize_regularized_system!'s three failed trials,
 * linear_solver.jl:6-17; LDLFactorizations' ldiv! [EXT]) is not one either. */
enum {
  MADIPM_EXC_NONE = 0,
  MADIPM_EXC_SOLVE = 1,         /* residual NaN, or > tol_linear_solve with check_residual */
  MADIPM_EXC_UNFACTORIZED = 2   /* solve with a failed factorization */
};

typedef struct madipm_iter_trace {
  int32_t k;
  double obj, inf_pr, inf_du, inf_compl, mu, alpha_p, alpha_d, del_w, dx_inf, residual;
} madipm_iter_trace;

typedef struct madipm_solver* madipm_solver_t;
void madipm_default_options(madipm_options* opt);
int madipm_solver_create(const madipm_qp* qp, const madipm_options* opt, madipm_solver_t* out);
/* Sharded across the processes of `comm` (shard = comm rank): every process runs the MPC loop on
 * replicated vectors; the LDL^T is subtree-sharded with RCCL all-reduces (SURVEY §8 e). */
int madipm_solver_create_dist(const madipm_qp* qp, const madipm_options* opt, madipm_comm_t comm,
                              madipm_solver_t* out);
/* initialize! alone (src/solver.jl:127-189); the next solve() then runs only the MPC loop.
 * Without it, solve() initializes first (as solve! does). */
int madipm_solver_initialize(madipm_solver_t s);
int madipm_solver_set_max_iter(madipm_solver_t s, int32_t max_iter);
int madipm_solver_solve(madipm_solver_t s, madipm_stats* stats);
/* any pointer may be NULL: x/zl/zu length nvar, y/cons length ncon (un-scaled, as MadNLP stats) */
int madipm_solver_get_solution(madipm_solver_t s, double* x, double* y, double* zl, double* zu, double* cons);
/* copies up to cap records, returns the number of recorded iterations */
int madipm_solver_trace(madipm_solver_t s, madipm_iter_trace* out, int32_t cap);
int madipm_solver_ldl_info(madipm_solver_t s, madipm_ldl_info* info);
/* fill-reducing pivot order of the K2 factorization (length nvar_std + ncon, K2 unknowns [x; y]) */
int madipm_solver_ldl_perm(madipm_solver_t s, int32_t* perm);
/* the solver's LDL^T: timing as madipm_ldl_set_timing / madipm_ldl_kernel_stats */
int madipm_solver_set_timing(madipm_solver_t s, uint32_t mask);
int madipm_solver_kernel_stats(madipm_solver_t s, madipm_kstat* out);
void madipm_solver_destroy(madipm_solver_t s);

#ifdef __cplusplus
}
#endif

#endif /* MADIPM_HIP_H */
