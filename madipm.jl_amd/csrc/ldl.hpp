// Multifrontal supernodal LDL^T on the GPU (gfx950) — the linear-solver plugin of SURVEY §8 a11/a14.
//
// Replaces `MadNLP.factorize!(kkt.linear_solver)` / `MadNLP.solve!(kkt.linear_solver, x)` for the
// solvers the reference plugs in (LDLFactorizations' LDLSolver, MadNLPGPU's CUDSSSolver with
// cudss_algorithm = LDL, HSL Ma57Solver): called from src/linear_solver.jl:10 and :26 via MadNLP.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "common.hpp"
#include "symbolic.hpp"

namespace madipm {

// the batch range a k_fact_tree task folds and its first batch's table entries, in one record loaded
// with the task's other per-front words (r5: the first batch's entries were a dependent round trip)
struct FoldStart {
  int32_t b0, b1;      // batches [b0, b1)
  int32_t kq0, kq1;    // the first batch's leaves [kq0, kq1) (fold_bat)
  int64_t row0, row1;  // its flat leaf rows (fold_row0)
  int64_t poff;        // its product entries (fold_poff, fold_plen)
  int32_t plen, pad;
};
struct FoldHelp {
  int32_t front, flag;  // the front, the flag the helper publishes
  int64_t img;          // its image in FrontTab::fimg: nimg doubles, entry k = LDS entry fimg_dst[dofs + k]
  int64_t dofs;         // its destinations in FrontTab::fimg_dst (the LDS entries its batches' products reach)
  int32_t nimg, pad;
  FoldStart fs;         // its batches
};

// Device view of the front table (SoA, all device pointers).
struct FrontTab {
  const int32_t* first;
  const int32_t* nrows;
  const int64_t* row_ptr;
  const int32_t* rows;
  const int64_t* l_off;
  const int64_t* u_off;
  const int32_t* u_ld;
  const int64_t* uvec_off;
  const int64_t* asm_ptr;
  const int64_t* asm_src;
  const int64_t* asm_dst;
  const int32_t* child_ptr;
  const int32_t* child_list;
  const int64_t* rel_ptr;
  const int32_t* rel;
  const int32_t* perm;
  const int64_t* fs_off;   // small fronts assembled by k_assemble: r x r scratch offset (else -1)
  const int64_t* sv_ptr;   // forward-solve gather lists (indexed by row_ptr[s] + i)
  const int64_t* sv_src;
  const uint16_t* sv_nt;   // per row: its trailing gather entries from tree tasks (tree solve tables)
  const int32_t* bigslot;  // big front -> slot in the panel-inverse scratch (64x64 per slot)
  // sharding: top fronts start their forward solve from the exchanged vector xch[xoff[s] + i]
  // (xoff = -1 elsewhere); wout[s] = 0 would suppress the write of x to the caller's vector (every
  // shard writes the top x it computes redundantly: all 1)
  const int64_t* xoff;
  const double* xch;
  const uint8_t* wout;
  // tree solves: update entry a of front c goes to gbuf[upos[rel_ptr[c] + a]] when c's parent is a
  // tree front (its contiguous gather range), else to uvec[uvec_off[c] + a] (upos = -1)
  const int64_t* upos;
  double* gbuf;
  // leaf folding (SymbolicPlan::absorb / fold_* / ab_*)
  const uint8_t* absorb;
  const uint8_t* fold_pk;
  const int32_t* mc_ptr;
  const int64_t* ab_first;
  const int32_t* ab_src0;
  const int32_t* ab_src1;
  const int32_t* ab_k;
  const int32_t* ab_f0;
  const int32_t* ab_wrc;
  const int64_t* ab_loff;
  const int32_t* fold_bptr;
  const int32_t* fold_bat;
  const int64_t* fold_row0;
  const int64_t* fold_poff;
  const int32_t* fold_plen;
  const int32_t* fold_rmax;
  const int32_t* fold_lmax;
  const uint32_t* fold_prod;
  const uint32_t* fold_chead;
  const uint8_t* fs_img;  // 1: fscratch holds the front's LDS image (tree fronts), else ld r
  int32_t* err;     // the status block's sticky error (LDLStatus::err): a timed-out hand-off inside a front
  int fpipe;        // pipelined in-LDS schedule (blocked_factor_pipe; MADIPM_FACT_PIPE=0: blocked_factor_lds)
  int pipe_fault;   // tests (MADIPM_DEBUG_PIPE_FAULT=1): blocked_factor_pipe drops one hand-off
  int lds_cap;      // k_fact_tree's dynamic LDS (bytes): a front (+ its leaf batches) beyond it is an error
  int asm_src_cap;  // assembly LDS source path: a tile of more sources is an error (kErrAsmSrc); tests shrink it
  // fold helpers (k_fact_tree tickets before the fronts): a helper folds the first batches of a front's
  // micro leaves into a zeroed LDS image and hands it over in HBM (fimg); the front folds the rest
  // from fstart[s] and adds the image after its waits (fold_help[s] = the helper, -1: none)
  const FoldStart* fstart;  // per front: the batches it folds itself
  const int32_t* fold_help;
  const FoldHelp* fhelp;
  double* fimg;
  const uint16_t* fimg_dst;  // per helper: the sorted LDS destinations of its products (FoldHelp::dofs)
  uint64_t* xll;  // big-front solves: panel solutions as self-validating words (ll_put / ll_get)
};

// LDLStatus::err bits (sticky; status() raises on any)
constexpr int32_t kErrHandoff = 1;   // a dependency hand-off (flag poll) timed out
constexpr int32_t kErrLdsCarve = 2;  // a k_fact_tree front or leaf batch did not fit its LDS carve
constexpr int32_t kErrAsmSrc = 4;    // an assembly tile on the LDS source path has more sources than its windows

// assembly: a big child's block on one 64x64 tile of its parent (SymbolicPlan::bt entry, split by
// column ranges so that na * nb <= kBigRecEntries).  The child's update rows on the tile are the
// consecutive rows a0 .. a0 + na - 1 (its rows are a sorted subset of the parent's), its columns
// b0 .. b0 + nb - 1; rows[i] / cols[j] = their tile row / column.  Entry e < na nb of the record is
// (i, j) = (e mod na, e div na), e div na = (e * na_inv) >> 16 (exact for e < 1024, na <= 64).
constexpr int kBigRecEntries = 1024;
struct BigChildRec {
  int64_t u_off;
  int32_t u_ld, a0, b0;
  uint16_t na, nb;
  uint32_t na_inv, pad;
  uint8_t rows[64], cols[64];
};

struct SolveTask {
  int32_t front, blk;
};

// a micro leaf (w <= 2, r <= 32, no children) folded into a tree-solve chain task: its L panel, first
// pivot, r | w << 8, the caller's indices of its two pivots, and the offset of its below rows' entries
// in the row table (int2: gbuf position of the forward update entry, xi index of the row)
struct SolveLeaf {
  int64_t loff;
  int32_t f0, rw, p0, p1, roff, pad;
};

struct LDLStatus {  // device-resident, read back by status()
  int32_t fail_pivot;  // min failing internal pivot + 1 (INT32_MAX when none)
  int32_t npos, nneg, nzero;
  int32_t err;  // sticky: a dependency hand-off (flag poll) timed out in a factorisation or solve
  int32_t pad_;
  // device wall clock (wall_clock64, hipDeviceAttributeWallClockRate): t0 at the start of the latest
  // factorisation, t1 at its end; ticks = the sum over the earlier ones (folded in by the next start)
  uint64_t t0, t1, ticks;
};

// Start of a factorisation (k_status_init's work; one thread): fold the previous factorisation's
// time in, stamp t0, clear the pivot check and the inertia counts.  A caller whose own kernel runs
// right before the factorisation does this itself (LinSolver::ext_reset) and saves that launch.
__device__ __forceinline__ void ldl_status_start(LDLStatus* st) {
  const uint64_t now = wall_clock64();
  if (st->t1 > st->t0) st->ticks += st->t1 - st->t0;
  st->t0 = st->t1 = now;
  st->fail_pivot = INT32_MAX;
  st->npos = st->nneg = st->nzero = 0;
}
// end of a factorisation whose inertia is counted lazily (LinSolver::lazy_inertia): stamp t1
__device__ __forceinline__ void ldl_status_end(LDLStatus* st) { st->t1 = wall_clock64(); }

// Kernel kinds for the live per-kernel timing (HIP events around each launch on the launch
// stream) and their algorithmic bytes / flops per launch (DESIGN.md "Kernels and their rooflines").
enum KernelKind {
  KK_ASM_CHUNKS = 0, KK_ASSEMBLE, KK_TINY, KK_SMALL, KK_DIAG, KK_TRSM, KK_UPDATE, KK_INERTIA,
  KK_FWD_SMALL, KK_FWD_GATHER, KK_FWD_BIG, KK_BWD_BELOW, KK_BWD_BIG, KK_BWD_SMALL, KK_FWD_TINY, KK_BWD_TINY,
  KK_LB_BUILD, KK_LB_SYRK, KK_LB_GEMV, KK_FWD_TREE, KK_BWD_TREE, KK_FACT_TREE, KK_ASM_UPDATE, KK_BIG_DAG,
  KK_COUNT
};
const char* kernel_kind_name(int k);

struct KernelStat {
  int64_t launches = 0;
  double ms = 0.0, bytes = 0.0, flops = 0.0;
  double alg_bytes = 0.0;  // SURVEY 8(d)'s bytes of the launches (8 nnzL + 12 nnzK of the columns factorised,
                           // 8 nnzL of the columns a solve launch substitutes); `bytes` = the staging model
};

// All-reduce (sum) of a device buffer across the shards of a sharded factorisation, ordered on
// `s`.  RcclComm (csrc/comm.cpp) is the multi-GPU implementation (RCCL over xGMI).
struct Comm {
  int rank = 0, size = 1;
  virtual ~Comm() = default;
  virtual void allreduce_sum(double* buf, int64_t n, hipStream_t s) = 0;
  // In-place all-gather of `size` slices of nper doubles: rank q's slice is buf[q nper, (q+1) nper)
  // and the other slices are zero on entry, so a sum all-reduce of the whole buffer is a valid (twice
  // as heavy) implementation — the default, for communicators without a gather (HostComm).
  virtual void allgather_inplace(double* buf, int64_t nper, hipStream_t s) { allreduce_sum(buf, nper * size, s); }
};
Comm* make_rccl_comm(int nranks, int rank, const void* unique_id /* 128 bytes */);
void rccl_unique_id(void* out /* 128 bytes */);
Comm* make_host_comm(int nranks, int rank, int (*fn)(double*, int64_t, void*), void* ctx);

// Linear-solver interface the MPC driver uses (MadNLP.AbstractLinearSolver methods).
class LinSolver {
 public:
  virtual ~LinSolver() = default;
  virtual void factorize_async(const double* Kx, hipStream_t s) = 0;
  // sync = false: the caller already waited for an event recorded after factorize_async
  virtual int status(hipStream_t s, bool sync = true) = 0;
  // Keep the factorisation status at caller-provided device / pinned-host addresses, so the caller's
  // own per-iteration read-back carries it (no separate copy); status(s, false) then reads the
  // caller's copy.  Returns false when unsupported (sharded solvers).
  virtual bool external_status(LDLStatus* dev, LDLStatus* host) {
    (void)dev;
    (void)host;
    return false;
  }
  virtual void solve_async(double* b, hipStream_t s) = 0;
  virtual const SymbolicPlan& plan() const = 0;
  virtual void set_timing(unsigned mask) = 0;
  virtual void kernel_stats(KernelStat out[]) = 0;
  virtual int n() const = 0;
  // doubles all-reduced per factorisation / per solve, and all-gathered per solve (the whole
  // buffer, nshards slices) — 0 unsharded
  virtual int64_t xch_fact() const { return 0; }
  virtual int64_t xch_solve() const { return 0; }
  virtual int64_t xch_gather() const { return 0; }
  // seconds of device time spent in factorisations so far (synchronises s; cnt.linear_solver_time)
  virtual double fact_seconds(hipStream_t s) = 0;
  bool spd = false;  // Cholesky semantics: any non-positive pivot fails (normal equations)
  // launch savings for a driver that owns the kernels around the factorisation (MPCSolver):
  //   ext_reset: the driver's kernel right before every factorisation runs ldl_status_start on the
  //     status block (external_status) — no k_status_init launch;
  //   lazy_inertia: no k_inertia after the factorisation (the driver's next kernel runs
  //     ldl_status_end); the pivot check does not need it unless spd, and inertia() counts on demand
  bool ext_reset = false, lazy_inertia = false;
  virtual void count_inertia(hipStream_t s) { (void)s; }
  // The factorisation's tail (an elimination-tree root factorised after the tree launch, LDLSolver::
  // root_async_) may run on a side stream after factorize_async returns, beside the next solve's
  // forward leaves and tree fronts.  join(s) orders s after it; solve_async, status(s, true),
  // count_inertia and fact_seconds join by themselves.  With tail_async() the status carried by a
  // kernel enqueued right after factorize_async is not final: read it after the next solve.
  virtual bool tail_async() const { return false; }
  virtual void join(hipStream_t s) { (void)s; }
};

// k_root_solve's fronts (up to kRootArgs) by value: their shapes come with the launch instead of two
// dependent table loads (front id, then first / nrows / row_ptr / l_off) before the gather
constexpr int kRootArgs = 4;
struct RootArgs {
  int32_t n;
  int32_t s[kRootArgs], f0[kRootArgs], w[kRootArgs], r[kRootArgs];
  int64_t e0[kRootArgs], loff[kRootArgs];
};

class LDLSolver : public LinSolver {
 public:
  LDLSolver(int n, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& sopt,
            double pivot_tol, const int32_t* user_perm = nullptr, Comm* comm = nullptr);
  ~LDLSolver();
  LDLSolver(const LDLSolver&) = delete;
  LDLSolver& operator=(const LDLSolver&) = delete;

  // Enqueue the numeric factorisation of the values `Kx` (device, caller's CSC order) on `s`.
  // Sharded: phase 1, all-reduce of the top fronts (comm), phase 2.
  void factorize_async(const double* Kx, hipStream_t s) override;
  // Synchronise `s` and return 0 or failing pivot + 1; fills the inertia.
  int status(hipStream_t s, bool sync = true) override;
  bool external_status(LDLStatus* dev, LDLStatus* host) override;
  // In-place solve K x = b for a device vector of length n (caller's ordering).
  void solve_async(double* b, hipStream_t s) override;

  // Phases of a sharded factorisation / solve, for callers that run their own collective
  // (ShardGroup below, or a host binding with its own RCCL communicator):
  //   factorize: fact_phase1; all-reduce fact_xbuf(); fact_phase2
  //   solve:     solve_phase1; all-reduce solve_xbuf(); solve_phase2; all-gather solve_gbuf()
  //              (nshards slices of solve_gper(); this shard's slice filled, the others zero);
  //              solve_phase3
  void fact_phase1(const double* Kx, hipStream_t s);
  void count_inertia(hipStream_t s) override;  // lazy_inertia: the counts of the current factor
  void fact_phase2(hipStream_t s);
  void solve_phase1(double* b, hipStream_t s);
  void solve_phase2(double* b, hipStream_t s);
  void solve_phase3(double* b, hipStream_t s);
  double* fact_xbuf() const { return xpack_.p; }  // the top fronts' lower triangles + status slots
  int64_t fact_xlen() const { return S_.nshards > 1 ? xpack_tri_ + 4 * S_.nshards : 0; }
  double* solve_xbuf() const { return xch_.p; }
  int64_t solve_xlen() const { return S_.nshards > 1 ? S_.xlen : 0; }
  double* solve_gbuf() const { return gsol_.p; }
  int64_t solve_gper() const { return gper_; }  // doubles per shard slice of solve_gbuf()
  bool sharded() const { return S_.nshards > 1; }
  int64_t xch_fact() const override { return fact_xlen(); }
  int64_t xch_solve() const override { return sharded() ? solve_xlen() : 0; }
  int64_t xch_gather() const override { return sharded() ? S_.nshards * gper_ : 0; }
  double fact_seconds(hipStream_t s) override;
  bool tail_async() const override { return root_async_; }
  void join(hipStream_t s) override;

  const SymbolicPlan& plan() const override { return S_; }
  int n() const override { return S_.N; }
  int npos = 0, nneg = 0, nzero = 0;
  bool factorized = false;
  double pivot_tol = 0.0;

  // device buffers for diagnostics
  const double* d_diag() const { return D_.p; }

  // live kernel timing: bit k of `mask` => HIP events around every launch of KernelKind k.
  // set_timing() clears the accumulated statistics; kernel_stats() synchronises the events.
  void set_timing(unsigned mask) override;
  void kernel_stats(KernelStat out[KK_COUNT]) override;

 private:
  enum Kind { ASSEMBLE = 0, SMALL32 = 1, SMALL64 = 2, SMALL128 = 3, BIG_DIAG = 4, BIG_TRSM = 5, BIG_UPDATE = 6,
              LB_BUILD = 7, LB_SYRK = 8, MICRO = 9, SMALL192 = 10, FTREE = 11, BIG_UPDATE128 = 12,
              ASM_UPDATE = 13, BIG_DAG = 14 };
  struct Launch {
    int kind;
    int step;       // panel step for BIG_DIAG / BIG_TRSM / BIG_UPDATE
    int64_t off;    // ASSEMBLE: first tile; SMALL*: front list in sched_; BIG_*: (front, item) pairs in sched_
    int nf;         // number of fronts (SMALL*)
    int64_t items;  // workgroups
    int64_t chunk0 = 0, nchunk = 0;  // ASSEMBLE: chunk range of the level
    double bytes = 0, flops = 0;       // staging traffic model / algorithmic work of the launch
    double alg = 0;                    // SURVEY 8(d) bytes of the columns the launch factorises
    double bytes2 = 0, flops2 = 0;     // ASSEMBLE: of the chunk pass
    bool lds = true;                   // SMALL*: some front is a leaf (assembled in LDS)
    int lds_bytes = 0;                 // SMALL*: dynamic LDS of the blocked kernel (largest front)
  };
  struct SolveLevel {
    int64_t tiny_off;  // fronts with r <= 32 (half a wave each)
    int ntiny;
    int64_t micro_off;  // fronts with r <= 32, w <= 2 (16 lanes each)
    int nmicro;
    double micro_bytes = 0, micro_flops = 0, micro_alg = 0;
    int64_t small_off;
    int nsmall;
    int64_t big_off;
    int nbig;
    int64_t gat_off;  // (front, 256-row chunk) pairs for k_fwd_gather
    int ngat;
    int64_t below_off;  // (front, panel | chunk << 16) pairs for k_bwd_below
    int nbelow;
    int64_t ftask_off;
    int nftask;
    int64_t btask_off;
    int nbtask;
    int small_lds = 0;  // dynamic LDS of the small-front solve kernels (largest panel, ld r | 1)
    double tiny_bytes = 0, tiny_flops = 0;
    double small_bytes = 0, small_flops = 0, big_bytes = 0, big_flops = 0, below_bytes = 0, gat_bytes = 0;
    // SURVEY 8(d) bytes per direction: 8 nnzL of the fronts' columns (big: diagonal block / below it)
    double tiny_alg = 0, small_alg = 0, big_alg = 0, below_alg = 0;
  };
  SymbolicPlan S_;
  FrontTab T_{};
  Comm* comm_ = nullptr;
  std::vector<Launch> fact1_, fact2_;      // phase 1 (this shard's subtrees; everything unsharded), phase 2 (top)
  std::vector<SolveLevel> slev1_, slev2_;  // per level, leaves first
  int64_t xg_off_ = 0;                     // (top front, 256-row chunk) pairs of the external forward gather
  int nxg_ = 0;
  // launches [b, e) of L on s; stamp: SMALL* launches stamp the factorisation's end into it
  void run_fact(const std::vector<Launch>& L, const double* Kx, hipStream_t s, size_t b = 0, size_t e = SIZE_MAX,
                LDLStatus* stamp = nullptr);
  // the root tail on a side stream (MADIPM_ROOT_ASYNC, default on): fact1_[side0_] (the last launch)
  // factorises elimination-tree roots that only k_root_solve reads.  It is enqueued on side_ and waits
  // on the device for rflag_[0] == repoch_ (raised by the roots' assembly, fact1_[side0_ - 1], on the
  // caller's stream), then raises rflag_[2 + k] for k_root_solve; ev_join_ (recorded after it) joins
  // the host-side users (status, fact_seconds, a factorisation no solve followed)
  bool root_async_ = false, root_pending_ = false, untimed_ = false;
  bool asm_side_ = false, side_phase_ = false;  // the roots' assembly tiles on side_ too; run_fact is enqueuing side_'s part
  size_t side0_ = 0;
  int nroot_side_ = 0, repoch_ = 0;
  bool side_tree_ = false;  // some side root is solved by its k_fwd_tree task (tside_), not k_root_solve
  DBuf<int32_t> rflag_;
  DBuf<uint8_t> tside_;
  hipStream_t side_ = nullptr;
  hipEvent_t ev_join_ = nullptr;
  void fwd_levels(const std::vector<SolveLevel>& V, int phase, double* b, hipStream_t s);
  void bwd_levels(const std::vector<SolveLevel>& V, int phase, double* b, hipStream_t s);
  DBuf<int64_t> xoff_, sx_ptr_, sx_src_;
  // batched leaf columns (SymbolicPlan::lb): W, pivots, member tables, per-level launch lists
  DBuf<double> lbW_, lbd_, lbpart_;
  DBuf<int32_t> lbmem_, lbgid_, lbwrow_, lbgpos_, lbxrow_;
  DBuf<int64_t> lbcs_, lbce_, lbwbase_, lbpoff_;
  DBuf<SymbolicPlan::LBGroup> lbg_;
  std::vector<std::vector<int>> lb_at_level_;
  void lb_syrk(int g, hipStream_t s);
  void lb_fwd(const double* b, hipStream_t s);
  void lb_bwd(int g, double* b, hipStream_t s);
  // tree solves (k_fwd_tree / k_bwd_tree): the phase-1 fronts solved by ONE dependency-driven launch
  // per direction (topological ticket order, forward dependencies = tree children, backward = tree
  // parent), between the level-0 launches and the remaining levels
  int ntree_ = 0, tree_lds_ = 0;
  double tree_bytes_ = 0, tree_flops_ = 0, tree_alg_ = 0;
  // SURVEY 8(d) bytes of front s: factorisation 8 nnzL + 12 nnzK of its columns; solve 8 nnzL
  double fact_alg(int s) const;
  double fact_alg_cols(int c0, int c1) const;
  double solve_alg(int s) const;
  double lb_alg(size_t g) const;
  DBuf<int32_t> tc_ptr_, tc_list_, tdep_ptr_, tdep_, tpar_, tflags_;
  DBuf<uint8_t> trootbwd_;  // per forward task: an elimination-tree root solved backward by k_fwd_tree
  int nroot_task_ = 0, root_lds_ = 0;  // tree-solve tasks of big etree roots (last, own forward launch)
  RootArgs rargs_{};                   // their fronts' shapes, passed by value to k_root_solve
  DBuf<uint8_t> tchunk_;    // per front: tree solves stream its panel in chunks (fwd_med_front / bwd_med_front)
  int ntask_ = 0;         // tree-solve tasks (one per tree front)
  int64_t nsleaf_ = 0;    // micro leaves solved from leaf records by the flat leaf launches
  double leaf_bytes_ = 0, leaf_flops_ = 0, leaf_alg_ = 0;  // the flat leaf launches (per direction)
  DBuf<SolveLeaf> tleaf_;
  DBuf<int2> tlrow_;
  DBuf<int64_t> tdbg_, upos_;
  DBuf<double> gbuf_;
  void tree_debug_dump(hipStream_t s, const char* what, const int64_t* dbuf, int nt, const char* p1, const char* p2,
                       const char* p3, const char* p4, const char* p5, int stride);
  // factorisation tree (k_fact_tree): fronts in topological order, their tree children, flags
  // (per-factorisation epoch), ticket counters (reset by the launch's last workgroup)
  int nftree_ = 0, ftree_lds_ = 0, fepoch_ = 0;
  bool ftree_checked_ = false;
  double ftree_bytes_ = 0, ftree_flops_ = 0, ftree_alg_ = 0;
  DBuf<int32_t> ft_order_, ft_dptr_, ft_dep_, fflags_, fcnt_;
  DBuf<uint64_t> xll_;
  DBuf<uint16_t> sv_nt_;
  DBuf<int64_t> fdbg_, ab_first_, ab_loff_, fold_poff_, fold_row0_;
  int big_kpan_ = 4;  // big fronts: panels per deferred trailing-update group (MADIPM_BIG_KPAN)
  bool big_dag_ = true;  // a level's big fronts in one k_big_dag launch (MADIPM_BIG_DAG=0: per panel step and kind)
  DBuf<int32_t> dag_tasks_;  // DagTask (4 int32) per task of every DAG launch, in launch order
  DBuf<int32_t> dag_dptr_;   // per task: its first dependency in dag_dlist_ (launch-local tickets), + end
  DBuf<int32_t> dag_dlist_;
  DBuf<int32_t> dag_flags_;  // per task: the epoch of the factorisation that completed it
  DBuf<int32_t> dag_cnt_;    // ticket + done counters (reset by the last workgroup out)
  DBuf<double> dag_m_;       // M_K blocks per (big front, panel)
  DBuf<int64_t> dag_mslot_;  // per front: its first panel's slot in dag_m_
  int cepoch_ = 0;
  int dag_grid_ = 256;
  DBuf<int64_t> dag_dbg_;          // MADIPM_DAG_DEBUG: 4 stamps per task
  std::vector<int32_t> dag_kind_;  // (its host copy of the task words)
  void dag_debug_dump(hipStream_t s, const Launch& L);
  bool upd_split_ = true;  // k_big_upd128 split K on launches of few tiles (MADIPM_UPD_SPLIT=0: off)
  DBuf<double> upsum_;    // its partial products
  DBuf<int32_t> uptick_;  // its per-tile tickets (reset by each tile's last part)
  int big_solve_wg_ = 512;
  DBuf<int32_t> ab_src0_, ab_src1_, ab_k_, ab_f0_, ab_wrc_, fold_bptr_, fold_bat_, fold_plen_, fold_rmax_, fold_lmax_;
  DBuf<FoldStart> fstart_;
  DBuf<int32_t> fold_help_;
  DBuf<FoldHelp> fhelp_;
  DBuf<double> fimg_;
  DBuf<uint16_t> fimg_dst_;
  int nfhelp_ = 0;  // fold helper tickets (k_fact_tree: before the fronts')
  DBuf<uint8_t> absorb_, fold_pk_, fs_img_;
  DBuf<int32_t> mc_ptr_;
  DBuf<uint32_t> fold_prod_, fold_chead_;
  DBuf<double> xch_;
  DBuf<double> xpack_;     // sharded: packed top-front lower triangles (+ status slots), all-reduced
  DBuf<int64_t> topcol_;   // per top-front column: arena offset, packed offset, length
  int ntopcol_ = 0;
  int64_t xpack_tri_ = 0;
  DBuf<uint8_t> wout_, colmask_;
  // sharded solve: caller positions of every shard's subtree columns, nshards slices of gper_
  // (padding -1), and the gathered solution slices
  DBuf<int32_t> gidx_;
  DBuf<double> gsol_;
  int64_t gper_ = 0;
  DBuf<int32_t> tasks_, flags_, flag_off_, counters_, bp_off_;
  DBuf<double> bpart_;
  int epoch_ = 0;
  // device data
  DBuf<int32_t> first_, nrows_, rows_, u_ld_, child_ptr_, child_list_, rel_, perm_, sched_;
  DBuf<int32_t> bigslot_, g_ptr_;
  DBuf<BigChildRec> brec_;
  DBuf<int64_t> fs_off_, sv_ptr_, sv_src_, g_src_, g_chunk_, chunk_ids_;
  DBuf<int32_t> g_src32_;
  DBuf<SymbolicPlan::AsmTile> atiles_;
  DBuf<double> minv_, fscratch_, gpart_;
  DBuf<int64_t> row_ptr_, l_off_, u_off_, uvec_off_, asm_ptr_, asm_src_, asm_dst64_, rel_ptr_;
  DBuf<double> arena_, D_, xi_, uvec_, vwork_;
  DBuf<LDLStatus> status_;
  LDLStatus* h_status_ = nullptr;
  LDLStatus* st_ = nullptr;    // status in use: status_ or the caller's (external_status)
  LDLStatus* h_st_ = nullptr;  // its host copy
  bool ext_status_ = false;
  bool inertia_stale_ = false;  // lazy_inertia: npos / nneg / nzero not counted for the current factor
  // live timing
  unsigned tmask_ = 0;
  std::vector<hipEvent_t> evs_;
  size_t ev_used_ = 0;
  struct Pending {
    int kind;
    size_t e0;
    double bytes, flops, alg;
  };
  std::vector<Pending> pend_;
  KernelStat kst_[KK_COUNT];
  bool t_begin(int kind, hipStream_t s);
  void t_end(int kind, hipStream_t s, double bytes, double alg, double flops);
};

// The shards of one sharded factorisation on ONE device (single process): the phases run shard by
// shard and the all-reduces are a device kernel over the shards' buffers (local_allreduce).  It runs
// the whole sharded data path of SURVEY §8 e on one GPU; across GPUs each process owns one
// LDLSolver shard with an RcclComm instead.
class ShardGroup : public LinSolver {
 public:
  ShardGroup(int nshards, int n, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& sopt,
             double pivot_tol, const int32_t* user_perm = nullptr);
  void factorize_async(const double* Kx, hipStream_t s) override;
  int status(hipStream_t s, bool sync = true) override;
  void solve_async(double* b, hipStream_t s) override;
  const SymbolicPlan& plan() const override { return sh_[0]->plan(); }
  void set_timing(unsigned mask) override { sh_[0]->set_timing(mask); }
  void kernel_stats(KernelStat out[]) override { sh_[0]->kernel_stats(out); }
  int n() const override { return sh_[0]->n(); }
  int64_t xch_fact() const override { return sh_[0]->xch_fact(); }
  int64_t xch_solve() const override { return sh_[0]->xch_solve(); }
  int64_t xch_gather() const override { return sh_[0]->xch_gather(); }
  double fact_seconds(hipStream_t s) override { return sh_[0]->fact_seconds(s); }
  LDLSolver& shard(int r) { return *sh_[r]; }
  int nshards() const { return (int)sh_.size(); }

 private:
  std::vector<std::unique_ptr<LDLSolver>> sh_;
  std::vector<DBuf<double>> rhs_;
};

// bufs[q][i] <- sum_{q' in order} bufs[q'][i] for every q (q = 0..nbuf-1, nbuf <= 16)
void local_allreduce(double* const* bufs, int nbuf, int64_t n, hipStream_t s);

}  // namespace madipm
