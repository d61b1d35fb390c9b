// extern "C" entry points of libmadipm_hip.so (declared in include/madipm_hip.h).
// Every entry point catches C++ exceptions and converts them to a negative return code plus
// madipm_last_error() text.
#include <cstring>
#include <memory>
#include <string>

#include "../../include/madipm_hip.h"
#include "common.hpp"
#include "ldl.hpp"
#include "mpc.hpp"
#include "symbolic.hpp"

namespace madipm {
namespace {
thread_local std::string g_last_error;
}
void set_last_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }
}  // namespace madipm

using namespace madipm;

#define MADIPM_API_BEGIN try {
#define MADIPM_API_END                                   \
  }                                                      \
  catch (const madipm::Error& e) {                       \
    set_last_error(e.what());                            \
    return e.code < 0 ? e.code : -1;                     \
  }                                                      \
  catch (const std::exception& e) {                      \
    set_last_error(std::string("exception: ") + e.what()); \
    return -1;                                           \
  }                                                      \
  catch (...) {                                          \
    set_last_error("unknown exception");                 \
    return -1;                                           \
  }

struct madipm_symbolic {
  SymbolicPlan plan;
};

struct madipm_solver {
  std::unique_ptr<MPCSolver> s;
};

struct madipm_ldl {
  std::unique_ptr<LDLSolver> own;  // unsharded, or one shard of a cross-process sharded factorisation
  std::unique_ptr<ShardGroup> g;   // ldl.nshards > 1: all shards on this device
  LDLSolver* s = nullptr;          // the (first) shard: plan, inertia, status flags
  LinSolver* lin = nullptr;        // factorize / solve entry
  hipStream_t last_stream = nullptr;
  bool pending = false;
  // sharded solve protocol (ABI 0.2): the phase the next madipm_ldl_solve_phase call must be (1 when
  // idle).  Phase 2 returns the all-gather buffer and phase 3 is required — a binding that follows the
  // 0.1 protocol (phase 2, then an all-reduce of x) is refused at its next call instead of silently
  // getting a wrong x
  int solve_next = 1;
};
static void require_idle(const madipm_ldl* ls) {
  MADIPM_REQUIRE(ls->solve_next == 1, "sharded solve protocol: phase " + std::to_string(ls->solve_next) +
                                          " of madipm_ldl_solve_phase is pending (phase 2 returns the gather "
                                          "buffer, phase 3 scatters it: ABI 0.2)");
}

struct madipm_comm {
  std::unique_ptr<Comm> c;
};

static SymbolicOptions to_sym_opts(const madipm_ldl_opts* o) {
  SymbolicOptions s;
  if (o) {
    s.ordering = o->ordering;
    s.dense_alpha = o->dense_alpha;
    s.relax = o->relax;
    s.small_front_max = o->small_front_max;
  }
  MADIPM_REQUIRE(!o || (o->nshards >= 1 && o->nshards <= 16), "nshards must be in [1,16]");
  MADIPM_REQUIRE(s.small_front_max >= 1 && s.small_front_max <= 192, "small_front_max must be in [1,192]");
  return s;
}

extern "C" {

int madipm_version(void) { return 203; }  // 0.2.3: madipm_ldl_info.root_tail_async (0.2.2: MADIPM_NKERNELS 24)

const char* madipm_last_error(void) { return last_error(); }

int madipm_set_device(int32_t dev) {
  MADIPM_API_BEGIN
  MADIPM_HIP(hipSetDevice(dev));
  // the runtime's one-off device set-up now (context, and the first stream of the process: 0.14 s on
  // the box), not inside the first solver construction — as the reference's CUDA initialisation
  // happens in its host-to-device conversion of the QP, before MPCSolver (benchmarks_gpu.jl:33-37)
  MADIPM_HIP(hipFree(nullptr));
  hipStream_t s = nullptr;
  MADIPM_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  MADIPM_HIP(hipStreamDestroy(s));
  return 0;
  MADIPM_API_END
}

int madipm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void madipm_ldl_default_opts(madipm_ldl_opts* o) {
  if (!o) return;
  o->ordering = 4;
  o->dense_alpha = 10.0;
  o->relax = 1;
  o->small_front_max = 128;
  o->pivot_tol = 0.0;
  o->nshards = 1;
  o->cholesky = 0;
}

int madipm_symbolic_analyze(int32_t n, const int64_t* colptr, const int32_t* rowval,
                            const madipm_ldl_opts* opts, const int32_t* user_perm,
                            madipm_symbolic_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out != nullptr && colptr != nullptr, "null argument");
  auto s = std::make_unique<madipm_symbolic>();
  symbolic_analyze(n, colptr, rowval, to_sym_opts(opts), user_perm, s->plan);
  *out = s.release();
  return 0;
  MADIPM_API_END
}

int madipm_symbolic_analyze_shard(int32_t n, const int64_t* colptr, const int32_t* rowval,
                                  const madipm_ldl_opts* opts, int32_t nshards, int32_t shard,
                                  const int32_t* user_perm, madipm_symbolic_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out != nullptr && colptr != nullptr, "null argument");
  SymbolicOptions so = to_sym_opts(opts);
  so.nshards = nshards;
  so.shard = shard;
  auto s = std::make_unique<madipm_symbolic>();
  symbolic_analyze(n, colptr, rowval, so, user_perm, s->plan);
  *out = s.release();
  return 0;
  MADIPM_API_END
}

int madipm_symbolic_shard_info(madipm_symbolic_t sym, int32_t* owner, double* top_cost, double* shard_cost_max,
                               double* shard_cost_sum) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(sym, "null handle");
  const SymbolicPlan& p = sym->plan;
  if (owner)
    for (int s = 0; s < p.nsuper; ++s) owner[s] = p.owner.empty() ? 0 : p.owner[s];
  if (top_cost) *top_cost = p.top_cost;
  if (shard_cost_max) *shard_cost_max = p.shard_cost_max;
  if (shard_cost_sum) *shard_cost_sum = p.shard_cost_sum;
  return 0;
  MADIPM_API_END
}

// madipm_ldl_info from a plan (+ the device solver for the exchange sizes, when there is one)
static void fill_info(const SymbolicPlan& p, const LinSolver* ls, madipm_ldl_info* info) {
  info->n = p.N;
  info->nnzK = p.nnzK;
  info->nnzL = p.nnzL;
  info->nnzL_stored = p.nnzL_super;
  info->flops = p.flops;
  info->nsuper = p.nsuper;
  info->nlevels = p.nlevels;
  info->max_front = p.max_front;
  info->nbig = p.nbig;
  info->arena_bytes = p.arena_size * 8 + p.lb_wsize * 8;
  info->lb_groups = (int32_t)p.lb.size();
  info->lb_members = (int32_t)p.lb_mem.size();
  info->fold_fronts = 0;
  for (uint8_t a : p.absorb) info->fold_fronts += a;
  info->fold_leaves = (int32_t)p.mc_list.size();
  info->xch_fact = ls ? ls->xch_fact() : 0;
  info->xch_solve = ls ? ls->xch_solve() : 0;
  info->xch_gather = ls ? ls->xch_gather() : 0;
  info->tree_fronts = info->tree_medium = 0;
  for (int s = 0; s < (int)p.ftree.size(); ++s)
    if (p.ftree[s]) {
      ++info->tree_fronts;
      info->tree_medium += p.nrows[s] > SymbolicPlan::kFactTreeMax;
    }
  info->root_tail_async = ls && ls->tail_async() ? 1 : 0;
  info->pad_ = 0;
}

int madipm_symbolic_info(madipm_symbolic_t sym, madipm_ldl_info* info) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(sym && info, "null argument");
  fill_info(sym->plan, nullptr, info);
  return 0;
  MADIPM_API_END
}

int madipm_symbolic_perm(madipm_symbolic_t sym, int32_t* perm) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(sym && perm, "null argument");
  std::memcpy(perm, sym->plan.perm.data(), sizeof(int32_t) * sym->plan.perm.size());
  return 0;
  MADIPM_API_END
}

int madipm_symbolic_supernodes(madipm_symbolic_t sym, int32_t* first, int32_t* parent, int32_t* nrows) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(sym, "null argument");
  const SymbolicPlan& p = sym->plan;
  if (first) std::memcpy(first, p.first.data(), sizeof(int32_t) * p.first.size());
  if (parent) std::memcpy(parent, p.parent.data(), sizeof(int32_t) * p.parent.size());
  if (nrows) std::memcpy(nrows, p.nrows.data(), sizeof(int32_t) * p.nrows.size());
  return 0;
  MADIPM_API_END
}

void madipm_symbolic_destroy(madipm_symbolic_t sym) { delete sym; }

// ------------------------------------------------------------------ LDL^T plugin
int madipm_ldl_analyze(int32_t n, const int64_t* colptr, const int32_t* rowval, const madipm_ldl_opts* opts,
                       const int32_t* user_perm, madipm_ldl_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out != nullptr && colptr != nullptr, "null argument");
  madipm_ldl_opts o;
  madipm_ldl_default_opts(&o);
  if (opts) o = *opts;
  auto ls = std::make_unique<madipm_ldl>();
  if (o.nshards > 1) {
    ls->g = std::make_unique<ShardGroup>(o.nshards, n, colptr, rowval, to_sym_opts(&o), o.pivot_tol, user_perm);
    ls->s = &ls->g->shard(0);
    ls->lin = ls->g.get();
  } else {
    ls->own = std::make_unique<LDLSolver>(n, colptr, rowval, to_sym_opts(&o), o.pivot_tol, user_perm);
    ls->s = ls->own.get();
    ls->lin = ls->s;
  }
  ls->lin->spd = o.cholesky != 0;
  if (ls->g)
    for (int q = 0; q < ls->g->nshards(); ++q) ls->g->shard(q).spd = ls->lin->spd;
  *out = ls.release();
  return 0;
  MADIPM_API_END
}

int madipm_ldl_analyze_shard(int32_t n, const int64_t* colptr, const int32_t* rowval, const madipm_ldl_opts* opts,
                             int32_t nshards, int32_t shard, const int32_t* user_perm, madipm_ldl_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out != nullptr && colptr != nullptr, "null argument");
  madipm_ldl_opts o;
  madipm_ldl_default_opts(&o);
  if (opts) o = *opts;
  o.nshards = 1;
  SymbolicOptions so = to_sym_opts(&o);
  so.nshards = nshards;
  so.shard = shard;
  auto ls = std::make_unique<madipm_ldl>();
  ls->own = std::make_unique<LDLSolver>(n, colptr, rowval, so, o.pivot_tol, user_perm);
  ls->s = ls->own.get();
  ls->lin = ls->s;
  ls->lin->spd = o.cholesky != 0;
  *out = ls.release();
  return 0;
  MADIPM_API_END
}

int madipm_ldl_factorize_phase(madipm_ldl_t ls, int32_t phase, const double* d_nzval, madipm_stream_t stream,
                               double** xbuf, int64_t* xlen) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && ls->own && (phase == 1 || phase == 2), "bad argument");
  require_idle(ls);
  hipStream_t st = (hipStream_t)stream;
  if (phase == 1) {
    ls->s->fact_phase1(d_nzval, st);
    if (xbuf) *xbuf = ls->s->fact_xbuf();
    if (xlen) *xlen = ls->s->fact_xlen();
  } else {
    ls->s->fact_phase2(st);
    ls->last_stream = st;
    ls->pending = true;
  }
  return 0;
  MADIPM_API_END
}

int madipm_ldl_solve_phase(madipm_ldl_t ls, int32_t phase, double* d_x, madipm_stream_t stream, double** xbuf,
                           int64_t* xlen) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && ls->own && phase >= 1 && phase <= 3 && d_x, "bad argument");
  MADIPM_REQUIRE(phase == ls->solve_next, "sharded solve protocol: phase " + std::to_string(phase) + " called, phase " +
                                             std::to_string(ls->solve_next) + " expected (1 -> 2 -> 3; ABI 0.2)");
  // the protocol advances only once the phase is enqueued: a phase that throws (a HIP error) resets it
  // to phase 1, so the handle is not left refusing every later call
  ls->solve_next = 1;
  hipStream_t st = (hipStream_t)stream;
  if (phase == 1) {
    ls->s->solve_phase1(d_x, st);
    if (xbuf) *xbuf = ls->s->solve_xbuf();
    if (xlen) *xlen = ls->s->solve_xlen();
  } else if (phase == 2) {
    ls->s->solve_phase2(d_x, st);
    if (xbuf) *xbuf = ls->s->solve_gbuf();
    if (xlen) *xlen = ls->s->xch_gather();
  } else {
    ls->s->solve_phase3(d_x, st);
    if (xbuf) *xbuf = nullptr;
    if (xlen) *xlen = 0;
  }
  ls->solve_next = phase == 3 ? 1 : phase + 1;
  return 0;
  MADIPM_API_END
}

int madipm_ldl_shard_info(madipm_ldl_t ls, int32_t* owner /* nsuper, may be NULL */, double* top_cost,
                          double* shard_cost_max, double* shard_cost_sum) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls, "null handle");
  const SymbolicPlan& p = ls->s->plan();
  if (owner) {
    for (int s = 0; s < p.nsuper; ++s) owner[s] = p.owner.empty() ? 0 : p.owner[s];
  }
  if (top_cost) *top_cost = p.top_cost;
  if (shard_cost_max) *shard_cost_max = p.shard_cost_max;
  if (shard_cost_sum) *shard_cost_sum = p.shard_cost_sum;
  return 0;
  MADIPM_API_END
}

int madipm_local_allreduce(double* const* d_bufs, int32_t nbuf, int64_t n, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  local_allreduce(d_bufs, nbuf, n, (hipStream_t)stream);
  return 0;
  MADIPM_API_END
}

int madipm_comm_unique_id(void* id128) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(id128, "null argument");
  rccl_unique_id(id128);
  return 0;
  MADIPM_API_END
}

int madipm_comm_create(int32_t nranks, int32_t rank, const void* id128, madipm_comm_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out && id128, "null argument");
  auto c = std::make_unique<madipm_comm>();
  c->c.reset(make_rccl_comm(nranks, rank, id128));
  *out = c.release();
  return 0;
  MADIPM_API_END
}

int madipm_comm_create_host(int32_t nranks, int32_t rank, madipm_allreduce_fn fn, void* ctx, madipm_comm_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out && fn, "null argument");
  auto c = std::make_unique<madipm_comm>();
  c->c.reset(make_host_comm(nranks, rank, fn, ctx));
  *out = c.release();
  return 0;
  MADIPM_API_END
}

int madipm_comm_allreduce(madipm_comm_t c, double* d_buf, int64_t n, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(c && (d_buf || n == 0), "null argument");
  c->c->allreduce_sum(d_buf, n, (hipStream_t)stream);
  return 0;
  MADIPM_API_END
}

int madipm_comm_allgather(madipm_comm_t c, double* d_buf, int64_t nper, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(c && (d_buf || nper == 0) && nper >= 0, "null argument");
  c->c->allgather_inplace(d_buf, nper, (hipStream_t)stream);
  return 0;
  MADIPM_API_END
}

void madipm_comm_destroy(madipm_comm_t c) { delete c; }

int madipm_ldl_get_info(madipm_ldl_t ls, madipm_ldl_info* info) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && info, "null argument");
  fill_info(ls->s->plan(), ls->lin, info);
  return 0;
  MADIPM_API_END
}

int madipm_ldl_factorize_async(madipm_ldl_t ls, const double* d_nzval, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls, "null handle");
  require_idle(ls);  // not between the phases of a sharded solve (as madipm_ldl_factorize)
  ls->lin->factorize_async(d_nzval, (hipStream_t)stream);
  ls->last_stream = (hipStream_t)stream;
  ls->pending = true;
  return 0;
  MADIPM_API_END
}

int madipm_ldl_factorize(madipm_ldl_t ls, const double* d_nzval, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls, "null handle");
  require_idle(ls);
  ls->lin->factorize_async(d_nzval, (hipStream_t)stream);
  ls->pending = false;
  return ls->lin->status((hipStream_t)stream);
  MADIPM_API_END
}

int madipm_ldl_is_factorized(madipm_ldl_t ls) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls, "null handle");
  if (ls->pending) {
    ls->lin->status(ls->last_stream);
    ls->pending = false;
  }
  return ls->s->factorized ? 1 : 0;
  MADIPM_API_END
}

int madipm_ldl_solve(madipm_ldl_t ls, double* d_x, int32_t nrhs, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && (d_x || ls->s->n() == 0), "null argument");
  require_idle(ls);
  for (int k = 0; k < nrhs; ++k) ls->lin->solve_async(d_x + (int64_t)k * ls->s->n(), (hipStream_t)stream);
  return 0;
  MADIPM_API_END
}

int madipm_ldl_inertia(madipm_ldl_t ls, int32_t* pos, int32_t* zero, int32_t* neg) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls, "null handle");
  if (ls->pending) {
    ls->lin->status(ls->last_stream);
    ls->pending = false;
  }
  if (pos) *pos = ls->s->npos;
  if (zero) *zero = ls->s->nzero;
  if (neg) *neg = ls->s->nneg;
  return 0;
  MADIPM_API_END
}

int madipm_ldl_get_d(madipm_ldl_t ls, double* h_d) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && h_d, "null argument");
  MADIPM_HIP(hipDeviceSynchronize());
  MADIPM_HIP(hipMemcpy(h_d, ls->s->d_diag(), sizeof(double) * ls->s->n(), hipMemcpyDeviceToHost));
  if (ls->g) {  // sharded on this device: each column's pivot from a shard that computed it
    const SymbolicPlan& p = ls->s->plan();
    std::vector<double> tmp(ls->s->n());
    for (int r = 1; r < ls->g->nshards(); ++r) {
      MADIPM_HIP(hipMemcpy(tmp.data(), ls->g->shard(r).d_diag(), sizeof(double) * tmp.size(), hipMemcpyDeviceToHost));
      for (int f = 0; f < p.nsuper; ++f)
        if (p.owner[f] == r)
          for (int j = p.first[f]; j < p.first[f + 1]; ++j) h_d[j] = tmp[j];
    }
  }
  return 0;
  MADIPM_API_END
}

int madipm_ldl_perm(madipm_ldl_t ls, int32_t* perm) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && perm, "null argument");
  std::memcpy(perm, ls->s->plan().perm.data(), sizeof(int32_t) * ls->s->n());
  return 0;
  MADIPM_API_END
}

void madipm_ldl_destroy(madipm_ldl_t ls) { delete ls; }

static void fill_kstats(LinSolver& l, madipm_kstat* out) {
  static_assert(MADIPM_NKERNELS == KK_COUNT, "kernel kinds");
  KernelStat st[KK_COUNT];
  l.kernel_stats(st);
  for (int k = 0; k < KK_COUNT; ++k) {
    std::memset(out[k].name, 0, sizeof(out[k].name));
    std::strncpy(out[k].name, kernel_kind_name(k), sizeof(out[k].name) - 1);
    out[k].launches = st[k].launches;
    out[k].time_ms = st[k].ms;
    out[k].bytes = st[k].bytes;
    out[k].flops = st[k].flops;
    out[k].alg_bytes = st[k].alg_bytes;
  }
}

int madipm_ldl_set_timing(madipm_ldl_t ls, uint32_t mask) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls, "null argument");
  ls->s->set_timing(mask);
  return 0;
  MADIPM_API_END
}

int madipm_ldl_kernel_stats(madipm_ldl_t ls, madipm_kstat* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(ls && out, "null argument");
  fill_kstats(*ls->s, out);
  return 0;
  MADIPM_API_END
}

// ------------------------------------------------------------------ native MPC solver
void madipm_default_options(madipm_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->tol = 1e-8;
  o->max_iter = 3000;
  o->max_wall_time = 1e6;
  o->divergence_tol = 1e4;
  o->scaling = 1;
  o->bound_push = 1e-2;
  o->bound_fac = 1e-2;
  o->bound_relax_factor = 1e-12;
  o->regularization = 1;
  o->delta_p = 1e-10;
  o->delta_d = 1e-10;
  o->delta_min = 1e-10;
  o->step_rule = 1;
  o->step_tau = 0.99;
  o->max_ncorr = 0;
  o->mu_init = 1e-1;
  o->mu_min = 1e-12;
  o->tol_linear_solve = 1e-8;
  o->check_residual = 0;
  o->kkt_system = 0;
  o->print_level = 0;
  madipm_ldl_default_opts(&o->ldl);
}

int madipm_solver_create(const madipm_qp* qp, const madipm_options* opt, madipm_solver_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(qp && out, "null argument");
  madipm_options o;
  madipm_default_options(&o);
  if (opt) o = *opt;
  MADIPM_REQUIRE(o.kkt_system >= 0 && o.kkt_system <= 2, "kkt_system must be 0 (K2), 1 (K2.5) or 2 (normal equations)");
  auto s = std::make_unique<madipm_solver>();
  s->s = std::make_unique<MPCSolver>(*qp, o);
  *out = s.release();
  return 0;
  MADIPM_API_END
}

int madipm_solver_create_dist(const madipm_qp* qp, const madipm_options* opt, madipm_comm_t comm,
                              madipm_solver_t* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(qp && out && comm, "null argument");
  madipm_options o;
  madipm_default_options(&o);
  if (opt) o = *opt;
  MADIPM_REQUIRE(o.kkt_system >= 0 && o.kkt_system <= 2, "kkt_system must be 0 (K2), 1 (K2.5) or 2 (normal equations)");
  o.ldl.nshards = 1;
  auto s = std::make_unique<madipm_solver>();
  s->s = std::make_unique<MPCSolver>(*qp, o, comm->c.get());
  *out = s.release();
  return 0;
  MADIPM_API_END
}

int madipm_solver_initialize(madipm_solver_t s) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s, "null handle");
  s->s->initialize_public();
  return 0;
  MADIPM_API_END
}

int madipm_solver_set_max_iter(madipm_solver_t s, int32_t max_iter) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s && max_iter >= 0, "bad argument");
  s->s->set_max_iter(max_iter);
  return 0;
  MADIPM_API_END
}

int madipm_solver_solve(madipm_solver_t s, madipm_stats* stats) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s, "null handle");
  s->s->solve(stats);
  return 0;
  MADIPM_API_END
}

int madipm_solver_get_solution(madipm_solver_t s, double* x, double* y, double* zl, double* zu, double* cons) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s, "null handle");
  s->s->get_solution(x, y, zl, zu, cons);
  return 0;
  MADIPM_API_END
}

int madipm_solver_trace(madipm_solver_t s, madipm_iter_trace* out, int32_t cap) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s, "null handle");
  const auto& t = s->s->trace();
  const int n = (int)std::min<size_t>(t.size(), cap > 0 ? (size_t)cap : 0);
  if (out) std::copy(t.begin(), t.begin() + n, out);
  return (int)t.size();
  MADIPM_API_END
}

int madipm_solver_ldl_info(madipm_solver_t s, madipm_ldl_info* info) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s && info, "null argument");
  fill_info(s->s->ldl().plan(), &s->s->ldl(), info);
  return 0;
  MADIPM_API_END
}

int madipm_solver_ldl_perm(madipm_solver_t s, int32_t* perm) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s && perm, "null argument");
  const auto& p = s->s->ldl().plan().perm;
  std::memcpy(perm, p.data(), sizeof(int32_t) * p.size());
  return 0;
  MADIPM_API_END
}

int madipm_solver_set_timing(madipm_solver_t s, uint32_t mask) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s, "null argument");
  s->s->ldl().set_timing(mask);
  return 0;
  MADIPM_API_END
}

int madipm_solver_kernel_stats(madipm_solver_t s, madipm_kstat* out) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(s && out, "null argument");
  fill_kstats(s->s->ldl(), out);
  return 0;
  MADIPM_API_END
}

void madipm_solver_destroy(madipm_solver_t s) { delete s; }

int madipm_update_step(int32_t rule, double tau, double mu, int32_t nlb, int32_t nub, const double* d_x_lr,
                       const double* d_xl_r, const double* d_zl_r, const double* d_dx_lr, const double* d_dzl,
                       const double* d_x_ur, const double* d_xu_r, const double* d_zu_r, const double* d_dx_ur,
                       const double* d_dzu, madipm_step_result* out, madipm_stream_t stream) {
  MADIPM_API_BEGIN
  MADIPM_REQUIRE(out, "null argument");
  MADIPM_REQUIRE(nlb == 0 || (d_x_lr && d_xl_r && d_zl_r && d_dx_lr && d_dzl), "null lower-bound vector");
  MADIPM_REQUIRE(nub == 0 || (d_x_ur && d_xu_r && d_zu_r && d_dx_ur && d_dzu), "null upper-bound vector");
  const double* v[10] = {d_x_lr, d_xl_r, d_zl_r, d_dx_lr, d_dzl, d_x_ur, d_xu_r, d_zu_r, d_dx_ur, d_dzu};
  update_step_standalone(rule, tau, mu, nlb, nub, v, out, (hipStream_t)stream);
  return 0;
  MADIPM_API_END
}

}  // extern "C"
