// Multifrontal supernodal LDL^T on the GPU (gfx950) — the linear-solver plugin of SURVEY §8 a11/a14.
//
// Replaces `MadNLP.factorize!(kkt.linear_solver)` / `MadNLP.solve!(kkt.linear_solver, x)` for the
// solvers the reference plugs in (LDLFactorizations' LDLSolver, MadNLPGPU's CUDSSSolver with
// cudss_algorithm = LDL, HSL Ma57Solver): called from src/linear_solver.jl:10 and :26 via MadNLP.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "common.hpp"
#include "symbolic.hpp"

namespace madipm {

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
  const int64_t* crow_off;
  const int64_t* crow;
  const int32_t* ce_child;
  const int32_t* ce_row;
  const int32_t* bigch_ptr;
  const int32_t* bigch_list;
  const int32_t* bigslot;  // big front -> slot in the panel-inverse scratch (64x64 per slot)
};

struct SolveTask {
  int32_t front, blk;
};

struct LDLStatus {  // device-resident, read back by status()
  int32_t fail_pivot;  // min failing internal pivot + 1 (INT32_MAX when none)
  int32_t npos, nneg, nzero;
};

class LDLSolver {
 public:
  LDLSolver(int n, const int64_t* colptr, const int32_t* rowval, const SymbolicOptions& sopt,
            double pivot_tol, const int32_t* user_perm = nullptr);
  ~LDLSolver();
  LDLSolver(const LDLSolver&) = delete;
  LDLSolver& operator=(const LDLSolver&) = delete;

  // Enqueue the numeric factorisation of the values `Kx` (device, caller's CSC order) on `s`.
  void factorize_async(const double* Kx, hipStream_t s);
  // Synchronise `s` and return 0 or failing pivot + 1; fills the inertia.
  int status(hipStream_t s);
  // In-place solve K x = b for a device vector of length n (caller's ordering).
  void solve_async(double* b, hipStream_t s);

  const SymbolicPlan& plan() const { return S_; }
  int n() const { return S_.N; }
  int npos = 0, nneg = 0, nzero = 0;
  bool factorized = false;
  double pivot_tol = 0.0;

  // device buffers for diagnostics
  const double* d_diag() const { return D_.p; }

 private:
  enum Kind { SMALL32 = 0, SMALL64 = 1, SMALL128 = 2, BIG_TILES = 3, BIG_PULL = 4, BIG_BIGCH = 5, BIG_DIAG = 6, BIG_TRSM = 7,
              BIG_UPDATE = 8 };
  struct Launch {
    int kind;
    int step;       // panel step for BIG_DIAG / BIG_TRSM / BIG_UPDATE
    int64_t off;    // offset of the front list in sched_ (then prefix[nf+1] for big kinds)
    int nf;         // number of fronts
    int64_t items;  // workgroups
  };
  struct SolveLevel {
    int64_t small_off;
    int nsmall;
    int64_t big_off;
    int nbig;
    int64_t ftask_off;
    int nftask;
    int64_t btask_off;
    int nbtask;
  };
  SymbolicPlan S_;
  FrontTab T_{};
  std::vector<Launch> fact_;
  std::vector<SolveLevel> slev_;  // per level, leaves first
  DBuf<int32_t> tasks_, flags_, flag_off_, counters_, err_;
  int epoch_ = 0;
  // device data
  DBuf<int32_t> first_, nrows_, rows_, u_ld_, child_ptr_, child_list_, rel_, perm_, sched_;
  DBuf<int32_t> ce_child_, ce_row_, bigch_ptr_, bigch_list_, bigslot_;
  DBuf<double> minv_;
  DBuf<int64_t> row_ptr_, l_off_, u_off_, uvec_off_, asm_ptr_, asm_src_, asm_dst64_, rel_ptr_, crow_off_, crow_;
  DBuf<double> arena_, D_, xi_, uvec_, vwork_;
  DBuf<LDLStatus> status_;
  LDLStatus* h_status_ = nullptr;
};

}  // namespace madipm
