// Native Mehrotra predictor-corrector driver (restates MadIPM's `mpc!`, src/solver.jl:332-360)
// on top of the HIP LDL^T and the fused IPM vector kernels.  All vectors stay in HBM; scalar
// reductions land in a device-resident state block; the host reads ONE small block per iteration.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/madipm_hip.h"
#include "common.hpp"
#include "ldl.hpp"

namespace madipm {

struct Csr {
  int64_t* rp = nullptr;
  int32_t* ci = nullptr;
  double* v = nullptr;
};

// Device-resident scalars (one struct, copied to host once per iteration).
struct DevState {
  double mu, mu_curr, mu_aff;
  double alpha_p, alpha_d;            // final step
  double alpha_aff_p, alpha_aff_d;    // predictor (tau = 1)
  double a_xl, a_xu, a_zl, a_zu;      // last ratio test pieces
  double obj_val;
  double inf_pr_raw, inf_du_raw, inf_compl_raw, dobj;
  double res_ratio;                   // last solve_system! residual ratio
  double max_res_ratio;               // max over the iteration's solves
  double dx_inf;                      // ||primal(d)||_inf (print_iter)
  double delta_x, delta_s, delta_x2, delta_s2;  // init_starting_point! shifts
  double init_viol;                   // init assertion violations
  int32_t i_xl, i_xu, i_zl, i_zu;     // argmin indices (-1 = init element)
  int32_t nan_flag;
  int32_t pad;
  LDLStatus ldl_status;  // the linear solver's status (external_status): one read-back per iteration
};

struct QPHost;  // host copy of the problem (mpc.hip)

class MPCSolver {
 public:
  // comm != nullptr (size > 1): this process holds shard comm->rank of the sharded factorisation
  MPCSolver(const madipm_qp& qp, const madipm_options& opt, Comm* comm = nullptr);
  ~MPCSolver();
  int solve(madipm_stats* stats);
  void initialize_public();  // initialize! alone (so that callers can time the MPC loop only)
  void set_max_iter(int k) { opt_.max_iter = k; }
  void get_solution(double* x, double* y, double* zl, double* zu, double* cons);
  const std::vector<madipm_iter_trace>& trace() const { return trace_; }
  LinSolver& ldl() { return *ldl_; }
  hipStream_t stream() const { return stream_; }

 private:
  void setup_host(const madipm_qp& qp);
  std::unique_ptr<LinSolver> make_linsolver(int n, const int64_t* cp, const int32_t* ri, const SymbolicOptions& so);
  void initialize();
  void init_starting_point();
  // amode >= 0: k_alpha of that mode runs after the residual and is finalised with it (one k_final less)
  // mu_nb > 0: the corrector's k_rhs finalises the barrier update from k_mu's mu_nb partials
  void solve_system(int mode, double mu, int reset = 0, int amode = -1, double atau = 1.0, int mu_nb = 0);
  void gondzio();
  // predictor + corrector directions (speculated before the status read); fuse_step: the corrector's
  // solve also runs update_step_size!'s step test (only when nothing changes d in between: no Gondzio)
  void directions(bool redo, bool fuse_step);
  void step_size(bool fused);
  void launch_reduce_final(int kind, int nvals, int amode = -1, int nb_eval = 0, LDLStatus* rs = nullptr,
                           bool publish = false);
  int step_alpha_mode(double& tau) const;
  void read_state();  // enqueue the publication of the device state to the host mirror
  void wait_state();  // wait (host spin) until the last publication has landed
  void kkt_diag(double dw, double dc);
  // build_kkt!: diagonal (+ K2.5 scaling / normal-matrix assembly) -> values handed to the LDL^T
  void assemble_kkt(double dw, double dc, bool diag_done = false);
  const double* kvals() const;
  // MadNLP.solve!(kkt, d) after the right-hand side is in d_: reduced solve in the chosen formulation
  void kkt_solve();
  void factor_enqueue(double dw, double dc);
  void timed_factorize();
  LDLStatus* fact_reset() const;
  LDLStatus* take_fact_end();
  int blocks(int64_t n) const;
  int spmv_blocks(int64_t rows) const;

  madipm_options opt_{};
  hipStream_t stream_ = nullptr;
  std::unique_ptr<QPHost> H_;
  std::unique_ptr<LinSolver> ldl_;
  Comm* comm_ = nullptr;
  // sizes
  int nx_ = 0, ns_ = 0, n_ = 0, m_ = 0, nlb_ = 0, nub_ = 0;
  int64_t nnzK_ = 0, L_ = 0;  // L_ = unreduced vector length
  // device vectors
  DBuf<double> x_, xl_, xu_, zl_, zu_, f_, jacl_, c_, y_, rhs_, pr_diag_, l_diag_, u_diag_, l_lower_, u_lower_;
  DBuf<double> d_, p_, corr_lb_, corr_ub_, dsave_;
  DBuf<double> Kx_, Hdiag_, cs_, gfix_, cfix_, lo_full_, hi_full_;
  DBuf<int64_t> diag_pos_;
  DBuf<int32_t> ind_lb_, ind_ub_, lbpos_, ubpos_;
  DBuf<uint8_t> fixed_;
  DBuf<int64_t> Hrp_, Jrp_, JTrp_;
  DBuf<int32_t> Hci_, Jci_, JTci_;
  DBuf<double> Hv_, Jv_, JTv_;
  DBuf<double> part_;
  // KKT formulation (0 K2, 1 K2.5, 2 normal equations)
  int kkt_ = 0;
  int spmv_g_ = 8;  // lanes per row in the SpMV kernels
  static constexpr int kFinDbg = 4096;
  DBuf<int64_t> fdbg_;  // MADIPM_FINAL_DEBUG: k_final stamps (ring of kFinDbg launches)
  int64_t fdbg_n_ = 0;
  int maxb_ = 2048;  // partial-reduction blocks per producer launch (<= MAXB; r3 / r5: 1024 or 512 measured slower)
  DBuf<double> sk_, K0_, Dinv_, bufm_, Cx_;
  DBuf<int32_t> Krow_, Kcol_, cprod_;
  DBuf<int64_t> cpp_;
  int64_t nnzC_ = 0;
  DBuf<DevState> st_;
  DevState* hst_ = nullptr;          // host mirror of st_ (coherent pinned memory, written by k_publish)
  uint32_t* hseq_ = nullptr;         // publication counter beside it
  uint32_t pub_seq_ = 0;
  bool publish_next_ = false;        // the next solve_system's k_rhs publishes the state
  bool fact_end_pending_ = false;    // the next solve_system's k_rhs stamps the factorisation's end
  // host scalars (MPCSolver fields of src/structure.jl:62-76)
  double del_w_ = 0, del_c_ = 0, norm_b_ = 0, norm_c_ = 0, best_compl_ = 0, obj_scale_ = 1, c0s_ = 0;
  bool eval_pending_ = false;  // k_eval's objective partials await the next FIN_TERM
  double adapt_dp_ = 0, adapt_dd_ = 0, adapt_dmin_ = 0;
  int status_ = 0, k_ = 0;
  int exception_ = 0;  // MADIPM_EXC_* of the last solve (what solve!'s catch-all caught)
  bool initialized_ = false;
  double inf_pr_ = 0, inf_du_ = 0, inf_compl_ = 0;
  double spec_near_ = 10.0;  // MADIPM_SPEC_NEAR: hold the speculative factorisation when residuals <= this x tol (0: never)
  double t_init_ = 0, t_total_ = 0, t_linsol_ = 0;
  std::vector<madipm_iter_trace> trace_;
  double fs0_ = 0;  // device factorisation seconds at initialize! (cnt.linear_solver_time origin)
  DevState last_{};                // the state of the last termination test
};

// update_step! on caller-given vectors (madipm_update_step); v = the 10 device pointers in header order
void update_step_standalone(int rule, double tau_param, double mu, int nlb, int nub, const double* const* v,
                            madipm_step_result* out, hipStream_t s);

}  // namespace madipm
