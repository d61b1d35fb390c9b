// RCCL communicator for the sharded factorisation (SURVEY §8 e): one process per GPU, one
// communicator per solver, every collective an in-place fp64 sum ordered on the solver's stream
// (no host synchronisation).  Over xGMI the ring all-reduce of the top fronts is per-link bound;
// the payload per factorisation is sum(top r (r+1)/2) doubles, per solve an all-reduce of sum(top r)
// doubles and an in-place all-gather of the shards' subtree solution slices (n - top columns).
#include <rccl/rccl.h>

#include <cstring>

#include "ldl.hpp"

namespace madipm {

#define MADIPM_NCCL(call)                                                                        \
  do {                                                                                           \
    ncclResult_t _r = (call);                                                                    \
    if (_r != ncclSuccess)                                                                       \
      throw ::madipm::Error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " +      \
                            __FILE__ + ":" + std::to_string(__LINE__), -2);                      \
  } while (0)

static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");

namespace {

struct RcclComm final : Comm {
  ncclComm_t c = nullptr;
  RcclComm(int nranks, int r, const void* id) {
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    rank = r;
    size = nranks;
    MADIPM_NCCL(ncclCommInitRank(&c, nranks, u, r));
  }
  ~RcclComm() override {
    if (c) (void)ncclCommDestroy(c);
  }
  void allreduce_sum(double* buf, int64_t n, hipStream_t s) override {
    if (n <= 0) return;
    MADIPM_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, c, s));
  }
  // in place: rank r's slice already sits at buf + r nper (ring: (size-1) nper doubles per link)
  void allgather_inplace(double* buf, int64_t nper, hipStream_t s) override {
    if (nper <= 0) return;
    MADIPM_NCCL(ncclAllGather(buf + (int64_t)rank * nper, buf, (size_t)nper, ncclDouble, c, s));
  }
};

// Host-staged all-reduce through a caller-supplied callback (e.g. torch.distributed / gloo): stream
// synchronised, D2H into a pinned buffer, callback, H2D.  For tests of the multi-process protocol
// where RCCL cannot run (several ranks sharing one GPU) — not a data path for production.
struct HostComm final : Comm {
  int (*fn)(double*, int64_t, void*) = nullptr;
  void* ctx = nullptr;
  double* host = nullptr;
  int64_t cap = 0;
  ~HostComm() override {
    if (host) (void)hipHostFree(host);
  }
  void allreduce_sum(double* buf, int64_t n, hipStream_t s) override {
    if (n <= 0) return;
    if (n > cap) {
      if (host) MADIPM_HIP(hipHostFree(host));
      MADIPM_HIP(hipHostMalloc((void**)&host, sizeof(double) * n, hipHostMallocDefault));
      cap = n;
    }
    MADIPM_HIP(hipMemcpyAsync(host, buf, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    MADIPM_HIP(hipStreamSynchronize(s));
    MADIPM_REQUIRE(fn(host, n, ctx) == 0, "host all-reduce callback failed");
    MADIPM_HIP(hipMemcpyAsync(buf, host, sizeof(double) * n, hipMemcpyHostToDevice, s));
    MADIPM_HIP(hipStreamSynchronize(s));
  }
};

}  // namespace

Comm* make_host_comm(int nranks, int rank, int (*fn)(double*, int64_t, void*), void* ctx) {
  MADIPM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks && fn, "bad communicator arguments");
  auto* c = new HostComm();
  c->rank = rank;
  c->size = nranks;
  c->fn = fn;
  c->ctx = ctx;
  return c;
}

void rccl_unique_id(void* out) {
  ncclUniqueId u;
  MADIPM_NCCL(ncclGetUniqueId(&u));
  std::memcpy(out, &u, sizeof(u));
}

Comm* make_rccl_comm(int nranks, int rank, const void* unique_id) {
  MADIPM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks && unique_id, "bad communicator arguments");
  return new RcclComm(nranks, rank, unique_id);
}

}  // namespace madipm
