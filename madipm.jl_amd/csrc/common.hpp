// Shared host-side utilities: error reporting across the C-ABI, HIP error checks, device buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <memory>
#include <utility>
#include <vector>

#include "hvec.hpp"

namespace madipm {

// Thread-local last error text, returned by madipm_last_error().
void set_last_error(const std::string& msg);
const char* last_error();

struct Error : std::runtime_error {
  int code;
  Error(const std::string& m, int c = -1) : std::runtime_error(m), code(c) {}
};

#define MADIPM_HIP(call)                                                                   \
  do {                                                                                     \
    hipError_t _e = (call);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw ::madipm::Error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " +  \
                            __FILE__ + ":" + std::to_string(__LINE__), -2);                \
  } while (0)

#define MADIPM_REQUIRE(cond, msg)                                                          \
  do {                                                                                     \
    if (!(cond)) throw ::madipm::Error(std::string(msg), -3);                              \
  } while (0)

// Owning device allocation (hipMalloc'd, released in the destructor).
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  DBuf() = default;
  explicit DBuf(size_t count) { alloc(count); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DBuf& operator=(DBuf&& o) noexcept {
    if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~DBuf() { release(); }
  void alloc(size_t count) {
    release();
    n = count;
    if (count) MADIPM_HIP(hipMalloc(&p, count * sizeof(T)));
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  void upload(const T* h, size_t count, hipStream_t s = nullptr) {
    if (count > n) alloc(count);
    if (count) MADIPM_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
  }
  template <class A>
  void upload(const std::vector<T, A>& v, hipStream_t s = nullptr) { upload(v.data(), v.size(), s); }
  void zero(hipStream_t s = nullptr) {
    if (n) MADIPM_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
  }
  operator T*() const { return p; }
};

// MADIPM_SYMBOLIC_TIMING=1: wall time of each construction phase on stderr (diagnostics: the dense
// QP's analysis_s breakdown)
struct PhaseClock {
  const char* who;
  bool on = std::getenv("MADIPM_SYMBOLIC_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit PhaseClock(const char* w) : who(w) {}
  void operator()(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "%s %-28s %9.3f s\n", who, what, std::chrono::duration<double>(n - t).count());
    t = n;
  }
};

}  // namespace madipm
