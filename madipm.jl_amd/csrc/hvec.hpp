// Host vectors whose resize() leaves new elements uninitialised (shared by the host-only analysis and
// the HIP-side headers).
#pragma once

#include <memory>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

namespace madipm {

// allocator whose resize() leaves new elements uninitialised: big host index / value arrays that the
// threads filling them write in full (first touch in parallel instead of a serial zero fill)
template <class T>
struct NoInit : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInit<U>;
  };
  NoInit() = default;
  template <class U>
  NoInit(const NoInit<U>&) {}
  template <class U>
  void construct(U* p) { ::new ((void*)p) U; }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T>
using hvec = std::vector<T, NoInit<T>>;

// Frees the given containers on a detached thread (big host arrays whose release only costs time).
template <class... V>
void free_async(V&&... v) {
  auto* box = new std::tuple<std::decay_t<V>...>(std::move(v)...);
  std::thread([box] { delete box; }).detach();
}

}  // namespace madipm
