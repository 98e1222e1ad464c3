// Fault attribution for the engines (round-6 verdict item 1).
//
// * TWTML_DEBUG_SYNC=1: every kernel launch (TWTML_LAUNCH) and every H2D of a
//   raw slot is followed by a synchronisation of its stream and an error
//   check that names the kernel / copy and its source line, so an
//   asynchronous fault surfaces at the launch that caused it instead of at
//   the next unrelated call.  Off: one predictable branch per launch.
// * Teardown errors: an engine destructor cannot throw, so the device error
//   its final synchronisation returns is printed and kept here; the GPU test
//   suite fails the test that left one (tests/conftest.py).
// * Host registrations: the live hipHostRegister ranges.  Registering a range
//   that overlaps a live one is refused: with the runtime's host-pointer map,
//   a registration of freed memory that was never unregistered captures every
//   later buffer mapped at an overlapping address.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace twtml {

inline bool debug_sync_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TWTML_DEBUG_SYNC");
    return e && e[0] == '1';
  }();
  return on;
}

inline void debug_sync_point(const char* what, hipStream_t s, const char* file, int line) {
  hipError_t e = hipGetLastError();   // launch-time error (bad grid, LDS, ...)
  const char* phase = "launch";
  if (e == hipSuccess) {
    e = hipStreamSynchronize(s);      // execution-time error (fault, abort)
    phase = "execution";
  }
  if (e != hipSuccess)
    throw std::runtime_error(std::string("TWTML_DEBUG_SYNC: ") + phase + " of " + what + " (" + file + ":" +
                             std::to_string(line) + "): " + hipGetErrorString(e));
}

#define TWTML_DEBUG_POINT(what, stream)                                                  \
  do {                                                                                   \
    if (::twtml::debug_sync_enabled()) ::twtml::debug_sync_point(what, stream, __FILE__, __LINE__); \
  } while (0)

// hipLaunchKernelGGL + the debug sync point (kernel name as written)
#define TWTML_LAUNCH(kernel, grid, block, lds, stream, ...)                \
  do {                                                                     \
    hipLaunchKernelGGL(kernel, grid, block, lds, stream, ##__VA_ARGS__);   \
    TWTML_DEBUG_POINT(#kernel, stream);                                    \
  } while (0)

// ---- teardown errors -------------------------------------------------------
inline std::mutex& teardown_mu() {
  static std::mutex m;
  return m;
}
inline std::vector<std::string>& teardown_log() {
  static std::vector<std::string> v;
  return v;
}
// Record (and print) a device error found while tearing `who` down.
inline void report_teardown_error(const char* who, int device, hipError_t e) {
  if (e == hipSuccess) return;
  const std::string msg = std::string(who) + " on device " + std::to_string(device) +
                          ": device error pending at teardown (raised by this engine's own work): " +
                          hipGetErrorString(e);
  std::fprintf(stderr, "[twtml] %s\n", msg.c_str());
  std::lock_guard<std::mutex> lk(teardown_mu());
  teardown_log().push_back(msg);
}
inline std::vector<std::string> take_teardown_errors() {
  std::lock_guard<std::mutex> lk(teardown_mu());
  std::vector<std::string> v;
  v.swap(teardown_log());
  return v;
}

// ---- host registrations ----------------------------------------------------
inline std::mutex& host_registry_mu() {
  static std::mutex m;
  return m;
}
inline std::map<uintptr_t, size_t>& host_registry() {
  static std::map<uintptr_t, size_t> r;
  return r;
}
inline void host_registry_add(uintptr_t p, size_t n) {
  if (n == 0) throw std::invalid_argument("host_register: empty range");
  std::lock_guard<std::mutex> lk(host_registry_mu());
  auto& r = host_registry();
  auto it = r.upper_bound(p);
  bool overlap = it != r.end() && it->first < p + n;
  if (!overlap && it != r.begin()) {
    auto prev = std::prev(it);
    overlap = prev->first + prev->second > p;
  }
  if (overlap)
    throw std::runtime_error("host_register: range overlaps a live registration (a registered buffer "
                             "was freed without host_unregister?)");
  r.emplace(p, n);
}
inline void host_registry_remove(uintptr_t p) {
  std::lock_guard<std::mutex> lk(host_registry_mu());
  if (host_registry().erase(p) == 0)
    throw std::invalid_argument("host_unregister: pointer was not registered");
}
inline std::vector<std::pair<uintptr_t, size_t>> host_registry_snapshot() {
  std::lock_guard<std::mutex> lk(host_registry_mu());
  return {host_registry().begin(), host_registry().end()};
}

}  // namespace twtml
