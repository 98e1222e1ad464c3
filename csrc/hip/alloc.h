// Device allocations of the engines.  TWTML_POISON=<byte> fills every new
// buffer with that byte (debugging: a result that changes under poison reads
// memory it never wrote).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>

#include "common.h"

namespace twtml {

// Bytes the engines have allocated so far (monotonic): the difference across
// an engine's construction is its device footprint (HBM batch sizing).
inline std::atomic<uint64_t>& dev_alloc_bytes() {
  static std::atomic<uint64_t> total{0};
  return total;
}

inline void* dev_alloc(size_t bytes) {
  void* p = nullptr;
  bytes = std::max<size_t>(1, bytes);
  TWTML_HIP_CHECK(hipMalloc(&p, bytes));
  dev_alloc_bytes() += bytes;
  static const int poison = [] {
    const char* e = std::getenv("TWTML_POISON");
    return e && *e ? std::atoi(e) & 0xFF : -1;
  }();
  if (poison >= 0) {
    TWTML_HIP_CHECK(hipMemset(p, poison, bytes));
    TWTML_HIP_CHECK(hipDeviceSynchronize());
  }
  return p;
}

}  // namespace twtml
