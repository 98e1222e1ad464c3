// Device allocations of the engines.  TWTML_POISON=<byte> fills every new
// buffer with that byte (debugging: a result that changes under poison reads
// memory it never wrote).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace twtml {

inline void* dev_alloc(size_t bytes) {
  void* p = nullptr;
  bytes = std::max<size_t>(1, bytes);
  TWTML_HIP_CHECK(hipMalloc(&p, bytes));
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
