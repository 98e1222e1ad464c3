// Device-scope atomic adds on a far-slot-sized counter array: u32 vs u64,
// with and without a returned value, random slots (the remap's far counts
// and the far CSC's cursors).  hipcc --offload-arch=gfx950 -O3 -o ubench_atomics ubench_atomics.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

template <typename T, bool RET>
__global__ __launch_bounds__(256) void k_add(const uint32_t* __restrict__ slot, int64_t n, T* cnt, T* out) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    if (RET) out[i] = atomicAdd(&cnt[slot[i]], T(1));
    else atomicAdd(&cnt[slot[i]], T(1));
  }
}

template <typename T, bool RET>
static float run(const uint32_t* slot, int64_t n, T* cnt, T* out, int nslots, int grid) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipMemset(cnt, 0, sizeof(T) * size_t(nslots));
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((k_add<T, RET>), dim3(grid), dim3(256), 0, 0, slot, n, cnt, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return best * 1e3f;
}

int main() {
  const int nslots = 175000;
  const int64_t n = 8000000;
  std::vector<uint32_t> h(static_cast<size_t>(n));
  uint64_t x = 88172645463325252ull;
  for (auto& v : h) {   // xorshift, Zipf-free uniform slots
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    v = uint32_t(x % uint64_t(nslots));
  }
  uint32_t* slot = nullptr;
  void* cnt = nullptr;
  void* out = nullptr;
  CHECK(hipMalloc(&slot, sizeof(uint32_t) * size_t(n)));
  CHECK(hipMalloc(&cnt, sizeof(uint64_t) * size_t(nslots)));
  CHECK(hipMalloc(&out, sizeof(uint64_t) * size_t(n)));
  CHECK(hipMemcpy(slot, h.data(), sizeof(uint32_t) * size_t(n), hipMemcpyHostToDevice));
  for (int grid : {1024, 2048, 8192}) {
    std::printf("grid %5d: u32 %7.1f us  u64 %7.1f us  u32+ret %7.1f us  u64+ret %7.1f us  (%lld adds, %d slots)\n", grid,
                run<uint32_t, false>(slot, n, static_cast<uint32_t*>(cnt), static_cast<uint32_t*>(out), nslots, grid),
                run<unsigned long long, false>(slot, n, static_cast<unsigned long long*>(cnt),
                                               static_cast<unsigned long long*>(out), nslots, grid),
                run<uint32_t, true>(slot, n, static_cast<uint32_t*>(cnt), static_cast<uint32_t*>(out), nslots, grid),
                run<unsigned long long, true>(slot, n, static_cast<unsigned long long*>(cnt),
                                              static_cast<unsigned long long*>(out), nslots, grid),
                static_cast<long long>(n), nslots);
  }
  CHECK(hipDeviceSynchronize());
  (void)hipFree(slot);
  (void)hipFree(cnt);
  (void)hipFree(out);
  return 0;
}
