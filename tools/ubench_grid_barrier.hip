// Grid-wide barrier cost on MI355X, with the barrier the persistent GD loop
// uses (tools/grid_sync.h: XCD-hierarchical arrival, relaxed polling with
// s_sleep, ONE agent-scope acquire after the exit).  Round 4's version put
// all 256 arrivals on one counter and polled with an acquire load per spin
// (an L1 invalidate per poll): 13.7 us per barrier.
//
//   hipcc -O3 --offload-arch=gfx950 -Icsrc tools/ubench_grid_barrier.hip -o /tmp/ubgb && /tmp/ubgb
//
// Per barrier every workgroup publishes a payload (0 B, 16 KB, or 104 KB =
// one GD partial row of the wide bench's 13K near slots), stored either
// write-through (sc1, 8-B agent stores) or plainly (the release fence then
// writes the dirty L2 lines back); after the barrier it reads the payload of
// workgroup (b + 37) % n -- another XCD under round-robin placement -- and
// checks every word (stale or torn reads are counted: the protocol check).
// Every workgroup is resident (1024 threads and 96 KB of LDS: one per CU),
// every spin is bounded.  The launch baseline is two empty 256-workgroup
// kernels back to back.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "grid_sync.h"

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

using twtml::grid_sync;
using gu64 = __attribute__((address_space(1))) unsigned long long;

__device__ __forceinline__ unsigned long long tag(unsigned e, unsigned b, unsigned i) {
  return (uint64_t(e) << 40) ^ (uint64_t(b) << 20) ^ uint64_t(i);
}

__global__ __launch_bounds__(1024) void k_barrier(uint32_t* sync, int iters, unsigned nblocks, int words,
                                                  unsigned long long* payload, int wt, unsigned* errors) {
  extern __shared__ uint32_t lds_pad[];   // one workgroup per CU, like the GD loop
  if (threadIdx.x == 0) lds_pad[0] = 0;
  const unsigned b = blockIdx.x;
  const unsigned src = (b + 37) % nblocks;
  unsigned bad = 0;
  for (int it = 1; it <= iters; ++it) {
    unsigned long long* mine = payload + size_t(b) * words;
    for (int i = threadIdx.x; i < words; i += 1024) {
      const unsigned long long v = tag(unsigned(it), b, unsigned(i));
      if (wt) __hip_atomic_store((gu64*)(mine + i), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else mine[i] = v;
    }
    // epochs are the barriers' ordinals: 1, 2, 3, ... (two per iteration with a payload)
    const unsigned e0 = words ? unsigned(2 * it - 1) : unsigned(it);
    if (!grid_sync(sync, e0, nblocks)) return;
    const unsigned long long* theirs = payload + size_t(src) * words;
    for (int i = threadIdx.x; i < words; i += 1024) bad += theirs[i] != tag(unsigned(it), src, unsigned(i));
    // the next epoch overwrites the payload only after everyone read it
    if (words && !grid_sync(sync, e0 + 1, nblocks)) return;
  }
  if (bad) atomicAdd(errors, bad);
}

__global__ void k_empty() {}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* sync = nullptr;
  unsigned long long* payload = nullptr;
  unsigned* errors = nullptr;
  CHECK(hipMalloc(&sync, twtml::kSyncBytes));
  CHECK(hipMalloc(&errors, 64));
  const int max_words = 13312;   // 104 KB per workgroup
  CHECK(hipMalloc(&payload, size_t(cus) * max_words * sizeof(unsigned long long)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::printf("CUs %d (%s); barrier: XCD-hierarchical, relaxed poll + s_sleep, one acquire\n", cus,
              prop.gcnArchName);
  const size_t lds = 96 * 1024;
  for (int words : {0, 2048, max_words}) {
    for (int wt : {1, 0}) {
      if (words == 0 && wt == 0) continue;
      for (int iters : {20, 1000}) {
        CHECK(hipMemset(sync, 0, twtml::kSyncBytes));
        CHECK(hipMemset(errors, 0, 64));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_barrier, dim3(cus), dim3(1024), lds, 0, sync, iters, unsigned(cus), words, payload,
                           wt, errors);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, a, b));
        unsigned err = 0, tmo = 0;
        CHECK(hipMemcpy(&err, errors, sizeof(unsigned), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(&tmo, sync + 18 * twtml::kSyncLine, sizeof(unsigned), hipMemcpyDeviceToHost));
        const int nbar = words ? 2 * iters : iters;
        std::printf("workgroups %4d, payload %6d B/WG %-13s %5d barriers: %8.3f ms, %6.2f us per barrier "
                    "(%s)  stale words %u%s\n",
                    cus, words * 8, words ? (wt ? "write-through" : "plain+release") : "", nbar, ms,
                    1e3 * ms / nbar, words ? "publish + barrier + read + barrier" : "barrier", err,
                    tmo ? "  TIMEOUT" : "");
      }
    }
  }
  CHECK(hipEventRecord(a));
  for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(k_empty, dim3(cus), dim3(1024), 0, 0);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("launch baseline: %d-workgroup empty kernels back to back: %.2f us per launch\n", cus, 1e3 * ms / 1000);
  return 0;
}
