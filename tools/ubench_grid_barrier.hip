// Grid-wide barrier cost on MI355X: the input to a persistent GD loop (one
// launch for all iterations, a grid barrier where the loop now ends one
// kernel and launches the next).
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_grid_barrier.hip -o /tmp/ubgb && /tmp/ubgb
//
// Every workgroup is resident (grid <= CUs x blocks per CU), the arrival
// counter and the generation word are device-scope atomics, and every wait
// is bounded: a workgroup that spins past kSpinLimit records a timeout and
// leaves the loop, so the grid always drains.  Prints microseconds per
// barrier for 1024-thread workgroups at 1 and 2 per CU, with and without a
// 16 KB per-workgroup write before each barrier (the partial-row traffic a
// fused update would publish).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr unsigned kSpinLimit = 1u << 22;

__global__ __launch_bounds__(1024) void k_grid_barrier(unsigned* sync, int iters, unsigned nblocks, int write_words,
                                                       unsigned* scratch, unsigned* timeouts, int zero) {
  // sync[0]: arrivals, sync[64]: generation (separate cache lines); the
  // lane-dependent offset (zero * tid, zero = 0 at run time) keeps the
  // atomics on the vector memory path
  const int tid = threadIdx.x;
  unsigned* arrive = sync + zero * tid;
  unsigned* gen = sync + 64 + zero * tid;
  __shared__ int bail;
  if (tid == 0) bail = 0;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    for (int i = tid; i < write_words; i += 1024)   // this workgroup's payload for the others
      scratch[size_t(blockIdx.x) * write_words + i] = unsigned(it + i);
    __syncthreads();
    if (tid == 0) {
      const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned prev = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == nblocks - 1) {
        __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        unsigned spins = 0;
        while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
          if (++spins >= kSpinLimit) {
            __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bail = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    if (bail) return;
  }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  unsigned *sync = nullptr, *scratch = nullptr, *timeouts = nullptr;
  CHECK(hipMalloc(&sync, 4096));
  CHECK(hipMalloc(&timeouts, 64));
  const int max_words = 4096;   // 16 KB per workgroup
  CHECK(hipMalloc(&scratch, size_t(2 * cus) * max_words * sizeof(unsigned)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::printf("CUs %d (%s)\n", cus, prop.gcnArchName);
  for (int per_cu = 1; per_cu <= 2; ++per_cu) {
    for (int words : {0, max_words}) {
      const unsigned nb = unsigned(cus * per_cu);
      for (int iters : {10, 1000}) {
        CHECK(hipMemset(sync, 0, 4096));
        CHECK(hipMemset(timeouts, 0, 64));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_grid_barrier, dim3(nb), dim3(1024), 0, 0, sync, iters, nb, words, scratch, timeouts, 0);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, a, b));
        unsigned to = 0;
        CHECK(hipMemcpy(&to, timeouts, sizeof(unsigned), hipMemcpyDeviceToHost));
        std::printf("workgroups %4u (%d per CU), payload %5d B/WG, %5d barriers: %9.3f ms total, %7.2f us per barrier%s\n",
                    nb, per_cu, words * 4, iters, ms, 1e3 * ms / iters, to ? "  (TIMEOUTS)" : "");
      }
    }
  }
  // the launch-per-iteration baseline: two empty kernels back to back
  CHECK(hipEventRecord(a));
  for (int i = 0; i < 1000; ++i)
    hipLaunchKernelGGL(k_grid_barrier, dim3(unsigned(cus)), dim3(1024), 0, 0, sync, 0, unsigned(cus), 0, scratch, timeouts, 0);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("launch baseline: %d-workgroup kernels back to back: %.2f us per launch\n", cus, 1e3 * ms / 1000);
  return 0;
}
