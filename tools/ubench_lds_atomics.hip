// Microbenchmark: LDS atomic throughput on gfx950 for the gradient-scatter
// access pattern (random slots in a ~1.4K-entry table, 64 lanes/instruction).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds_atomics.hip -o /tmp/ub
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kSlots = 1472;
constexpr int kOps = 512;

template <int MODE>
__global__ __launch_bounds__(512) void k(float* out, uint32_t seed) {
  __shared__ float f[kSlots * 4];
  __shared__ unsigned long long u64[kSlots];
  uint32_t* u = reinterpret_cast<uint32_t*>(f);
  for (int i = threadIdx.x; i < kSlots * 4; i += 512) f[i] = 0.f;
  for (int i = threadIdx.x; i < kSlots; i += 512) u64[i] = 0;
  __syncthreads();
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  float acc = 0.f;
  for (int i = 0; i < kOps; ++i) {
    x = x * 1664525u + 1013904223u;
    const uint32_t s = (x >> 8) % kSlots;
    if (MODE == 0) atomicAdd(&f[s], 1.0f);                        // ds_add_f32
    if (MODE == 1) atomicAdd(&u[s], 1u);                          // ds_add_u32
    if (MODE == 2) atomicAdd(&u64[s], 1ull);                      // ds_add_u64
    if (MODE == 3) acc += f[s];                                   // ds_read_b32
    if (MODE == 4) f[s] = acc;                                    // ds_write_b32
    if (MODE == 5) atomicAdd(&f[s * 4 + (threadIdx.x & 3)], 1.f); // replicated x4
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = f[7] + acc + float(u64[3]);
}

template <int MODE>
float run(float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<MODE>, dim3(1024), dim3(512), 0, 0, out, 1u);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(1024), dim3(512), 0, 0, out, 1u + r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  float* out;
  hipMalloc(&out, 1024 * sizeof(float));
  const double ops = 1024.0 * 512 * kOps;
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64", "ds_read_b32", "ds_write_b32", "ds_add_f32 rep4"};
  float t[6] = {run<0>(out), run<1>(out), run<2>(out), run<3>(out), run<4>(out), run<5>(out)};
  for (int i = 0; i < 6; ++i)
    printf("%-16s %8.3f ms  %8.1f Gop/s  %6.1f cyc/wave-instr/CU @2.1GHz\n", names[i], t[i],
           ops / t[i] / 1e6, t[i] * 1e-3 * 2.1e9 * 256 / (ops / 64));
  return 0;
}
