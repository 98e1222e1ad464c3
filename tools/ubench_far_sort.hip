// Far CSC build, micro-benchmark (alone on the GPU): n (row, slot) entries
// grouped by slot
//   (a) the engine's way: a 64-bit cursor atomic per entry + a scattered
//       8-byte store (k_far_csc, hot_split.hip), cursors from a prior scan;
//   (b) rocprim::radix_sort_pairs on the slot bits (key = slot, value = row).
// hipcc -O3 --offload-arch=gfx950 -I/opt/rocm/include tools/ubench_far_sort.hip -o /tmp/ubfs
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ void k_scatter(const uint32_t* slot, const uint32_t* row, int64_t n, unsigned long long* cur, uint2* out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = slot[i];
    const unsigned long long at = atomicAdd(&cur[s], 1ull);
    out[at] = make_uint2(row[i], s);
  }
}

__global__ void k_scatter32(const uint32_t* slot, const uint32_t* row, int64_t n, uint32_t* cur, uint2* out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = slot[i];
    const uint32_t at = atomicAdd(&cur[s], 1u);
    out[at] = make_uint2(row[i], s);
  }
}

// atomics only: the position goes to a coalesced store
__global__ void k_atomics_only(const uint32_t* slot, int64_t n, unsigned long long* cur, uint2* out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = slot[i];
    const unsigned long long at = atomicAdd(&cur[s], 1ull);
    out[i] = make_uint2(uint32_t(at), s);
  }
}

__global__ void k_pack(const uint32_t* ks, const uint32_t* vs, int64_t n, uint2* out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = make_uint2(vs[i], ks[i]);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 2000000;
  const uint32_t nslots = argc > 2 ? uint32_t(std::atoll(argv[2])) : 1000000u;
  const int reps = 20;
  std::mt19937 rng(7);
  std::vector<uint32_t> hs(static_cast<size_t>(n)), hr(static_cast<size_t>(n));
  std::vector<unsigned long long> hc(nslots + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    hs[size_t(i)] = rng() % nslots;
    hr[size_t(i)] = uint32_t(i / 3);
  }
  // rows in order (the engine reads the chunk lists row by row)
  for (int64_t i = 0; i < n; ++i) hc[hs[size_t(i)] + 1]++;
  for (uint32_t s = 0; s < nslots; ++s) hc[s + 1] += hc[s];
  uint32_t *ds, *dr, *ks2, *vs2;
  unsigned long long *dc0, *dc;
  uint2* out;
  CK(hipMalloc(&ds, n * 4));
  CK(hipMalloc(&dr, n * 4));
  CK(hipMalloc(&ks2, n * 4));
  CK(hipMalloc(&vs2, n * 4));
  CK(hipMalloc(&dc0, (nslots + 1) * 8));
  CK(hipMalloc(&dc, (nslots + 1) * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMemcpy(ds, hs.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, hr.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc0, hc.data(), (nslots + 1) * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms = 0;
  // (a) atomics + scatter (the cursor copy is part of the engine's scan: not timed)
  float tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpy(dc, dc0, (nslots + 1) * 8, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_scatter, dim3(2048), dim3(256), 0, 0, ds, dr, n, dc, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 1) tot += ms;
  }
  std::printf("n %lld slots %u  atomic scatter          : %8.1f us\n", (long long)n, nslots, 1e3 * tot / (reps - 2));
  tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpy(dc, dc0, (nslots + 1) * 8, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_atomics_only, dim3(2048), dim3(256), 0, 0, ds, n, dc, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 1) tot += ms;
  }
  std::printf("n %lld slots %u  64-bit atomics only     : %8.1f us\n", (long long)n, nslots, 1e3 * tot / (reps - 2));
  {
    std::vector<uint32_t> h32(nslots + 1);
    for (uint32_t s = 0; s <= nslots; ++s) h32[s] = uint32_t(hc[s]);
    uint32_t *c32, *c320;
    CK(hipMalloc(&c32, (nslots + 1) * 4));
    CK(hipMalloc(&c320, (nslots + 1) * 4));
    CK(hipMemcpy(c320, h32.data(), (nslots + 1) * 4, hipMemcpyHostToDevice));
    tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemcpy(c32, c320, (nslots + 1) * 4, hipMemcpyDeviceToDevice));
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_scatter32, dim3(2048), dim3(256), 0, 0, ds, dr, n, c32, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (r > 1) tot += ms;
    }
    std::printf("n %lld slots %u  32-bit atomic scatter   : %8.1f us\n", (long long)n, nslots, 1e3 * tot / (reps - 2));
  }
  int bits = 1;
  while ((1u << bits) < nslots) ++bits;
  size_t tmp_bytes = 0;
  CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, ds, ks2, dr, vs2, size_t(n), 0, bits));
  void* tmp;
  CK(hipMalloc(&tmp, tmp_bytes));
  for (int pack = 0; pack < 2; ++pack) {
    tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a));
      CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, ds, ks2, dr, vs2, size_t(n), 0, bits));
      if (pack) hipLaunchKernelGGL(k_pack, dim3(2048), dim3(256), 0, 0, ks2, vs2, n, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (r > 1) tot += ms;
    }
    std::printf("n %lld slots %u  rocprim sort (%2d bits)%s: %8.1f us  (temp %zu B)\n", (long long)n, nslots, bits,
                pack ? " + pack" : "       ", 1e3 * tot / (reps - 2), tmp_bytes);
  }
  // check: sorted keys ascending
  std::vector<uint32_t> ck(static_cast<size_t>(n));
  CK(hipMemcpy(ck.data(), ks2, n * 4, hipMemcpyDeviceToHost));
  bool ok = std::is_sorted(ck.begin(), ck.end());
  std::printf("sorted %s\n", ok ? "yes" : "NO");
  return ok ? 0 : 1;
}
