// Shared device/host helpers for the MI355X (gfx950, CDNA4) engine.
//
// Wave64 everywhere: reductions use 64-lane DPP/shuffles, masks are 64-bit.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "debug.h"   // TWTML_LAUNCH (debug sync points), teardown errors, host registrations

#define TWTML_HIP_CHECK(expr)                                                            \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);      \
  } while (0)

namespace twtml {

constexpr int kWave = 64;
constexpr int kBlock = 256;          // 4 waves per workgroup
constexpr int kLanesPerRow = 4;      // a row's entries are dealt round-robin to 4 lanes
constexpr int kRowsPerChunk = kWave / kLanesPerRow;  // 16 rows per chunk (one wave)
constexpr int kGroup = 8;            // entries per lane per 16-byte slot load (u16 slots)
constexpr int kChunkStride = kWave * kGroup;  // entries per (chunk, group) = 512
constexpr int kMaxRegGroups = 10;    // groups a lane keeps in VGPRs (row nnz <= 320)
constexpr int kNumNumeric = 4;       // numeric features (MllibHelper.scala:13)
constexpr int kPadSlots = 64;        // one zero-weight pad slot per lane
constexpr int kLenBuckets = 4096;    // counting-sort buckets for row length

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// fp32 wave sum on the VALU (no LDS permute traffic): DPP quad permutes and
// row rotates inside each 16-lane row, then the four row totals through
// v_readlane.  Every lane returns the total.  (The gfx950
// v_permlane{16,32}_swap builtins are avoided: with both operands the same
// value the compiler read one swap result twice -- wrong sums, measured.)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float rdlane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// per-row sum over the 4 lanes of each quad-column: lanes j, j+4, j+8, j+12 of a row
__device__ __forceinline__ float row_sum_mod4(float v) {
  v += dpp_mov<0x124>(v);   // row_ror:4
  v += dpp_mov<0x128>(v);   // row_ror:8
  return v;
}
__device__ __forceinline__ float wave_sum_f32(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]: lane ^ 2
  v = row_sum_mod4(v);      // every lane: its 16-lane row total
  return (rdlane(v, 0) + rdlane(v, 16)) + (rdlane(v, 32) + rdlane(v, 48));
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

// LDS hand-off between the lanes of one wave (no other wave touches the
// region): drain this wave's LDS traffic, then re-converge.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v |= uint32_t(__shfl_xor(int(v), off, kWave));
  return v;
}

// Block-wide sum for kBlock threads; `scratch` needs kBlock/kWave entries.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x / kWave;
  __syncthreads();
  if (lane_id() == 0) scratch[w] = v;
  __syncthreads();
  T r = T(0);
  const int nw = blockDim.x / kWave;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// Bit-identical to oracle.mllib.sgd_uniform (Bernoulli row sampling).
__device__ __forceinline__ double sample_uniform(uint64_t seed, uint64_t row) {
  const uint64_t key = row ^ (seed * 0xD1B54A32D192ED03ULL);
  return double(splitmix64(key) >> 11) * (1.0 / 9007199254740992.0);
}

// Utils.round: BigDecimal HALF_UP = round half away from zero.
__device__ __forceinline__ double round_half_away(double x) {
  const double t = trunc(x);
  return fabs(x - t) >= 0.5 ? t + (x > 0 ? 1.0 : -1.0) : t;
}

// x mod d for 32-bit x and a runtime divisor, without an integer division
// (Lemire, Kaser & Kurz 2019: M = floor((2^64 - 1) / d) + 1, then
// mod = hi64((M * x mod 2^64) * d)).  One 64-bit division per thread setup.
struct FastMod32 {
  uint64_t M = 1;
  uint32_t d = 1;
  __device__ __forceinline__ explicit FastMod32(uint32_t div) : M(~0ull / div + 1ull), d(div) {}
  __device__ __forceinline__ uint32_t mod(uint32_t x) const {
    return uint32_t(__umul64hi(M * uint64_t(x), uint64_t(d)));
  }
};
#endif

inline int ceil_div(long long a, long long b) { return int((a + b - 1) / b); }

}  // namespace twtml
