// Sparse snapshot of the fp64 master weights for non-blocking checkpoints
// (SURVEY §5 checkpoint row; VERDICT r2 missing #5).
//
// MLlib's Saveable layout stores the weights as a VectorUDT, sparse when
// under 25 % of them are non-zero -- the usual case for hashed text weights at
// F = 1e8 (checkpoint/saveable.py).  Instead of copying all F+4 fp64 weights
// to the host (800 MB at F = 1e8) and scanning them there on the training
// thread, the engine compacts the non-zeros on the device, stream-ordered
// right behind the batch the checkpoint is taken after:
//   k_nz_count  one count per chunk of kSnapChunk weights (ballot popcounts)
//   k_nz_scan   one workgroup: exclusive chunk offsets + the total
//   k_nz_write  ordered (index, value) pairs, one tile of kBlock at a time
// Two streaming passes over the weights (HBM-bound: ~0.3 ms at F = 1e8); the
// writer thread then copies only the pairs to the host on its own stream
// (engine.cpp snapshot_fetch) while training goes on.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace twtml {

__device__ __forceinline__ uint32_t nz_prefix(uint64_t mask) {
  // set bits of `mask` below this lane
  return uint32_t(__builtin_amdgcn_mbcnt_hi(uint32_t(mask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mask), 0u)));
}

__global__ __launch_bounds__(kBlock) void k_nz_count(const double* __restrict__ w, int64_t n,
                                                     uint32_t* __restrict__ cnt) {
  __shared__ uint32_t red[kBlock / kWave];
  const int64_t b0 = int64_t(blockIdx.x) * kSnapChunk;
  const int64_t b1 = std::min<int64_t>(n, b0 + kSnapChunk);
  uint32_t c = 0;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += kBlock) c += (w[i] != 0.0) ? 1u : 0u;
  c = block_sum(c, red);
  if (threadIdx.x == 0) cnt[blockIdx.x] = c;
}

// Exclusive offsets of `nb` chunk counts (one workgroup); off[nb] = total,
// also published to the host word `host_total` (page-locked, mapped).
__global__ __launch_bounds__(kBlock) void k_nz_scan(const uint32_t* __restrict__ cnt, int64_t nb,
                                                    int64_t* __restrict__ off, volatile int64_t* host_total) {
  __shared__ int64_t part[kBlock];
  const int64_t per = (nb + kBlock - 1) / kBlock;
  const int64_t a = int64_t(threadIdx.x) * per, e = std::min<int64_t>(nb, a + per);
  int64_t s = 0;
  for (int64_t i = a; i < e; ++i) s += cnt[i];
  part[threadIdx.x] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan of the kBlock thread sums
  for (int d = 1; d < kBlock; d <<= 1) {
    const int64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t run = part[threadIdx.x] - s;   // exclusive
  for (int64_t i = a; i < e; ++i) {
    off[i] = run;
    run += cnt[i];
  }
  if (threadIdx.x == kBlock - 1) {
    off[nb] = part[kBlock - 1];
    *host_total = part[kBlock - 1];
  }
}

__global__ __launch_bounds__(kBlock) void k_nz_write(const double* __restrict__ w, int64_t n,
                                                     const int64_t* __restrict__ off, int32_t* __restrict__ idx,
                                                     double* __restrict__ val) {
  __shared__ uint32_t wtot[kBlock / kWave];
  const int64_t b0 = int64_t(blockIdx.x) * kSnapChunk;
  const int64_t b1 = std::min<int64_t>(n, b0 + kSnapChunk);
  const int wv = threadIdx.x / kWave;
  int64_t base = off[blockIdx.x];
  for (int64_t t0 = b0; t0 < b1; t0 += kBlock) {
    const int64_t i = t0 + threadIdx.x;
    const double x = i < b1 ? w[i] : 0.0;
    const bool nz = x != 0.0;
    const uint64_t m = __ballot(nz);
    if (lane_id() == 0) wtot[wv] = uint32_t(__popcll(m));
    __syncthreads();
    uint32_t before = 0, tile = 0;
#pragma unroll
    for (int k = 0; k < kBlock / kWave; ++k) {
      before += k < wv ? wtot[k] : 0u;
      tile += wtot[k];
    }
    if (nz) {
      const int64_t o = base + before + nz_prefix(m);
      idx[o] = int32_t(i);
      val[o] = x;
    }
    base += tile;
    __syncthreads();   // wtot is rewritten by the next tile
  }
}

int64_t snapshot_chunks(int64_t n) { return (n + kSnapChunk - 1) / kSnapChunk; }

void launch_snapshot(const double* w, int64_t n, uint32_t* cnt, int64_t* off, int32_t* idx, double* val,
                     volatile int64_t* host_total, hipStream_t s) {
  const int64_t nb = snapshot_chunks(n);
  if (nb <= 0) return;
  TWTML_LAUNCH(k_nz_count, dim3(unsigned(nb)), dim3(kBlock), 0, s, w, n, cnt);
  TWTML_LAUNCH(k_nz_scan, dim3(1), dim3(kBlock), 0, s, cnt, nb, off, host_total);
  TWTML_LAUNCH(k_nz_write, dim3(unsigned(nb)), dim3(kBlock), 0, s, w, n, off, idx, val);
}

}  // namespace twtml
