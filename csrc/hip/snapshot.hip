// Sparse snapshot of the fp64 master weights for non-blocking checkpoints
// (SURVEY §5 checkpoint row; VERDICT r2 missing #5).
//
// MLlib's Saveable layout stores the weights as a VectorUDT, sparse when
// under 25 % of them are non-zero -- the usual case for hashed text weights at
// F = 1e8 (checkpoint/saveable.py).  Instead of copying all F+4 fp64 weights
// to the host (800 MB at F = 1e8) and scanning them there on the training
// thread, the engine compacts the non-zeros on the device, stream-ordered
// right behind the batch the checkpoint is taken after:
//   k_nz_pack   per chunk of kSnapChunk weights: its ordered (index, value)
//               pairs packed at the chunk's own base in a scratch pair array,
//               and its count
//   k_nz_scan   one workgroup: exclusive chunk offsets + the total
//   k_nz_move   every chunk's pairs to their final offset
// One streaming pass over the weights (800 MB at F = 1e8) plus the pairs
// (12 B per non-zero) twice: the weights were read twice before (count, then
// write), and every GD workgroup that meets a snapshot workgroup on its CU
// waits for it -- the snapshot's device time is the batch's p99 cost.  The
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

// Marks of 4 consecutive weights (one byte each) as 4 bits, the lowest
// address in bit 0.
__device__ __forceinline__ uint32_t mark_bits(uint32_t v) {
  return ((v & 0xFFu) ? 1u : 0u) | ((v & 0xFF00u) ? 2u : 0u) | ((v & 0xFF0000u) ? 4u : 0u) |
         ((v & 0xFF000000u) ? 8u : 0u);
}

// touched (nullable): a weight never written is zero and is not read -- at
// F = 1e8 the model's non-zeros are a few percent of the array, so most
// lines of the 800 MB weight array are never fetched (100 MB of marks are).
// A lane takes kNzPer consecutive weights per tile: their marks in one
// 16-byte load, then only the marked weights; pairs are placed by a wave
// scan of the lanes' counts and one workgroup step per 4096 weights (was
// one lane and one workgroup step per weight / per 256: 183 us per call at
// F = 1e8, the checkpoint gate's kernel trace).
constexpr int kNzPer = 16;
static_assert(kSnapChunk % (kBlock * kNzPer) == 0, "a chunk is whole tiles");
__global__ __launch_bounds__(kBlock) void k_nz_pack(const double* __restrict__ w,
                                                    const uint8_t* __restrict__ touched, int64_t n,
                                                    int32_t* __restrict__ tidx, double* __restrict__ tval,
                                                    uint32_t* __restrict__ cnt) {
  __shared__ uint32_t wtot[kBlock / kWave];
  const int64_t b0 = int64_t(blockIdx.x) * kSnapChunk;
  const int64_t b1 = std::min<int64_t>(n, b0 + kSnapChunk);
  const int wv = threadIdx.x / kWave, lane = lane_id();
  int64_t base = b0;   // the chunk's pairs at its own base (<= kSnapChunk of them)
  for (int64_t t0 = b0; t0 < b1; t0 += int64_t(kBlock) * kNzPer) {
    const int64_t i0 = t0 + int64_t(threadIdx.x) * kNzPer;
    uint32_t mk = 0;   // bit j: weight i0 + j may be non-zero
    if (i0 + kNzPer <= b1) {
      if (touched != nullptr) {   // i0 is a multiple of 16: an aligned 16-byte load
        const uint4 v = *reinterpret_cast<const uint4*>(touched + i0);
        mk = mark_bits(v.x) | (mark_bits(v.y) << 4) | (mark_bits(v.z) << 8) | (mark_bits(v.w) << 12);
      } else {
        mk = (1u << kNzPer) - 1u;
      }
    } else {
      for (int j = 0; j < kNzPer; ++j)
        if (i0 + j < b1 && (touched == nullptr || touched[i0 + j] != 0)) mk |= 1u << j;
    }
    double x[kNzPer];
    uint32_t nzm = 0;
#pragma unroll
    for (int j = 0; j < kNzPer; ++j) x[j] = ((mk >> j) & 1u) ? w[i0 + j] : 0.0;
#pragma unroll
    for (int j = 0; j < kNzPer; ++j) nzm |= x[j] != 0.0 ? (1u << j) : 0u;
    const uint32_t c = uint32_t(__popc(nzm));
    uint32_t incl = c;   // inclusive scan of the lanes' counts
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t y = uint32_t(__shfl_up(int(incl), d, kWave));
      if (lane >= d) incl += y;
    }
    if (lane == kWave - 1) wtot[wv] = incl;
    __syncthreads();
    uint32_t before = 0, tile = 0;
#pragma unroll
    for (int k = 0; k < kBlock / kWave; ++k) {
      before += k < wv ? wtot[k] : 0u;
      tile += wtot[k];
    }
    if (nzm != 0) {
      int64_t o = base + before + (incl - c);
#pragma unroll
      for (int j = 0; j < kNzPer; ++j) {
        if ((nzm >> j) & 1u) {
          tidx[o] = int32_t(i0 + j);
          tval[o] = x[j];
          ++o;
        }
      }
    }
    base += tile;
    __syncthreads();   // wtot is rewritten by the next tile
  }
  if (threadIdx.x == 0) cnt[blockIdx.x] = uint32_t(base - b0);
}

__global__ __launch_bounds__(kBlock) void k_nz_move(const int32_t* __restrict__ tidx,
                                                    const double* __restrict__ tval,
                                                    const uint32_t* __restrict__ cnt,
                                                    const int64_t* __restrict__ off, int32_t* __restrict__ idx,
                                                    double* __restrict__ val) {
  const int64_t b0 = int64_t(blockIdx.x) * kSnapChunk, o = off[blockIdx.x];
  const int64_t c = cnt[blockIdx.x];
  for (int64_t j = threadIdx.x; j < c; j += kBlock) {
    idx[o + j] = tidx[b0 + j];
    val[o + j] = tval[b0 + j];
  }
}

int64_t snapshot_chunks(int64_t n) { return (n + kSnapChunk - 1) / kSnapChunk; }

__global__ __launch_bounds__(kBlock) void k_mark_nonzero(const double* __restrict__ w, uint8_t* __restrict__ touched,
                                                         int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    touched[i] = w[i] != 0.0 ? 1 : 0;
}

void launch_mark_nonzero(const double* w, uint8_t* touched, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  TWTML_LAUNCH(k_mark_nonzero, dim3(unsigned(std::min<int64_t>((n + kBlock - 1) / kBlock, 8192))), dim3(kBlock), 0,
               s, w, touched, n);
}

void launch_snapshot(const double* w, const uint8_t* touched, int64_t n, uint32_t* cnt, int64_t* off,
                     int32_t* tidx, double* tval, int32_t* idx, double* val, volatile int64_t* host_total,
                     hipStream_t s) {
  const int64_t nb = snapshot_chunks(n);
  if (nb <= 0) return;
  TWTML_LAUNCH(k_nz_pack, dim3(unsigned(nb)), dim3(kBlock), 0, s, w, touched, n, tidx, tval, cnt);
  TWTML_LAUNCH(k_nz_scan, dim3(1), dim3(kBlock), 0, s, cnt, nb, off, host_total);
  TWTML_LAUNCH(k_nz_move, dim3(unsigned(nb)), dim3(kBlock), 0, s, tidx, tval, cnt, off, idx, val);
}

}  // namespace twtml
