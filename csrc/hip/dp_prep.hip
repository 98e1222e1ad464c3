// DP batch preparation: the one prep collective per batch (SURVEY §2.5 CS3,
// CS4 and the active-set union of CS2).
//
// Each rank prepares its shard of batch t+1 locally (decode .. featurize ..
// its own active ids + sampled counts) on the prep stream while batch t
// trains, then packs ONE packet:
//   [ header: 16 int64 -- kept rows, active ids, batch bounds (8 fp64) ]
//   [ (id, sampled count) pairs, padded with id -1 to the largest rank's ]
// The training thread all-gathers the packets on the compute stream between
// two GD iterations of batch t (engine.cpp issue_c1: a point every rank
// reaches in the same collective order), and the prep thread finishes batch
// t+1 from the gathered packets without any further collective: union of the
// ids (flags + compaction), per-slot summed counts (the tiered layout's near
// tier), global kept rows / sampling offsets / bounds from the headers.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace twtml {

__global__ __launch_bounds__(kBlock) void k_pack_c1(DevPrepared p, const double* bounds, int32_t* packet) {
  const int64_t nU = p.counters[1];
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i == 0) {
    int64_t* h = reinterpret_cast<int64_t*>(packet);
    h[0] = p.counters[0];
    h[1] = nU;
    for (int k = 0; k < kBoundsLen; ++k) h[2 + k] = __builtin_bit_cast(int64_t, bounds[k]);
    for (int k = 2 + kBoundsLen; k < kC1HeaderWords / 2; ++k) h[k] = 0;
  }
  for (int64_t u = i; u < nU; u += int64_t(gridDim.x) * kBlock) {
    int32_t* pr = packet + kC1HeaderWords + 2 * u;
    pr[0] = p.uniq[u];
    pr[1] = int32_t(p.slot_hist[kNumNumeric + u]);
  }
}

void launch_pack_c1(const DevPrepared& p, const double* bounds, int32_t* packet, int64_t n_unique, hipStream_t s) {
  const int grid = int(std::max<int64_t>(1, std::min<int64_t>((n_unique + kBlock - 1) / kBlock, 2048)));
  TWTML_LAUNCH(k_pack_c1, dim3(grid), dim3(kBlock), 0, s, p, bounds, packet);
}

// Flag every id of every rank's gathered pairs (-1: padding).
__global__ __launch_bounds__(kBlock) void k_union_flag(const int32_t* gathered, int world, int64_t max_u,
                                                       uint8_t* flags, int64_t flag_len) {
  const int64_t pw = c1_packet_words(max_u);
  const int64_t n = int64_t(world) * max_u;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int64_t r = i / max_u, u = i - r * max_u;
    const int32_t id = gathered[r * pw + kC1HeaderWords + 2 * u];
    if (id >= 0 && id < flag_len) flags[id] = 1;
  }
}

void launch_union_flag(const int32_t* gathered, int world, int64_t max_u, const DevPrepared& p, hipStream_t s) {
  const int64_t n = int64_t(world) * max_u;
  if (n <= 0) return;
  const int grid = int(std::min<int64_t>((n + kBlock - 1) / kBlock, 4096));
  TWTML_LAUNCH(k_union_flag, dim3(grid), dim3(kBlock), 0, s, gathered, world, max_u, p.flags, p.flag_len);
}

// Summed sampled counts of the union slots: hist[4 + slot_of[id]] += count.
__global__ __launch_bounds__(kBlock) void k_union_hist(const int32_t* gathered, int world, int64_t max_u,
                                                       const int32_t* slot_of, uint32_t* hist) {
  const int64_t pw = c1_packet_words(max_u);
  const int64_t n = int64_t(world) * max_u;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int64_t r = i / max_u, u = i - r * max_u;
    const int32_t* pr = gathered + r * pw + kC1HeaderWords + 2 * u;
    const int32_t id = pr[0];
    if (id >= 0 && pr[1] != 0) atomicAdd(&hist[kNumNumeric + slot_of[id]], uint32_t(pr[1]));
  }
}

void launch_union_hist(const int32_t* gathered, int world, int64_t max_u, const DevPrepared& p, hipStream_t s) {
  const int64_t n = int64_t(world) * max_u;
  if (n <= 0) return;
  const int grid = int(std::min<int64_t>((n + kBlock - 1) / kBlock, 4096));
  TWTML_LAUNCH(k_union_hist, dim3(grid), dim3(kBlock), 0, s, gathered, world, max_u, p.slot_of, p.slot_hist);
}

}  // namespace twtml
