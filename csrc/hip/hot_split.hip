// Hybrid dense-hot layout of the SGD slot stream, built by the remap pass.
//
// A GD iteration streams every (row, bigram) entry of the batch twice (dot
// product, then gradient), and on tweet text the bigram distribution is very
// skewed: on the bench data the 128 most frequent of ~1.4K active bigrams
// carry 81 % of all entries.  Those hot slots are stored per row as 4-bit
// counts -- 128 nibbles = 64 B per row, 16 B per lane of the SELL-16x4 chunk
// -- and only the remaining cold entries stay in a SELL stream.  The hot
// gradient then accumulates in VGPRs instead of contended LDS atomics
// (sgd.hip, k_sgd_iter_hyb).  A hot id whose count in a row exceeds 15 stays
// cold for that row (every occurrence in its own lane), so the layout is
// exact for any text and a lane never holds more cold entries than before.
//
//   k_slot_hist      sampled slot histogram (every kHistChunks-th chunk of idx)
//   k_hot_select     top-kHot by binary search on the count threshold
//   k_remap_hybrid   replaces k_remap: one wave per 16-row chunk maps hashed
//                    ids to slots, counts hot slots per row in LDS, and writes
//                    the 4-bit hot counts plus each lane's cold entries
//
// Chunks with rows too long for the register-resident pass (L8 >
// kMaxRegGroups) get the plain u16 layout and clen8c = -1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "narrow_text.h"

namespace twtml {

namespace {

constexpr int kHistBlock = 1024;
constexpr int kSplitWaves = 4;

// One wave per sampled chunk (c % kHistChunks == 0: the lazy featurizer
// writes ids for exactly those fast chunks), all of its groups.
__global__ __launch_bounds__(kHistBlock) void k_slot_hist(DevPrepared p, int64_t pad_base, uint32_t* hist) {
  extern __shared__ uint32_t h[];
  for (int64_t s = threadIdx.x; s < pad_base; s += kHistBlock) h[s] = 0u;
  __syncthreads();
  const int lane = lane_id();
  const int64_t n_kept = p.counters[0];
  const int64_t nsamp = ((n_kept + kRowsPerChunk - 1) / kRowsPerChunk + kHistChunks - 1) / kHistChunks;
  const int64_t wave = (int64_t(blockIdx.x) * kHistBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * kHistBlock / kWave;
  for (int64_t sc = wave; sc < nsamp; sc += nwaves) {
    const int64_t c = sc * kHistChunks;
    const int32_t L8 = p.clen8[c];
    const int32_t* src = p.idx + p.cbase[c] * kChunkStride + lane * kGroup;
    for (int32_t g = 0; g < L8; ++g) {
      const int4* s4 = reinterpret_cast<const int4*>(src + int64_t(g) * kChunkStride);
      const int4 a = s4[0], b = s4[1];
      const int32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (v[e] >= 0) atomicAdd(&h[kNumNumeric + p.slot_of[v[e]]], 1u);
    }
  }
  __syncthreads();
  for (int64_t s = threadIdx.x; s < pad_base; s += kHistBlock)
    if (h[s]) atomicAdd(&hist[s], h[s]);
}

// Top-kHot slots by sampled count: the largest threshold T with at least
// kHot slots counting >= T (binary search, block-wide counts), then slots
// above T and the first ties at T get ids.  Zero counts are never hot.
__global__ __launch_bounds__(1024) void k_hot_select(const uint32_t* hist, int64_t ns, int64_t pad_base,
                                                     uint8_t* hot_of, int32_t* hot_slot) {
  __shared__ int32_t part[1024 / kWave];
  __shared__ uint32_t n_gt, n_eq;
  const int tid = threadIdx.x;
  auto count_ge = [&](uint32_t T) {
    int32_t c = 0;
    for (int64_t s = kNumNumeric + tid; s < pad_base; s += 1024) c += hist[s] >= T ? 1 : 0;
    c = wave_sum(c);
    __syncthreads();
    if (lane_id() == 0) part[tid / kWave] = c;
    __syncthreads();
    int32_t t = 0;
    for (int k = 0; k < 1024 / kWave; ++k) t += part[k];
    return t;
  };
  uint32_t lo = 1, hi = 0;   // answer in [lo, hi]: count_ge(lo) >= kHot
  {
    uint32_t m = 0;
    for (int64_t s = kNumNumeric + tid; s < pad_base; s += 1024) m = max(m, hist[s]);
    m = wave_max(m);
    __syncthreads();
    if (lane_id() == 0) part[tid / kWave] = int32_t(m);
    __syncthreads();
    for (int k = 0; k < 1024 / kWave; ++k) hi = max(hi, uint32_t(part[k]));
  }
  uint32_t T = 1;
  if (hi >= 1 && count_ge(1) > kHot) {
    while (lo < hi) {            // largest T with count_ge(T) >= kHot
      const uint32_t mid = lo + (hi - lo + 1) / 2;
      if (count_ge(mid) >= kHot) lo = mid; else hi = mid - 1;
    }
    T = lo;
  }
  // T = 1 with <= kHot non-zero slots: every non-zero slot is hot
  const int32_t above = count_ge(T + 1);            // strictly above T: < kHot
  const uint32_t need_eq = uint32_t(kHot - above);
  if (tid == 0) { n_gt = 0; n_eq = 0; }
  for (int h = tid; h < kHot; h += 1024) hot_slot[h] = int32_t(pad_base);   // unused ids
  __syncthreads();
  for (int64_t s = tid; s < ns; s += 1024) {
    uint32_t h = 0xFFu;
    if (s >= kNumNumeric && s < pad_base) {
      const uint32_t c = hist[s];
      if (c > T) {
        const uint32_t k = atomicAdd(&n_gt, 1u);
        if (k < uint32_t(kHot)) h = k;
      } else if (c == T && c > 0u) {
        const uint32_t k = atomicAdd(&n_eq, 1u);
        if (k < need_eq) h = uint32_t(above) + k;
      }
    }
    hot_of[s] = uint8_t(h);
    if (h != 0xFFu) hot_slot[h] = int32_t(s);
  }
}

__device__ __forceinline__ uint32_t pack2(uint32_t a, uint32_t b) { return a | (b << 16); }

constexpr int kCntStride = kHot / 2 + 4;
// Hashed ids below kCodeIds (every Java-hash bigram of Latin-1 text) are
// remapped through an LDS table of 16-bit codes: 0x8000 | hot id, or the
// compact slot.  Larger ids read slot_of / hot_of from global memory.
constexpr int kCodeIds = 8192;
constexpr uint32_t kCodeHot = 0x8000u;

// code[id] for id < kCodeIds (0xFFFF: id not active in this batch; never
// looked up, but slot_of is only defined for active ids -- checked via uniq)
__global__ __launch_bounds__(1024) void k_code_table(DevPrepared p, uint16_t* code) {
  const int id = blockIdx.x * 1024 + threadIdx.x;
  if (id >= kCodeIds) return;
  const int64_t nU = p.counters[1];
  uint32_t c = 0xFFFFu;
  if (id < p.flag_len) {
    const int32_t u = p.slot_of[id];
    if (u >= 0 && u < nU && p.uniq[u] == id) {
      const uint32_t sl = uint32_t(kNumNumeric + u);
      const uint32_t h = p.hot_of[sl];
      c = h != 0xFFu ? (kCodeHot | h) : sl;
    }
  }
  code[id] = uint16_t(c);
}

// Larger active ids carry their hot id in slot_of itself (k_code_tag:
// bit 31 hot, bits 16..23 hot id, bits 0..15 compact index), one dependent
// load per lookup instead of slot_of then hot_of.
constexpr uint32_t kTagHot = 0x80000000u;

__device__ __forceinline__ uint32_t slot_index(int32_t so) { return uint32_t(so) & 0xFFFFu; }

// Tiered layout: slot_of holds the (renumbered) slot itself, tagged hot
// (kTagHot | hot id << 16 | slot) or far (kTagFar | slot, 28 bits); the LDS
// code of a small far id is kCodeFar16 ("look slot_of up").  Codes are 32
// bit: kCodeHot | hot id, kCodeFar | far slot, or a near slot (< 2^14).
constexpr uint32_t kTagFar = 0x40000000u;
constexpr uint32_t kTagSlot = 0x0FFFFFFFu;
constexpr uint32_t kCodeFar16 = 0x4000u;
constexpr uint32_t kCodeFar = 0x40000000u;
static_assert(kMaxHybridSlots <= int(kCodeFar16), "near slots must stay below the far LDS code");

template <bool TIERED>
__device__ __forceinline__ uint32_t id_code(const uint16_t* lcode, const DevPrepared& p, int32_t id) {
  if (id < kCodeIds) {
    const uint32_t c = lcode[id];
    if (TIERED && c == kCodeFar16) return kCodeFar | (uint32_t(p.slot_of[id]) & kTagSlot);
    return c;
  }
  const uint32_t so = uint32_t(p.slot_of[id]);
  if (so & kTagHot) return kCodeHot | ((so >> 16) & 0xFFu);
  if (TIERED) return (so & kTagFar) ? (kCodeFar | (so & kTagSlot)) : (so & kTagSlot);
  return uint32_t(kNumNumeric) + (so & 0xFFFFu);
}

__global__ __launch_bounds__(1024) void k_code_tag(DevPrepared p, int64_t n_unique) {
  const int64_t u = int64_t(blockIdx.x) * 1024 + threadIdx.x;
  if (u >= n_unique) return;
  const int32_t id = p.uniq[u];
  if (id < kCodeIds) return;
  const uint32_t h = p.hot_of[kNumNumeric + u];
  p.slot_of[id] = int32_t(uint32_t(u) | (h != 0xFFu ? (kTagHot | (h << 16)) : 0u));
}

// One wave per 16-row chunk (SELL-16x4 input layout of featurize):
//   pass 1  ids -> codes; hot ids counted per row (LDS u16 pairs), cold
//           slots dealt round robin over the row's 4 lanes (an LDS counter
//           per row) and stored straight to the cold stream
//   dense   this lane's 32 hot ids of its row as 4-bit counts
//   rare    a hot id counting > 15 in a row: its entries are re-read and
//           appended cold the same way
//   pad     every lane's cold stream padded to the chunk's max group count
// Cold stream: groups of kColdGroup u16 per lane (8 B), entry k of lane l
// at cbase * 512 + (k / 4) * 256 + l * 4 + k % 4.  Dealing a row's cold
// entries over its lanes and 4-entry groups pad the chunk to ~12 slots per
// lane instead of ~19 (a lane kept the cold entries of its own text quarter,
// in 8-entry groups: 37 % of the cold stream was padding).
//   text    (from_text) fast chunks re-derive their ids from the raw text
//           (narrow_text.h) instead of reading idx
//   far     (TIERED) entries of far slots go to the chunk's far list
//           (row << 28 | slot, at cbase * 512 ..) and count into fhist
// NW waves per workgroup (the code table is loaded once per workgroup): 4,
// or 8 with a 6-waves-per-SIMD register budget (TWTML_REMAP_WAVES=8, A/B)
template <bool TIERED, int NW>
__global__ __launch_bounds__(NW * kWave) __attribute__((amdgpu_waves_per_eu(NW == 8 ? 6 : 1))) void k_remap_hybrid(DevPrepared p, int64_t ns,
                                                                      int64_t pad_base,
                                                                      const uint16_t* code,
                                                                      DevRawBatch rb, FeaturizeParams fp,
                                                                      int from_text) {
  __shared__ uint16_t lcode[kCodeIds];
  __shared__ uint32_t cnt[NW][kRowsPerChunk * kCntStride];
  __shared__ uint32_t ccnt[NW][kRowsPerChunk];
  __shared__ uint32_t fcnt[NW];
  for (int i = threadIdx.x; i < kCodeIds / 8; i += NW * kWave)
    reinterpret_cast<uint4*>(lcode)[i] = reinterpret_cast<const uint4*>(code)[i];
  __syncthreads();
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t wave = int64_t(blockIdx.x) * NW + w;
  const int64_t nwaves = int64_t(gridDim.x) * NW;
  uint32_t* cw = cnt[w];
  uint32_t* crow = cw + r * kCntStride;
  const uint32_t pad = uint32_t(pad_base + lane);
  uint16_t* plain = static_cast<uint16_t*>(p.slot);
  const NarrowHash nh(fp);
  const uint32_t near_end = uint32_t(p.near_end);

  // the next chunk's packed row-text words are loaded one chunk ahead
  const int64_t c_end = nch < fp.c_hi ? nch : fp.c_hi;   // this launch's chunk slice
  const int64_t c_first = fp.c_lo + wave;
  int64_t rt_next = (from_text && c_first < c_end) ? p.rtext[c_first * kRowsPerChunk + lane / kLanesPerRow] : 0;
  for (int64_t c = c_first; c < c_end; c += nwaves) {
    const int64_t rt = rt_next;
    if (from_text && c + nwaves < c_end) rt_next = p.rtext[(c + nwaves) * kRowsPerChunk + lane / kLanesPerRow];
    const int32_t L8 = p.clen8[c];
    const int64_t off = p.cbase[c] * kChunkStride + lane * kGroup;
    const int32_t* src = p.idx + off;
    uint32_t* flist = TIERED ? p.fslot + p.cbase[c] * kChunkStride : nullptr;
    if (TIERED) {
      if (lane == 0) fcnt[w] = 0u;
      wave_lds_sync();
    }
    auto far_put = [&](uint32_t cd) {   // TIERED: far entry of row r -> the chunk's far list
      const uint32_t sl = cd & kTagSlot;
      const uint32_t k = atomicAdd(&fcnt[w], 1u);
      flist[k] = (uint32_t(r) << 28) | sl;
      atomicAdd(reinterpret_cast<unsigned long long*>(&p.fhist[sl - near_end]), 1ull);
    };
    if (L8 > kMaxRegGroups) {   // plain layout (as k_remap)
      for (int32_t g = 0; g < L8; ++g) {
        const int4* s4 = reinterpret_cast<const int4*>(src + int64_t(g) * kChunkStride);
        const int4 a = s4[0], b = s4[1];
        const int32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t o[8];
        if constexpr (TIERED) {   // rare (rows of > 320 bigrams): far entries to the far list
          for (int e = 0; e < 8; ++e) {
            uint32_t x = pad;
            if (v[e] >= 0) {
              const uint32_t cd = id_code<true>(lcode, p, v[e]);
              if (cd & kCodeFar) far_put(cd);   // far codes carry a 28-bit slot: test first
              else if (cd & kCodeHot) x = uint32_t(p.hot_slot[cd & 0xFFu]);
              else x = cd;
            }
            o[e] = x;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = v[e] >= 0 ? uint32_t(kNumNumeric) + slot_index(p.slot_of[v[e]]) : pad;
        }
        *reinterpret_cast<uint4*>(plain + off + int64_t(g) * kChunkStride) =
            make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
      }
      if (TIERED) {
        wave_lds_sync();
        if (lane == 0) p.fcount[c] = int32_t(fcnt[w]);
      }
      if (lane == 0) p.clen8c[c] = -1;
      continue;
    }
    for (int i = lane; i < kRowsPerChunk * kCntStride; i += kWave) cw[i] = 0u;
    if (lane < kRowsPerChunk) ccnt[w][lane] = 0u;
    wave_lds_sync();
    uint16_t* dstc = p.cslot + p.cbase[c] * kChunkStride;   // the chunk's cold stream
    auto put = [&](uint32_t sl) {   // next cold entry of row r -> lane 4r + k % 4, position k / 4
      const uint32_t k = atomicAdd(&ccnt[w][r], 1u);
      const uint32_t kk = k >> 2;
      dstc[int64_t(kk / kColdGroup) * kColdStride + (kLanesPerRow * r + (k & 3)) * kColdGroup +
           (kk % kColdGroup)] = uint16_t(sl);
    };
    auto count = [&](uint32_t cd) {
      if (TIERED && (cd & kCodeFar)) {   // far codes carry a 28-bit slot (bit 15 may be set)
        far_put(cd);
      } else if (cd & kCodeHot) {
        const uint32_t h = cd & 0xFFu;
        atomicAdd(&crow[h >> 1], 1u << ((h & 1u) * 16));
      } else {
        put(cd);
      }
    };
    auto big = [&](uint32_t cd) {   // rare pass: hot ids counting > 15 in the row go cold
      if ((TIERED && (cd & kCodeFar)) || !(cd & kCodeHot)) return;
      const uint32_t h = cd & 0xFFu;
      if (((crow[h >> 1] >> ((h & 1u) * 16)) & 0xFFFFu) > 15u) put(uint32_t(p.hot_slot[h]));
    };
    const bool text = from_text && p.cfast[c];   // wave-uniform
    NarrowLane L;
    uint32_t a[kFastAl];
    if (text) {
      narrow_lane_load_rt(rb, c, n_kept, rt, L, a);
#pragma unroll
      for (int g = 0; g < kFastMaxQ / kGroup; ++g) {
        if (g >= L8) break;                               // wave-uniform
#pragma unroll
        for (int e8 = 0; e8 < kGroup; ++e8) {
          const int e = g * kGroup + e8;
          if (e < L.my) count(id_code<TIERED>(lcode, p, int32_t(narrow_id(L, a, e, nh))));
        }
      }
    } else {
      for (int32_t g = 0; g < L8; ++g) {
        const int4* s4 = reinterpret_cast<const int4*>(src + int64_t(g) * kChunkStride);
        const int4 a = s4[0], b = s4[1];
        const int32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        // the group's 8 codes first (their slot_of gathers in flight together:
        // a far entry's list store may alias slot_of, which kept the compiler
        // from hoisting the next entry's gather above it), then the counts
        uint32_t cd[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) cd[e] = v[e] >= 0 ? id_code<TIERED>(lcode, p, v[e]) : 0u;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] >= 0) count(cd[e]);
      }
    }
    wave_lds_sync();
    // dense part: this lane's 32 hot ids of its row; counts > 15 stay cold
    uint32_t nib[4] = {0u, 0u, 0u, 0u};
    bool ovf = false;
    {
      const uint4* c4 = reinterpret_cast<const uint4*>(crow + 16 * t);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 cv = c4[j];
        const uint32_t ws[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const uint32_t n = (ws[q] >> (16 * hh)) & 0xFFFFu;
            const int i = 8 * j + 2 * q + hh;          // hot id 32t + i
            if (n <= 15u) nib[i >> 3] |= n << (4 * (i & 7));
            else ovf = true;
          }
        }
      }
    }
    reinterpret_cast<uint4*>(p.hot_dense)[c * kWave + lane] = make_uint4(nib[0], nib[1], nib[2], nib[3]);
    if (__any(ovf)) {   // rare: a hot bigram more than 15 times in one row
      if (text) {   // reload the text (keeping a[] live here costs registers everywhere)
        uint32_t a2[kFastAl];
        narrow_lane_load_rt(rb, c, n_kept, rt, L, a2);
#pragma unroll
        for (int g = 0; g < kFastMaxQ / kGroup; ++g) {
          if (g >= L8) break;
#pragma unroll
          for (int e8 = 0; e8 < kGroup; ++e8) {
            const int e = g * kGroup + e8;
            if (e < L.my) big(id_code<TIERED>(lcode, p, int32_t(narrow_id(L, a2, e, nh))));
          }
        }
      } else {
        for (int32_t g = 0; g < L8; ++g) {
          const int4* s4 = reinterpret_cast<const int4*>(src + int64_t(g) * kChunkStride);
          const int4 a = s4[0], b = s4[1];
          const int32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (v[e] >= 0) big(id_code<TIERED>(lcode, p, v[e]));
        }
      }
    }
    wave_lds_sync();   // every cold entry of the chunk is counted
    if (TIERED && lane == 0) p.fcount[c] = int32_t(fcnt[w]);
    const uint32_t rc = ccnt[w][r];
    const int32_t mine = rc > uint32_t(t) ? int32_t((rc - uint32_t(t) + 3u) >> 2) : 0;   // this lane's entries
    const int32_t L4c = wave_max((mine + kColdGroup - 1) / kColdGroup);
    uint16_t* own = dstc + lane * kColdGroup;
    for (int32_t kk = mine; kk < L4c * kColdGroup; ++kk)    // pad this lane's stream
      own[int64_t(kk / kColdGroup) * kColdStride + kk % kColdGroup] = uint16_t(pad);
    if (lane == 0) p.clen8c[c] = L4c;
    wave_lds_sync();   // the next chunk clears / refills this wave's LDS
  }
}


// ---------------------------------------------------------------------------
// Tiered layout (active set beyond LDS).
// ---------------------------------------------------------------------------
// Sampled counts of compact slots [lo, hi) (slot_of still holds compact
// indices): LDS histogram of the range, non-zero bins flushed with one
// global atomic each.  Multiple ranges = multiple launches.
constexpr int kTierHistSpan = 32768;

// step: every step-th sampled chunk (the same subset in every span pass),
// so the passes over wide active sets cost one sampled pass in total.
__global__ __launch_bounds__(kHistBlock) void k_tier_hist(DevPrepared p, int64_t n_unique, int64_t step) {
  __shared__ uint32_t h[kTierHistSpan];
  const int64_t lo = int64_t(blockIdx.y) * kTierHistSpan;   // this workgroup's slot span
  const int64_t span = std::min<int64_t>(n_unique - lo, kTierHistSpan);
  for (int64_t i = threadIdx.x; i < span; i += kHistBlock) h[i] = 0u;
  __syncthreads();
  const int lane = lane_id();
  const int64_t n_kept = p.counters[0];
  const int64_t nsamp = ((n_kept + kRowsPerChunk - 1) / kRowsPerChunk + kHistChunks - 1) / kHistChunks;
  const int64_t wave = (int64_t(blockIdx.x) * kHistBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * kHistBlock / kWave;
  for (int64_t sc = wave * step; sc < nsamp; sc += nwaves * step) {
    const int64_t c = sc * kHistChunks;
    const int32_t L8 = p.clen8[c];
    const int32_t* src = p.idx + p.cbase[c] * kChunkStride + lane * kGroup;
    for (int32_t g = 0; g < L8; ++g) {
      const int4* s4 = reinterpret_cast<const int4*>(src + int64_t(g) * kChunkStride);
      const int4 a = s4[0], b = s4[1];
      const int32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (v[e] >= 0) {
          const int64_t u = p.slot_of[v[e]] - lo;
          if (u >= 0 && u < span) atomicAdd(&h[u], 1u);
        }
    }
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < span; i += kHistBlock)
    if (h[i]) atomicAdd(&p.slot_hist[kNumNumeric + lo + i], h[i]);
}

// Count buckets: exact below 2048, then 128 log-spaced buckets per octave
// (monotone in the count).
constexpr int kCountBuckets = 4096;
__device__ __forceinline__ int count_bucket(uint32_t c) {
  if (c < 2048u) return int(c);
  const int e = 31 - __builtin_clz(c);                 // >= 11
  const int b = 2048 + (e - 11) * 128 + int((c >> (e - 7)) & 127u);
  return b < kCountBuckets ? b : kCountBuckets - 1;
}

__global__ __launch_bounds__(1024) void k_tier_buckets(const uint32_t* hist, int64_t n, uint32_t* cb) {
  __shared__ uint32_t lb[kCountBuckets];
  for (int i = threadIdx.x; i < kCountBuckets; i += 1024) lb[i] = 0u;
  __syncthreads();
  for (int64_t u = int64_t(blockIdx.x) * 1024 + threadIdx.x; u < n; u += int64_t(gridDim.x) * 1024)
    atomicAdd(&lb[count_bucket(hist[u])], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < kCountBuckets; i += 1024)
    if (lb[i]) atomicAdd(&cb[i], lb[i]);
}

// Threshold bucket B: the K near slots are every slot in a bucket above B
// plus the first `need` slots (by compact index) of bucket B, i.e. B is the
// highest bucket whose suffix count reaches K.  One workgroup: thread t owns
// buckets [4t, 4t + 4), a block scan gives each thread the count above its
// range, the thread holding B publishes it.  (A single-thread walk over the
// 4096 buckets was 4096 dependent loads: 210 us per batch.)
__global__ __launch_bounds__(1024) void k_tier_threshold(const uint32_t* cb, int64_t K, int64_t* tparam) {
  constexpr int P = kCountBuckets / 1024;
  __shared__ int64_t above_s[1024];
  __shared__ int best;
  const int t = threadIdx.x;
  uint32_t c[P];
  int64_t mine = 0;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    c[k] = cb[t * P + k];
    mine += c[k];
  }
  above_s[t] = mine;
  if (t == 0) best = -1;
  __syncthreads();
  // inclusive suffix scan (Hillis-Steele): above_s[t] = sum of ranges >= t
  for (int off = 1; off < 1024; off <<= 1) {
    const int64_t v = t + off < 1024 ? above_s[t + off] : 0;
    __syncthreads();
    above_s[t] += v;
    __syncthreads();
  }
  int64_t run = above_s[t] - mine;   // count in buckets above this thread's range
  int found = -1;
  int64_t need = 0;
#pragma unroll
  for (int k = P - 1; k >= 0; --k) {
    if (found < 0 && run + int64_t(c[k]) >= K) {
      found = t * P + k;
      need = K - run;
    }
    run += c[k];
  }
  if (found >= 0) atomicMax(&best, found);
  __syncthreads();
  if (found >= 0 && found == best) {
    tparam[0] = found;
    tparam[1] = need;
  } else if (t == 0 && best < 0) {   // K beyond every slot (not produced by the host)
    tparam[0] = 0;
    tparam[1] = K - above_s[0];
  }
}

__global__ __launch_bounds__(1024) void k_tier_eqflag(const uint32_t* hist, int64_t n, const int64_t* tparam,
                                                      int64_t* flag) {
  const int B = int(tparam[0]);
  for (int64_t u = int64_t(blockIdx.x) * 1024 + threadIdx.x; u < n; u += int64_t(gridDim.x) * 1024)
    flag[u] = count_bucket(hist[u]) == B ? 1 : 0;
}

// eqrank (scanned) -> near flag, kept in newslot until the numbering pass
__global__ __launch_bounds__(1024) void k_tier_nearflag(const uint32_t* hist, int64_t n, const int64_t* tparam,
                                                        int64_t* scan, int32_t* newslot) {
  const int B = int(tparam[0]);
  const int64_t need = tparam[1];
  for (int64_t u = int64_t(blockIdx.x) * 1024 + threadIdx.x; u < n; u += int64_t(gridDim.x) * 1024) {
    const int b = count_bucket(hist[u]);
    const bool near = b > B || (b == B && scan[u] < need);
    newslot[u] = near ? 1 : 0;
    scan[u] = near ? 1 : 0;
  }
}

// near rank (scanned) -> slot numbering: near slots 4.., far from near_end
__global__ __launch_bounds__(1024) void k_tier_number(DevPrepared p, const uint32_t* hist, int64_t n,
                                                      const int64_t* scan) {
  const int64_t near_end = p.near_end;
  for (int64_t u = int64_t(blockIdx.x) * 1024 + threadIdx.x; u < n; u += int64_t(gridDim.x) * 1024) {
    const int64_t nr = scan[u];
    const bool near = p.newslot[u] != 0;
    const int64_t sl = near ? kNumNumeric + nr : near_end + (u - nr);
    p.newslot[u] = int32_t(sl);
    p.slot_fid[sl] = p.uniq[u];
    if (near) p.hist_near[sl] = hist[u];
  }
}

// Codes of small ids (LDS table) and tags of every active id (tiered).
__global__ __launch_bounds__(1024) void k_code_table_tiered(DevPrepared p, uint16_t* code) {
  const int id = blockIdx.x * 1024 + threadIdx.x;
  if (id >= kCodeIds) return;
  const int64_t nU = p.counters[1];
  uint32_t c = 0xFFFFu;
  if (id < p.flag_len) {
    const int32_t u = p.slot_of[id];
    if (u >= 0 && u < nU && p.uniq[u] == id) {
      const int64_t sl = p.newslot[u];
      if (sl >= p.near_end) {
        c = kCodeFar16;
      } else {
        const uint32_t h = p.hot_of[sl];
        c = h != 0xFFu ? (kCodeHot | h) : uint32_t(sl);
      }
    }
  }
  code[id] = uint16_t(c);
}

__global__ __launch_bounds__(1024) void k_code_tag_tiered(DevPrepared p, int64_t n_unique) {
  const int64_t u = int64_t(blockIdx.x) * 1024 + threadIdx.x;
  if (u >= n_unique) return;
  const int32_t id = p.uniq[u];
  const uint32_t sl = uint32_t(p.newslot[u]);
  uint32_t tag;
  if (int64_t(sl) >= p.near_end) {
    tag = kTagFar | sl;
  } else {
    const uint32_t h = p.hot_of[sl];
    tag = h != 0xFFu ? (kTagHot | (h << 16) | sl) : sl;
  }
  p.slot_of[id] = int32_t(tag);
}

// Far CSC: every far entry of every chunk list -> its slot's segment.
__global__ __launch_bounds__(256) void k_far_csc(DevPrepared p, int64_t c_lo, int64_t c_hi) {
  const int lane = lane_id();
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t wave = (int64_t(blockIdx.x) * 256 + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * 256 / kWave;
  const uint32_t near_end = uint32_t(p.near_end);
  for (int64_t c = c_lo + wave; c < nch && c < c_hi; c += nwaves) {
    const int32_t fc = p.fcount[c];
    const uint32_t* fl = p.fslot + p.cbase[c] * kChunkStride;
    for (int32_t k = lane; k < fc; k += kWave) {
      const uint32_t e = fl[k];
      const uint32_t sl = e & kTagSlot;
      const uint64_t at = atomicAdd(reinterpret_cast<unsigned long long*>(&p.fcur[sl - near_end]), 1ull);
      p.fcsc[at] = make_uint2(uint32_t(c * kRowsPerChunk + (e >> 28)), sl);
    }
  }
}

// k_remap_hybrid over the chunk range in prep_slices() launches; a
// persistent-style grid per launch (each workgroup loads the 16 KB code
// table once)
template <bool TIERED>
void launch_remap_slices(const DevPrepared& p, int64_t ns, int64_t pad_base, int64_t cmax, int num_cu,
                         const DevRawBatch& b, const FeaturizeParams& fp, bool from_text, hipStream_t s) {
  const int nsl = prep_slices();
  for (int k = 0; k < nsl; ++k) {
    FeaturizeParams f = fp;
    f.c_lo = cmax * k / nsl;
    f.c_hi = cmax * (k + 1) / nsl;
    if (f.c_hi <= f.c_lo) continue;
    static const int nw = [] {
      const char* e = std::getenv("TWTML_REMAP_WAVES");
      return e && std::atoi(e) == 8 ? 8 : kSplitWaves;
    }();
    int grid = int(std::min<int64_t>(int64_t(num_cu) * 4 * prep_grid_mult(TIERED ? 4 : 1) * kSplitWaves / nw,
                                     (f.c_hi - f.c_lo + nw - 1) / nw));
    if (grid < 1) grid = 1;
    if (nw == 8)
      TWTML_LAUNCH((k_remap_hybrid<TIERED, 8>), dim3(grid), dim3(8 * kWave), 0, s, p, ns, pad_base, p.code, b, f,
                   from_text ? 1 : 0);
    else
      TWTML_LAUNCH((k_remap_hybrid<TIERED, kSplitWaves>), dim3(grid), dim3(kSplitWaves * kWave), 0, s, p, ns,
                   pad_base, p.code, b, f, from_text ? 1 : 0);
  }
}

}  // namespace

void launch_remap_hybrid(const DevPrepared& p, int64_t entries, int64_t ns, int64_t pad_base, int num_cu,
                         const DevRawBatch& b, const FeaturizeParams& fp, bool from_text, hipStream_t s) {
  if (ns > kMaxHybridSlots) throw std::invalid_argument("hybrid layout: too many active slots");
  if (entries == 0) return;
  // slot_hist was zeroed by launch_prep_init
  const int64_t cmax = (p.cap_rows + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t nsamp = (cmax + kHistChunks - 1) / kHistChunks;
  int gh = int((nsamp + kHistBlock / kWave - 1) / (kHistBlock / kWave));
  gh = std::max(1, std::min(gh, num_cu));
  TWTML_LAUNCH(k_slot_hist, dim3(gh), dim3(kHistBlock), size_t(pad_base) * sizeof(uint32_t), s,
                     p, pad_base, p.slot_hist);
  TWTML_LAUNCH(k_hot_select, dim3(1), dim3(1024), 0, s, p.slot_hist, ns, pad_base, p.hot_of,
                     p.hot_slot);
  TWTML_LAUNCH(k_code_table, dim3(kCodeIds / 1024), dim3(1024), 0, s, p, p.code);
  const int64_t nU = pad_base - kNumNumeric;
  if (nU > 0) TWTML_LAUNCH(k_code_tag, dim3(int((nU + 1023) / 1024)), dim3(1024), 0, s, p, nU);
  launch_remap_slices<false>(p, ns, pad_base, cmax, num_cu, b, fp, from_text, s);
}


void launch_tier_hist(const DevPrepared& p, int64_t n_unique, int num_cu, hipStream_t s) {
  // slot_hist[4 .. 4 + nU) zeroed by the caller
  const int64_t cmax = (p.cap_rows + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t nsamp = (cmax + kHistChunks - 1) / kHistChunks;
  // one LDS-privatised pass per 32K-slot span; each reads every step-th
  // sampled chunk, step = number of spans (the near tier only needs the
  // frequency order of the top slots: ~1/100 of the entries at 200K slots)
  const int64_t step = std::max<int64_t>(1, (n_unique + kTierHistSpan - 1) / kTierHistSpan);
  // every span in one launch (blockIdx.y), the CUs shared out among them:
  // one workgroup (128 KB of LDS) per CU, no span waiting for another
  const int64_t spans = step;
  int gh = int((nsamp / step + kHistBlock / kWave - 1) / (kHistBlock / kWave));
  gh = std::max(1, std::min<int>(gh, int(std::max<int64_t>(1, num_cu / spans))));
  TWTML_LAUNCH(k_tier_hist, dim3(gh, unsigned(spans)), dim3(kHistBlock), 0, s, p, n_unique, step);
}

int64_t tier_near_cap() {
  // LDS slot space 4 + n_near + pads (rounded to 64) must fit the hybrid
  // kernel plus the tiered kernel's far-dot scratch
  for (int64_t n = kMaxHybridSlots; n >= 64; n -= 64) {
    const int64_t nl = (kNumNumeric + n + kPadSlots + 63) / 64 * 64;
    if (nl <= kMaxHybridSlots && sgd_hybrid_fits(nl)) return n;
  }
  return 0;
}

__global__ __launch_bounds__(1024) void k_tier_zero(uint32_t* buckets, uint32_t* hist_near, uint64_t* fhist,
                                                    int64_t n_fhist) {
  const int64_t i0 = int64_t(blockIdx.x) * 1024 + threadIdx.x, st = int64_t(gridDim.x) * 1024;
  for (int64_t i = i0; i < kCountBuckets; i += st) buckets[i] = 0u;
  for (int64_t i = i0; i < kMaxHybridSlots; i += st) hist_near[i] = 0u;
  for (int64_t i = i0; i < n_fhist; i += st) fhist[i] = 0ull;
}

void launch_tier_layout(const DevPrepared& p, int64_t entries, int64_t n_unique, int64_t n_near, int64_t ns,
                        int64_t nl, int num_cu, const DevRawBatch& b, const FeaturizeParams& fp, bool from_text,
                        hipStream_t s) {
  if (n_unique + kNumNumeric + kPadSlots >= (int64_t(1) << 28)) throw std::invalid_argument("tiered layout: too many active slots");
  if (nl > kMaxHybridSlots) throw std::invalid_argument("tiered layout: near tier exceeds LDS");
  const uint32_t* hist = p.slot_hist + kNumNumeric;
  const int g = int(std::max<int64_t>(1, std::min<int64_t>((n_unique + 1023) / 1024, int64_t(num_cu) * 4)));
  // count buckets: 4096 u32 after the cap_tier + 1 scan elements of tscan
  uint32_t* buckets = reinterpret_cast<uint32_t*>(p.tscan + p.cap_tier + 1);
  const int64_t n_far = kNumNumeric + n_unique - p.near_end;
  // the count buckets, the near-slot histogram and the far counts zeroed in
  // one launch (three fills before; each prep-stream launch waits for a gap
  // between the GD loop's kernels)
  TWTML_LAUNCH(k_tier_zero, dim3(int(std::min<int64_t>(256, (n_far + 1 + 1023) / 1024 + 1))), dim3(1024), 0, s,
                     buckets, p.hist_near, p.fhist, n_far + 1);
  TWTML_LAUNCH(k_tier_buckets, dim3(g), dim3(1024), 0, s, hist, n_unique, buckets);
  TWTML_LAUNCH(k_tier_threshold, dim3(1), dim3(1024), 0, s, buckets, n_near, p.tparam);
  TWTML_LAUNCH(k_tier_eqflag, dim3(g), dim3(1024), 0, s, hist, n_unique, p.tparam, p.tscan);
  launch_scan_excl(p.tscan, p.tscan, n_unique, p.tparam + 3, p.tscan_blk, s);
  TWTML_LAUNCH(k_tier_nearflag, dim3(g), dim3(1024), 0, s, hist, n_unique, p.tparam, p.tscan, p.newslot);
  launch_scan_excl(p.tscan, p.tscan, n_unique, p.tparam + 3, p.tscan_blk, s);
  TWTML_LAUNCH(k_tier_number, dim3(g), dim3(1024), 0, s, p, hist, n_unique, p.tscan);
  // hot ids among the near slots (new numbering)
  TWTML_LAUNCH(k_hot_select, dim3(1), dim3(1024), 0, s, p.hist_near, nl, p.near_end, p.hot_of,
                     p.hot_slot);
  TWTML_LAUNCH(k_code_table_tiered, dim3(kCodeIds / 1024), dim3(1024), 0, s, p, p.code);
  TWTML_LAUNCH(k_code_tag_tiered, dim3(int((n_unique + 1023) / 1024)), dim3(1024), 0, s, p, n_unique);
  if (entries > 0) {
    const int64_t cmax = (p.cap_rows + kRowsPerChunk - 1) / kRowsPerChunk;
    launch_remap_slices<true>(p, ns, p.near_end, cmax, num_cu, b, fp, from_text, s);
  }
  // CSC offsets (exclusive scan of the far counts, in place), cursors, scatter
  // CSC offsets, and the scatter cursors as a second copy of them
  launch_scan_excl(reinterpret_cast<const int64_t*>(p.fhist), reinterpret_cast<int64_t*>(p.fhist), n_far,
                   p.tparam + 2, p.tscan_blk, s, reinterpret_cast<int64_t*>(p.fcur));
  if (entries > 0) {
    const int64_t cmax = (p.cap_rows + kRowsPerChunk - 1) / kRowsPerChunk;
    const int nsl = prep_slices();
    for (int k = 0; k < nsl; ++k) {   // chunk slices (prep_slices)
      const int64_t lo = cmax * k / nsl, hi = cmax * (k + 1) / nsl;
      if (hi <= lo) continue;
      const int grid = int(std::max<int64_t>(1, std::min<int64_t>((hi - lo + 3) / 4, int64_t(num_cu) * 8 * prep_grid_mult(4))));
      TWTML_LAUNCH(k_far_csc, dim3(grid), dim3(256), 0, s, p, lo, hi);
    }
  }
}

}  // namespace twtml
