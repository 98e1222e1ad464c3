// Ingest-side kernels: filter (K3), length sort, SELL layout, bigram
// hashing + numeric features (K1+K2), active-set compaction and remap.
//
// Reference semantics: MllibHelper.filtrate / featurize
// (spark/src/main/scala/com/giorgioinf/twtml/spark/MllibHelper.scala:42-95).
//
// Layout produced for the SGD kernels ("SELL-16x4", length-sorted):
//   kept rows are sorted by descending bigram count and cut into chunks of
//   16 rows; a chunk is one wave, each row owns 4 consecutive lanes and its
//   entries are dealt round-robin to them (entry j -> lane 4r + j%4, local
//   position jj = j/4).  A chunk owns clen8[c] groups; local entry jj of
//   lane l lives at
//       (cbase[c] + jj/8) * 512 + l * 8 + jj % 8
//   so one 16-byte load gives a lane 8 u16 slots and a wave reads 1 KiB
//   contiguous per instruction.  Padding entries point at a per-lane
//   zero-weight pad slot.  Row-level arrays (y, num, perm) are indexed by the
//   sorted position p = 16c + r.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>

#include "../common/unicode_tables.h"
#include "common.h"
#include "kernels.h"
#include "narrow_text.h"
#include "text_stage.h"

namespace twtml {

// ---------------------------------------------------------------------------
// Generic single-workgroup exclusive scan (int64), in-place safe.  A tile of
// 1024 x kScanPer elements is loaded coalesced into LDS (thread t takes
// elements t, t+1024, ...: one memory latency per tile), then each thread
// scans kScanPer consecutive LDS elements, the thread totals are scanned
// with wave shuffles + one LDS pass, and the tile is stored coalesced.
// (A thread reading its consecutive elements straight from global memory
// makes every load instruction touch 64 cache lines: 16 us per tile.)
// ---------------------------------------------------------------------------
constexpr int kScanPer = 8;
constexpr int kScanTile = 1024 * kScanPer;   // single-block scans: 1024 threads
// Multi-block scans run 256-thread blocks over 2048-element tiles: on the
// prep stream every block waits for free wave slots on a CU the GD loop
// shares, and a 1024-thread block needs 16 of them (k_tile_sum 33 us under
// overlap for ~1 us of work, round 5).
constexpr int kScanBT = 256;
constexpr int kScanTileBig = kScanBT * kScanPer;

// Sum of ts[0, b) over the BT threads of a block (every thread gets it).
// The multi-block scans take their tile's carry from the UNSCANNED tile sums
// this way (a few hundred values at most) instead of a separate
// single-block scan launch between the two passes: on the prep stream every
// launch waits for a gap between the GD loop's kernels.
template <int BT>
__device__ __forceinline__ int64_t block_prefix_of_sums(const int64_t* ts, int64_t b, int64_t* wsum) {
  int64_t c = 0;
  for (int64_t j = threadIdx.x; j < b; j += BT) c += ts[j];
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  int64_t t = 0;
#pragma unroll
  for (int k = 0; k < BT / 64; ++k) t += wsum[k];
  __syncthreads();
  return t;
}

// Block b scans [b * span, min(n, (b + 1) * span)) starting from the sum of
// tile_sums[0, b) (0 without tile_sums); single block: span = n.  out2, if
// given, receives the same values.  total: the grand total (written by the
// last block).
template <int BT>
__global__ __launch_bounds__(BT) void k_scan_excl(const int64_t* in, int64_t* out, int64_t n,
                                                  int64_t* total, const int64_t* tile_sums = nullptr,
                                                  int64_t span = 0, int64_t* out2 = nullptr) {
  constexpr int kTile = BT * kScanPer;
  constexpr int kW = BT / 64;
  __shared__ int64_t tile_v[kTile + kTile / 32];   // +1 word per 32: fewer bank conflicts
  __shared__ int64_t wsum[kW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto at = [](int i) { return i + (i >> 5); };
  int64_t carry = tile_sums ? block_prefix_of_sums<BT>(tile_sums, blockIdx.x, wsum) : 0;
  const int64_t b0 = tile_sums ? int64_t(blockIdx.x) * span : 0;
  const int64_t b1 = tile_sums ? (b0 + span < n ? b0 + span : n) : n;
  for (int64_t base = b0; base < b1; base += kTile) {
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      const int64_t i = base + k * BT + tid;
      tile_v[at(k * BT + tid)] = i < b1 ? in[i] : 0;
    }
    __syncthreads();
    int64_t v[kScanPer];
    int64_t tsum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      v[k] = tile_v[at(tid * kScanPer + k)];
      tsum += v[k];
    }
    int64_t x = tsum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int64_t woff = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      const int64_t ws = wsum[k];
      woff += k < w ? ws : 0;
      tot += ws;
    }
    int64_t run = carry + woff + x - tsum;   // exclusive prefix of this thread's first element
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      tile_v[at(tid * kScanPer + k)] = run;
      run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      const int64_t i = base + k * BT + tid;
      if (i < b1) {
        const int64_t v = tile_v[at(k * BT + tid)];
        out[i] = v;
        if (out2) out2[i] = v;
      }
    }
    carry += tot;
    __syncthreads();
  }
  if (tid == 0 && total && blockIdx.x == gridDim.x - 1) *total = carry;
}

// Tile sums for the multi-block scan: block b sums in[b * tile, ...).
template <int BT>
__global__ __launch_bounds__(BT) void k_tile_sum(const int64_t* in, int64_t n, int64_t* tsum) {
  __shared__ int64_t wsum[BT / 64];
  int64_t v = 0;
  const int64_t b0 = int64_t(blockIdx.x) * (BT * kScanPer);
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = b0 + k * BT + threadIdx.x;
    v += i < n ? in[i] : 0;
  }
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int k = 0; k < BT / 64; ++k) t += wsum[k];
    tsum[blockIdx.x] = t;
  }
}

static void scan_excl(const int64_t* in, int64_t* out, int64_t n, int64_t* total, hipStream_t s,
                      int64_t* out2 = nullptr) {
  TWTML_LAUNCH(k_scan_excl<1024>, dim3(1), dim3(1024), 0, s, in, out, n, total, nullptr, int64_t(0), out2);
}

// Multi-block exclusive scan (in place safe): tile sums, then every tile
// scanned from the sum of the tile sums before it -- two launches.
// tsum: ceil(n / kScanTileBig) + 1.
static void scan_excl_big(const int64_t* in, int64_t* out, int64_t n, int64_t* total, int64_t* tsum,
                          hipStream_t s, int64_t* out2 = nullptr) {
  if (n <= kScanTile) {
    scan_excl(in, out, n, total, s, out2);
    return;
  }
  const int tiles = int((n + kScanTileBig - 1) / kScanTileBig);
  TWTML_LAUNCH(k_tile_sum<kScanBT>, dim3(tiles), dim3(kScanBT), 0, s, in, n, tsum);
  TWTML_LAUNCH(k_scan_excl<kScanBT>, dim3(tiles), dim3(kScanBT), 0, s, in, out, n, total,
                     static_cast<const int64_t*>(tsum), int64_t(kScanTileBig), out2);
}

void launch_scan_excl(const int64_t* in, int64_t* out, int64_t n, int64_t* total, int64_t* tsum, hipStream_t s,
                      int64_t* out2) {
  scan_excl_big(in, out, n, total, tsum, s, out2);
}

void scan_excl_launch(const int64_t* in, int64_t* out, int64_t n, int64_t* total, hipStream_t s) {
  scan_excl(in, out, n, total, s);
}

// Packed row words -> offsets [n+1] + flags [n], a three-phase scan over
// tiles of 8192 rows (one 1024-thread block, 8 consecutive rows per thread
// = one 16-byte load): tile sums, a scan of the ~120 tile sums, then each
// tile's block-level exclusive scan plus its tile offset.
constexpr int kRowTile = 8192;

__device__ __forceinline__ void row_words(const uint16_t* rp, int64_t n, int64_t i0, uint32_t (&w)[8]) {
  if (i0 + 8 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(rp + i0);
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[2 * k] = d[k] & 0xFFFFu;
      w[2 * k + 1] = d[k] >> 16;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = i0 + k < n ? uint32_t(rp[i0 + k]) : 0u;
  }
}

__device__ __forceinline__ int64_t block_excl_scan_1024(int64_t v, int64_t* wsum, int64_t* total) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  int64_t x = v;   // inclusive wave scan
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int64_t y = __shfl_up(x, off, kWave);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int k = 0; k < 1024 / kWave; ++k) {
      const int64_t t = wsum[k];
      wsum[k] = acc;
      acc += t;
    }
    *total = acc;
  }
  __syncthreads();
  return wsum[w] + x - v;
}

__global__ __launch_bounds__(1024) void k_rows_tilesum(const uint16_t* rp, int64_t n, int64_t* tsum) {
  __shared__ int64_t wsum[1024 / kWave];
  __shared__ int64_t total;
  const int64_t i0 = int64_t(blockIdx.x) * kRowTile + int64_t(threadIdx.x) * 8;
  uint32_t w[8];
  row_words(rp, n, i0, w);
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += w[k] & ((1u << kRowLenBits) - 1u);
  (void)block_excl_scan_1024(s, wsum, &total);
  if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_rows_scan(const uint16_t* rp, int64_t n, const int64_t* tsum,
                                                    int64_t* offsets, uint8_t* flags) {
  __shared__ int64_t wsum[1024 / kWave];
  __shared__ int64_t total;
  const int64_t i0 = int64_t(blockIdx.x) * kRowTile + int64_t(threadIdx.x) * 8;
  uint32_t w[8];
  row_words(rp, n, i0, w);
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += w[k] & ((1u << kRowLenBits) - 1u);
  const int64_t carry = block_prefix_of_sums<1024>(tsum, blockIdx.x, wsum);
  int64_t o = carry + block_excl_scan_1024(s, wsum, &total);
  if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) offsets[n] = carry + total;   // total bytes
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (i0 + k < n) {
      offsets[i0 + k] = o;
      flags[i0 + k] = uint8_t(w[k] >> kRowLenBits);
    }
    o += w[k] & ((1u << kRowLenBits) - 1u);
  }
}

void launch_unpack_rows(const uint16_t* rowpack, int64_t n, int64_t* offsets, uint8_t* flags, int64_t* tsum,
                        hipStream_t s) {
  if (n <= 0) {
    TWTML_HIP_CHECK(hipMemsetAsync(offsets, 0, sizeof(int64_t), s));
    return;
  }
  const int tiles = int((n + kRowTile - 1) / kRowTile);
  TWTML_LAUNCH(k_rows_tilesum, dim3(tiles), dim3(1024), 0, s, rowpack, n, tsum);
  TWTML_LAUNCH(k_rows_scan, dim3(tiles), dim3(1024), 0, s, rowpack, n, tsum, offsets, flags);
}

// ---------------------------------------------------------------------------
// cesu wire rows (csrc/host/wire.h) and UTF-8 rows (load_utf8) -> UTF-16LE
// rows after the wire bytes.  A row of B wire bytes has at most B units (a
// 4-byte UTF-8 sequence is 2 units), so it expands into
// [tail + 2 * start, tail + 2 * end): no count or scan pass.  A wave takes 64
// rows; lane l owns row l's offsets / flags, and the wave walks the flagged
// rows among them (ballot) together.  An all-ASCII row (UTF-8 ingest: most
// tweets) is only checked -- 4 bytes per lane per step -- and stays a narrow
// row in place.  Otherwise 64 bytes per step: a unit starts at every
// non-continuation byte (two at a 4-byte lead: the surrogate pair), its index
// is the running count plus popcounts of the lead masks below the lane.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lanes_below() {
  return (uint64_t(1) << lane_id()) - 1u;
}

__device__ __forceinline__ int64_t bcast_lane64(int64_t v, int l) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int32_t(uint32_t(v)), l));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int32_t(uint32_t(uint64_t(v) >> 32)), l));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// Byte readers of the decode: the wave's staged LDS copy of its 64-row group,
// or global memory (groups too long to stage).
struct GlobalBytes {
  const uint8_t* text;
  __device__ __forceinline__ uint32_t byte(int64_t i) const { return text[i]; }
  __device__ __forceinline__ uint32_t dword(int64_t w) const { return *reinterpret_cast<const uint32_t*>(text + w); }
};
struct LdsBytes {
  const uint8_t* lds;   // staged bytes of [a0, a0 + staged)
  int64_t a0;
  __device__ __forceinline__ uint32_t byte(int64_t i) const { return lds[i - a0]; }
  __device__ __forceinline__ uint32_t dword(int64_t w) const {
    return *reinterpret_cast<const uint32_t*>(lds + (w - a0));
  }
};

// Row class from its bytes (aligned dwords, bytes outside [o, e) masked
// off): 0 ASCII, 1 Latin-1 (valid UTF-8 whose bytes are all < 0xC4, i.e.
// every code point < U+0100), 2 other.
template <typename Src>
__device__ __forceinline__ int row_class(const Src& src, int64_t o, int64_t e) {
  const int64_t a0 = o & ~int64_t(3);
  uint32_t acc = 0;
  bool big = false;
  for (int64_t w = a0 + 4 * lane_id(); w < e; w += 4 * kWave) {
    uint32_t v = src.dword(w);
    if (w < o) v &= 0xFFFFFFFFu << (8 * (o - w));
    if (w + 4 > e) v &= 0xFFFFFFFFu >> (8 * (w + 4 - e));
    acc |= v;
#pragma unroll
    for (int k = 0; k < 4; ++k) big |= ((v >> (8 * k)) & 0xFFu) >= 0xC4u;
  }
  if (__any(big)) return 2;
  return __any((acc & 0x80808080u) != 0u) ? 1 : 0;
}

// Byte flags of a dword -> a 4-bit mask: `x` holds 0/1 in bits 0, 8, 16, 24.
__device__ __forceinline__ uint32_t byte_bits(uint32_t x) {
  return (x * 0x10204080u) >> 28;   // the four products land on bits 28..31, no carries
}

// Bytes of x equal to b (per byte: bit 7 set), exact (no borrow between bytes).
__device__ __forceinline__ uint32_t bytes_eq(uint32_t x, uint32_t b) {
  const uint32_t t = x ^ (b * 0x01010101u);
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}

// UTF-8 byte pairs that start a unit whose lower-casing is not one UTF-16
// unit per unit (rows.hip's special rows): C4 B0 (U+0130), CE A3 (U+03A3,
// Final_Sigma), F0 90 / F0 91 / F0 96 / F0 9E (the planes of the astral
// cased letters: Deseret, Osage, Old Hungarian, Warang Citi, Medefaidrin,
// Adlam; emoji, F0 9F, are not), and ED A0: a high surrogate D800..D83F
// written as its own 3-byte sequence (CESU-8 / Java's modified UTF-8: the
// same astral letters as a surrogate pair of 3-byte sequences).
// A superset of the special rows: the normaliser checks every flagged row
// exactly.  v: four bytes, n: the byte after each of them.
__device__ __forceinline__ uint32_t special_pairs(uint32_t v, uint32_t n) {
  const uint32_t c4 = bytes_eq(v, 0xC4u), ce = bytes_eq(v, 0xCEu), f0 = bytes_eq(v, 0xF0u);
  const uint32_t ed = bytes_eq(v, 0xEDu);
  if (!(c4 | ce | f0 | ed)) return 0u;   // most multi-byte text (CJK, Cyrillic, Arabic, ...) has none of the leads
  uint32_t m = (c4 & bytes_eq(n, 0xB0u)) | (ce & bytes_eq(n, 0xA3u)) | (ed & bytes_eq(n, 0xA0u));
  if (f0)
    m |= f0 & (bytes_eq(n, 0x90u) | bytes_eq(n, 0x91u) | bytes_eq(n, 0x96u) | bytes_eq(n, 0x9Eu));
  return m;
}

// One decode step of row [o, e) (class 1 or 2, output at text + d0): the
// lane's aligned dword v of the row at w0 + 4 lane (and the next one, v2,
// for the continuation bytes of its leads); k = the row's units so far.
// A lane takes an aligned dword of the row per step (256 bytes per wave
// step: a tweet is one or two steps).  A unit starts at every
// non-continuation byte (two at a 4-byte lead: the surrogate pair); a lane's
// units (0..8) are ranked across the wave from four ballots of their bit
// planes.
// UTF-16 (class 2) rows also OR their special-pair candidates into `spec`
// (the lane's dword, bytes inside the row, each paired with the byte after
// it): one check per dword here, where all 64 lanes walk the row together.
__device__ __forceinline__ void decode_step(uint8_t* text, int64_t o, int32_t ie, int64_t d0, bool nar,
                                            int64_t w0, uint32_t v, uint32_t v2, int32_t& k, uint32_t& spec) {
  uint16_t* dst = reinterpret_cast<uint16_t*>(text + d0);
  uint8_t* dst8 = text + d0;
  const int lane = lane_id();
  const uint64_t below = lanes_below();
  const int32_t iw = int32_t(w0 - o) + 4 * lane;   // the lane's dword, relative to o (>= -3)
  // bytes j of the dword inside the row: 0 <= iw + j < ie
  const int32_t lo = iw < 0 ? -iw : 0;
  const int32_t hi = ie - iw >= 4 ? 4 : (ie - iw < 0 ? 0 : ie - iw);
  const uint32_t rng = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
  if (!nar) {
    const uint32_t bm = (hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u)) & ~((1u << (8 * lo)) - 1u);
    const uint32_t vm = v & bm;
    if (vm & 0x80808080u) spec |= special_pairs(vm, (v >> 8) | (v2 << 24));
  }
  // a 4-byte lead also needs iw + j + 3 < ie
  const int32_t h3 = ie - iw - 3;
  const uint32_t rng3 = h3 >= 4 ? 0xFu : (h3 <= 0 ? 0u : (1u << h3) - 1u);
  // lead: top two bits != 10; 4-byte lead: top nibble 1111 (SWAR over the dword)
  const uint32_t t = ((v >> 6) & 0x03030303u) ^ 0x02020202u;
  const uint32_t lead = byte_bits(((t + 0x7F7F7F7Fu) >> 7) & 0x01010101u) & rng;
  const uint32_t f = ((v >> 4) & 0x0F0F0F0Fu) + 0x01010101u;
  const uint32_t four = byte_bits((f >> 4) & 0x01010101u) & lead & rng3;
  const uint32_t cnt = uint32_t(__popc(lead) + __popc(four));
  const uint64_t p0 = __ballot(cnt & 1u), p1 = __ballot(cnt & 2u), p2 = __ballot(cnt & 4u),
                 p3 = __ballot(cnt & 8u);
  int32_t at = k + __popcll(p0 & below) + 2 * __popcll(p1 & below) + 4 * __popcll(p2 & below) +
               8 * __popcll(p3 & below);
  const uint64_t q = uint64_t(v) | (uint64_t(v2) << 32);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!((lead >> j) & 1u)) continue;
    const uint32_t c0 = uint32_t(q >> (8 * j)) & 0xFFu;
    const uint32_t c1 = uint32_t(q >> (8 * j + 8)) & 0x3Fu;
    const uint32_t c2 = uint32_t(q >> (8 * j + 16)) & 0x3Fu;
    if ((four >> j) & 1u) {
      const uint32_t c3 = uint32_t(q >> (8 * j + 24)) & 0x3Fu;
      const uint32_t cp = ((c0 & 0x07u) << 18) | (c1 << 12) | (c2 << 6) | c3;
      dst[at] = uint16_t(0xD800u + ((cp - 0x10000u) >> 10));
      dst[at + 1] = uint16_t(0xDC00u + ((cp - 0x10000u) & 0x3FFu));
      at += 2;
    } else {
      uint32_t u = c0;
      if (c0 >= 0xE0u) u = ((c0 & 0x0Fu) << 12) | (c1 << 6) | c2;
      else if (c0 >= 0x80u) u = ((c0 & 0x1Fu) << 6) | c1;
      if (nar) dst8[at] = uint8_t(u);
      else dst[at] = uint16_t(u);
      at += 1;
    }
  }
  k += __popcll(p0) + 2 * __popcll(p1) + 4 * __popcll(p2) + 8 * __popcll(p3);
}

// Decode row [o, e) (class 1 or 2) to dst (tail + 2 o); returns its units.
template <typename Src>
__device__ __forceinline__ int64_t decode_row(const Src& src, uint8_t* text, int64_t o, int64_t e, int64_t d0,
                                              bool nar, bool& sp) {
  const int32_t ie = int32_t(e - o);   // row bytes (< 2^13)
  int32_t k = 0;
  uint32_t spec = 0;
  for (int64_t w0 = o & ~int64_t(3); w0 < e; w0 += 4 * kWave) {
    const int32_t iw = int32_t(w0 - o) + 4 * lane_id();
    uint32_t v = 0, v2 = 0;
    if (iw < ie) {
      v = src.dword(w0 + 4 * lane_id());
      v2 = src.dword(w0 + 4 * lane_id() + 4);
    }
    decode_step(text, o, ie, d0, nar, w0, v, v2, k, spec);
  }
  sp = __any(spec != 0u);
  return k;
}

// Two staged rows decoded in lock step: their LDS reads are issued together
// and their two ballot / store chains interleave.  (One row at a time the
// per-row chain -- LDS read, SWAR, four ballots, stores -- left the decode
// latency-bound at ~0.1 instructions per cycle per SIMD.)
__device__ __forceinline__ void decode_rows2(const LdsBytes& src, uint8_t* text, int64_t oA, int64_t eA,
                                             int64_t d0A, bool narA, int32_t& kA, int64_t oB, int64_t eB,
                                             int64_t d0B, bool narB, int32_t& kB, bool& spA, bool& spB) {
  const int32_t ieA = int32_t(eA - oA), ieB = int32_t(eB - oB);
  const int lane = lane_id();
  kA = 0;
  kB = 0;
  uint32_t sA = 0, sB = 0;
  int64_t wA = oA & ~int64_t(3), wB = oB & ~int64_t(3);
  while (wA < eA || wB < eB) {
    const bool actA = wA < eA, actB = wB < eB;   // wave-uniform
    const bool okA = actA && int32_t(wA - oA) + 4 * lane < ieA;
    const bool okB = actB && int32_t(wB - oB) + 4 * lane < ieB;
    // unconditional reads of a valid staged address, selected after
    const int64_t aA = okA ? wA + 4 * lane : src.a0, aB = okB ? wB + 4 * lane : src.a0;
    uint32_t vA = src.dword(aA), v2A = src.dword(aA + 4);
    uint32_t vB = src.dword(aB), v2B = src.dword(aB + 4);
    if (!okA) vA = v2A = 0u;
    if (!okB) vB = v2B = 0u;
    if (actA) {
      decode_step(text, oA, ieA, d0A, narA, wA, vA, v2A, kA, sA);
      wA += 4 * kWave;
    }
    if (actB) {
      decode_step(text, oB, ieB, d0B, narB, wB, vB, v2B, kB, sB);
      wB += 4 * kWave;
    }
  }
  spA = __any(sA != 0u);
  spB = __any(sB != 0u);
}

// One lane's row class from the staged bytes [lo, le) (as row_class).
__device__ __forceinline__ int lane_row_class(const uint8_t* lbuf, int lo, int le) {
  uint32_t acc = 0, big = 0;
  for (int w = lo & ~3; w < le; w += 4) {
    uint32_t v = *reinterpret_cast<const uint32_t*>(lbuf + w);
    if (w < lo) v &= 0xFFFFFFFFu << (8 * (lo - w));
    if (w + 4 > le) v &= 0xFFFFFFFFu >> (8 * (w + 4 - le));
    acc |= v;
    big |= v & ((v & 0x7F7F7F7Fu) + 0x3C3C3C3Cu);   // a byte >= 0xC4 sets its bit 7
  }
  if (big & 0x80808080u) return 2;
  return (acc & 0x80808080u) ? 1 : 0;
}

// LDS staging per wave: the 64 rows of a group are consecutive on the wire,
// so their bytes are one range, loaded with 16-B loads (8 per lane in
// flight) -- one memory round trip per group instead of several per row.
// bytes per wave (groups beyond: two windows, or global reads): 6 KB leaves
// room for 6 workgroups (24 waves) per CU; r5 same-box A/B, decode under
// overlap 12 KB 466 us, 8 KB 436, 6 KB 414, 4 KB 455 (profiles/r5/ab_decode_stage.txt)
constexpr int kDecStage = 6144;
constexpr int kDecWaves = 4;

__global__ __launch_bounds__(kDecWaves * kWave) void k_cesu_decode(uint8_t* text, const int64_t* offsets,
                                                                   uint8_t* flags, int64_t n, int64_t tail,
                                                                   int64_t* rstart, int64_t* rend,
                                                                   int64_t* stats, int32_t* special) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kDecWaves][kDecStage + 16];
  const int lane = lane_id();
  const int wv = threadIdx.x / kWave;
  uint8_t* lbuf = stage[wv];
  const int64_t wave = (int64_t(blockIdx.x) * kDecWaves * kWave + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * kDecWaves;
  const GlobalBytes gsrc{text};
  int n_nar = 0;
  for (int64_t g = wave; g * kWave < n; g += nwaves) {
    const int64_t r = g * kWave + lane;
    uint8_t fl = r < n ? flags[r] : 0;
    const bool mine = r < n && (fl & kRowCesu);
    int64_t s0 = r < n ? offsets[r] : 0, s1 = r < n ? offsets[r + 1] : 0;
    // windows of consecutive rows whose bytes fit the wave's staging buffer
    // (a whole 64-row group when it fits; long multi-byte groups take two):
    // a group walked from global memory pays a memory round trip per row
    // step and became the kernel's tail
    uint64_t todo = __ballot(mine);
    while (todo) {
      const int lf = __builtin_ctzll(todo);
      const int64_t a0 = bcast_lane64(s0, lf) & ~int64_t(15);
      const uint64_t fit = __ballot(r < n && lane >= lf && s1 - a0 <= kDecStage);
      uint64_t win, m;
      bool staged = (fit >> lf) & 1u;
      if (staged) {   // offsets grow with the lane: the fitting rows are lanes lf..lk
        const int lk = 63 - __builtin_clzll(fit);
        win = (lk == 63 ? ~uint64_t(0) : ((uint64_t(1) << (lk + 1)) - 1u)) & ~((uint64_t(1) << lf) - 1u);
        const int64_t ge = bcast_lane64(s1, lk);
        const int64_t nq = (ge - a0 + 15) >> 4;   // 16-B chunks
        for (int64_t q0 = 0; q0 < nq; q0 += 8 * kWave) {
          uint4 v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int64_t q = q0 + j * kWave + lane;
            v[j] = q < nq ? *reinterpret_cast<const uint4*>(text + a0 + 16 * q) : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int64_t q = q0 + j * kWave + lane;
            if (q < nq) *reinterpret_cast<uint4*>(lbuf + 16 * q) = v[j];
          }
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
      } else {   // a single row longer than the buffer: from global memory
        win = uint64_t(1) << lf;
      }
      m = todo & win;
      todo &= ~win;
      const LdsBytes lsrc{lbuf, a0};
      // staged: every lane classifies its own row from LDS (aligned dwords),
      // so ASCII rows -- most tweets -- leave the wave's per-row walk entirely
      int my_cls = -1;
      if (staged) {
        const bool in_win = (m >> lane) & 1u;
        if (in_win) my_cls = lane_row_class(lbuf, int(s0 - a0), int(s1 - a0));
        if (my_cls == 0) fl = uint8_t(fl & ~kRowCesu);
        m = __ballot(my_cls > 0);
      }
      if (staged) {   // m holds class 1 / 2 rows only: two at a time
        while (m) {
          const int lA = __builtin_ctzll(m);
          m &= m - 1;
          const bool two = m != 0;
          const int lB = two ? __builtin_ctzll(m) : lA;
          if (two) m &= m - 1;
          const int64_t oA = bcast_lane64(s0, lA), eA = bcast_lane64(s1, lA);
          // a lone last row runs as row B with an empty extent
          const int64_t oB = two ? bcast_lane64(s0, lB) : (eA & ~int64_t(3));
          const int64_t eB = two ? bcast_lane64(s1, lB) : oB;
          const bool narA = __builtin_amdgcn_readlane(my_cls, lA) == 1;
          const bool narB = two && __builtin_amdgcn_readlane(my_cls, lB) == 1;
          const int64_t d0A = tail + 2 * oA, d0B = tail + 2 * oB;
          int32_t kA = 0, kB = 0;
          bool spA = false, spB = false;
          decode_rows2(lsrc, text, oA, eA, d0A, narA, kA, oB, eB, d0B, narB, kB, spA, spB);
          if (lane == lA) {
            s0 = d0A;
            s1 = d0A + (narA ? kA : 2 * kA);
            fl = narA ? uint8_t(fl & ~kRowCesu) : uint8_t((fl & ~kRowCesu) | kRowWide | (spA ? kRowSpecial : 0));
          }
          if (two && lane == lB) {
            s0 = d0B;
            s1 = d0B + (narB ? kB : 2 * kB);
            fl = narB ? uint8_t(fl & ~kRowCesu) : uint8_t((fl & ~kRowCesu) | kRowWide | (spB ? kRowSpecial : 0));
          }
          n_nar += (narA ? 1 : 0) + (narB ? 1 : 0);
        }
      }
      while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        // the row's extents from lane l's registers (a load here would put a
        // memory round trip on every row of the wave's sequential walk)
        const int64_t o = bcast_lane64(s0, l), e = bcast_lane64(s1, l);
        const int cls = staged ? __builtin_amdgcn_readlane(my_cls, l) : row_class(gsrc, o, e);
        if (cls == 0) {   // ASCII: narrow row as it is
          if (lane == l) fl = uint8_t(fl & ~kRowCesu);
          continue;
        }
        // Latin-1 rows decode straight to narrow bytes (no UTF-16 pass, no
        // narrowing pass in k_row_normalize); others to UTF-16
        const bool nar = cls == 1;
        const int64_t d0 = tail + 2 * o;
        bool sp = false;
        const int64_t k = staged ? decode_row(lsrc, text, o, e, d0, nar, sp) : decode_row(gsrc, text, o, e, d0, nar, sp);
        if (lane == l) {
          s0 = d0;
          s1 = d0 + (nar ? k : 2 * k);
          fl = nar ? uint8_t(fl & ~kRowCesu) : uint8_t((fl & ~kRowCesu) | kRowWide | (sp ? kRowSpecial : 0));
        }
        n_nar += nar ? 1 : 0;
      }
      __builtin_amdgcn_wave_barrier();   // LDS reads of this window precede the next staging
    }
    if (r < n) {
      rstart[r] = s0;
      rend[r] = s1;
      if (mine) flags[r] = fl;
    }
    if (special) {   // the group's special rows onto the list (~0.3 % of rows: one atomic per wave that has any)
      const bool sp = mine && (fl & kRowSpecial);
      const uint64_t bm = __ballot(sp);
      if (bm) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(reinterpret_cast<unsigned long long*>(&stats[2]), (unsigned long long)__popcll(bm));
        base = (unsigned long long)bcast_lane64(int64_t(base), 0);
        if (sp) special[int64_t(base) + __popcll(bm & lanes_below())] = int32_t(r);
      }
    }
  }
  if (stats && lane == 0 && n_nar) atomicAdd(reinterpret_cast<unsigned long long*>(&stats[1]), (unsigned long long)n_nar);
}

void launch_cesu_expand(uint8_t* text, const int64_t* offsets, uint8_t* flags, int64_t n, int64_t tail,
                        int64_t* rstart, int64_t* rend, int64_t* stats, hipStream_t s, int32_t* special) {
  if (special && !stats) throw std::invalid_argument("cesu_expand: the special-row list needs stats[2]");
  if (n <= 0) return;
  // one wave per 64-row group, 4 waves (48 KB of staging) per workgroup
  const int grid = int(std::min<int64_t>((n + kDecWaves * kWave - 1) / (kDecWaves * kWave), 4096));
  TWTML_LAUNCH(k_cesu_decode, dim3(grid), dim3(kDecWaves * kWave), 0, s, text, offsets, flags, n, tail,
                     rstart, rend, stats, special);
}

// nnz[k] carries the row's bigram count in bits 0..29 and the wide (UTF-16
// wire) flag in bit 30.  Sort key: narrow rows first, then wide rows, each
// by descending length, so a chunk mixes narrow and wide rows at most once
// (the narrow fast featurizer takes whole chunks).
constexpr int32_t kNnzWide = 1 << 30;
constexpr int32_t kNnzMask = kNnzWide - 1;
constexpr int kHalfBuckets = kLenBuckets / 2;

__device__ __forceinline__ int len_key(int32_t v) {
  const int32_t n32 = v & kNnzMask;
  const int k = kHalfBuckets - 1 - (n32 < kHalfBuckets - 1 ? n32 : kHalfBuckets - 1);
  return (v & kNnzWide) ? kHalfBuckets + k : k;
}

// ---------------------------------------------------------------------------
// K3 filter: isRetweet && begin <= retweetCount <= end, order-preserving.
// The per-row bigram count is bucketed into an LDS histogram (descending key)
// so the global histogram sees one atomic per (block, bucket).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool keep_row(const DevRawBatch& b, int64_t r, const FeaturizeParams& fp) {
  if (r >= b.n) return false;
  if (fp.require_retweet && !(b.flags[r] & kRowRetweet)) return false;
  if (fp.range_filter) {
    const int64_t rc = raw_scalar(b, 0, r);
    if (rc < fp.begin || rc > fp.end) return false;
  }
  return true;
}

// Rows are processed in segments of kSegRows (1024 threads x 4 consecutive
// rows): ~250 workgroups per 1M-row batch, so the global histogram / cursor
// atomics are ~250 per bucket instead of ~4000 (same-address atomics
// serialise at the memory-side atomic units).
constexpr int kSegThreads = 1024;
constexpr int kSegPer = 4;
constexpr int kSegRows = kSegThreads * kSegPer;

__global__ __launch_bounds__(kSegThreads) void k_filter_count(DevRawBatch b, FeaturizeParams fp,
                                                              int64_t* blk) {
  const int64_t r0 = int64_t(blockIdx.x) * kSegRows + int64_t(threadIdx.x) * kSegPer;
  __shared__ int wtot[kSegThreads / kWave];
  int c = 0;
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) c += keep_row(b, r0 + k, fp) ? 1 : 0;
  const int t = wave_sum(c);
  if (lane_id() == 0) wtot[threadIdx.x / kWave] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t tot = 0;
    for (int k = 0; k < kSegThreads / kWave; ++k) tot += wtot[k];
    blk[blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(kSegThreads) void k_filter_write(DevRawBatch b, FeaturizeParams fp,
                                                              const int64_t* blk_off, int64_t* kept,
                                                              int32_t* nnz, int64_t* hist) {
  __shared__ int wtot[kSegThreads / kWave];
  __shared__ int lhist[kLenBuckets];
  for (int i = threadIdx.x; i < kLenBuckets; i += kSegThreads) lhist[i] = 0;
  const int64_t r0 = int64_t(blockIdx.x) * kSegRows + int64_t(threadIdx.x) * kSegPer;
  bool pred[kSegPer];
  int c = 0;
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) {
    pred[k] = keep_row(b, r0 + k, fp);
    c += pred[k] ? 1 : 0;
  }
  // exclusive prefix of c over the block (rows stay in source order)
  const int lane = lane_id(), w = threadIdx.x / kWave;
  int x = c;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int y = __shfl_up(x, off, kWave);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) wtot[w] = x;
  __syncthreads();
  int woff = 0;
  for (int k = 0; k < w; ++k) woff += wtot[k];
  int64_t pos = blk_off[blockIdx.x] + woff + x - c;
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) {
    if (!pred[k]) continue;
    const int64_t r = r0 + k;
    kept[pos] = r;
    const RowText rt = row_text(b, r);
    const int64_t nz = rt.len >= 2 ? rt.len - 1 : rt.len;
    const int32_t n32 = int32_t(nz > kNnzMask ? kNnzMask : nz) | (rt.wide ? kNnzWide : 0);
    nnz[pos] = n32;
    atomicAdd(&lhist[len_key(n32)], 1);
    ++pos;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLenBuckets; i += kSegThreads)
    if (lhist[i]) atomicAdd(reinterpret_cast<unsigned long long*>(&hist[i]), (unsigned long long)lhist[i]);
}

// Counting-sort scatter: one global atomic per (segment, bucket) reserves a
// range; rows take positions inside it through LDS counters.
__global__ __launch_bounds__(kSegThreads) void k_sort_scatter(const int32_t* nnz, const int64_t* counters,
                                                              int64_t* cursor, int32_t* sorted,
                                                              int64_t cap) {
  __shared__ int lcnt[kLenBuckets];
  __shared__ long long lbase[kLenBuckets];
  const int64_t n_kept = counters[0] < cap ? counters[0] : cap;
  for (int64_t base = int64_t(blockIdx.x) * kSegRows; base < n_kept; base += int64_t(gridDim.x) * kSegRows) {
    for (int i = threadIdx.x; i < kLenBuckets; i += kSegThreads) lcnt[i] = 0;
    __syncthreads();
    int key[kSegPer], rank[kSegPer];
#pragma unroll
    for (int k = 0; k < kSegPer; ++k) {
      const int64_t q = base + int64_t(threadIdx.x) * kSegPer + k;
      key[k] = q < n_kept ? len_key(nnz[q]) : -1;
    }
#pragma unroll
    for (int k = 0; k < kSegPer; ++k) rank[k] = key[k] >= 0 ? atomicAdd(&lcnt[key[k]], 1) : 0;
    __syncthreads();
    for (int i = threadIdx.x; i < kLenBuckets; i += kSegThreads)
      if (lcnt[i])
        lbase[i] = (long long)atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[i]),
                                        (unsigned long long)lcnt[i]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSegPer; ++k)
      if (key[k] >= 0) sorted[lbase[key[k]] + rank[k]] = int32_t(base + int64_t(threadIdx.x) * kSegPer + k);
    __syncthreads();
  }
}

// Per-batch zeroing of the small prep buffers in one launch (instead of a
// hipMemsetAsync per buffer): counters, length histogram, DP kept counts,
// hybrid slot histogram, the batch's fixed-point scale bounds (max-reduced
// by k_batch_bounds later in the same prep).
__global__ __launch_bounds__(1024) void k_prep_init(DevPrepared p, int64_t* n_global, int ng, double* bounds,
                                                    int nb) {
  const int64_t i = int64_t(blockIdx.x) * 1024 + threadIdx.x;
  if (i < 8) p.counters[i] = 0;
  if (i < kLenBuckets + 1) p.hist[i] = 0;
  if (i < ng) n_global[i] = 0;
  if (i < kMaxHybridSlots) p.slot_hist[i] = 0u;
  if (bounds && i < nb) bounds[i] = 0.0;
}

void launch_prep_init(const DevPrepared& p, int64_t* n_global, int ng, hipStream_t s, double* bounds, int nb) {
  const int64_t n = std::max<int64_t>(kLenBuckets + 1, kMaxHybridSlots);
  TWTML_LAUNCH(k_prep_init, dim3(ceil_div(n, 1024)), dim3(1024), 0, s, p, n_global, ng, bounds, nb);
}

void launch_filter_sort(const DevRawBatch& b, const DevPrepared& p, const FeaturizeParams& fp,
                        hipStream_t s) {
  const int nb = ceil_div(b.n > 0 ? b.n : 1, kSegRows);
  TWTML_LAUNCH(k_filter_count, dim3(nb), dim3(kSegThreads), 0, s, b, fp, p.blk);
  scan_excl(p.blk, p.blk, nb, &p.counters[0], s);
  TWTML_LAUNCH(k_filter_write, dim3(nb), dim3(kSegThreads), 0, s, b, fp, p.blk, p.kept, p.nnz,
                     p.hist);
  scan_excl(p.hist, p.hist, kLenBuckets, nullptr, s);
  TWTML_LAUNCH(k_sort_scatter, dim3(nb), dim3(kSegThreads), 0, s, p.nnz, p.counters, p.hist,
                     p.sorted, p.cap_rows);
}

// Filter + order-preserving compaction only (k-means: no length sort needed).
void launch_filter_only(const DevRawBatch& b, const DevPrepared& p, const FeaturizeParams& fp,
                        hipStream_t s) {
  const int nb = ceil_div(b.n > 0 ? b.n : 1, kSegRows);
  TWTML_HIP_CHECK(hipMemsetAsync(p.hist, 0, sizeof(int64_t) * (kLenBuckets + 1), s));
  TWTML_LAUNCH(k_filter_count, dim3(nb), dim3(kSegThreads), 0, s, b, fp, p.blk);
  scan_excl(p.blk, p.blk, nb, &p.counters[0], s);
  TWTML_LAUNCH(k_filter_write, dim3(nb), dim3(kSegThreads), 0, s, b, fp, p.blk, p.kept, p.nnz,
                     p.hist);
}

// ---------------------------------------------------------------------------
// Chunk layout: groups of 8 local entries per lane for every 16-row chunk.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_chunk_len(const int32_t* sorted, const int32_t* nnz,
                                                      const int64_t* counters, int64_t cmax,
                                                      int64_t* clen_scratch, int32_t* clen8,
                                                      uint8_t* cfast) {
  const int64_t n_kept = counters[0];
  const int lane = lane_id();
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * kBlock / kWave;
  // one wave = 4 chunks of 16 rows (lane -> row 16*(4*wave + lane/16) + lane%16)
  for (int64_t c4 = wave; c4 * 4 < cmax; c4 += nwaves) {
    const int64_t c = c4 * 4 + lane / kRowsPerChunk;
    const int64_t p = c * kRowsPerChunk + (lane % kRowsPerChunk);
    const int32_t raw = (c < cmax && p < n_kept) ? nnz[sorted[p]] : 0;
    int32_t v = raw & kNnzMask, wide = raw & kNnzWide;
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {  // max / any within each 16-lane segment
      const int32_t o = __shfl_xor(v, off, kWave);
      v = o > v ? o : v;
      wide |= __shfl_xor(wide, off, kWave);
    }
    if ((lane % kRowsPerChunk) == 0 && c < cmax) {
      const int32_t per_lane = (v + kLanesPerRow - 1) / kLanesPerRow;
      const int32_t g = (per_lane + kGroup - 1) / kGroup;
      clen8[c] = g;
      clen_scratch[c] = g;
      cfast[c] = (!wide && per_lane <= kFastMaxQ) ? 1 : 0;
    }
  }
}

void launch_chunk_layout(const DevRawBatch& b, const DevPrepared& p, hipStream_t s) {
  const int64_t cmax = (b.n + kRowsPerChunk - 1) / kRowsPerChunk;
  if (cmax == 0) {
    TWTML_HIP_CHECK(hipMemsetAsync(p.cbase, 0, sizeof(int64_t), s));
    TWTML_HIP_CHECK(hipMemsetAsync(&p.counters[2], 0, sizeof(int64_t), s));
    return;
  }
  int grid = ceil_div((cmax + 3) / 4, kBlock / kWave);
  if (grid > 4096) grid = 4096;
  TWTML_LAUNCH(k_chunk_len, dim3(grid), dim3(kBlock), 0, s, p.sorted, p.nnz, p.counters,
                     cmax, p.cbase, p.clen8, p.cfast);
  scan_excl_big(p.cbase, p.cbase, cmax, &p.counters[2], p.scan_tmp, s);
}

// ---------------------------------------------------------------------------
// K1 + K2: lower-case, bigram hash, numeric features, active-set flags.
// ---------------------------------------------------------------------------

// Active-feature flags: ids below kFlagLds are first collected in a per-block
// LDS bitmap (Java bigram hashes of ASCII text are < 4096, so almost every
// entry lands here) and flushed once per block; the rest go straight to the
// byte flags in global memory.
constexpr int kFlagLds = 1 << 16;
constexpr int kFlagWords = kFlagLds / 32;

constexpr int kFeatWaves = kBlock / kWave;

// K2 (label + 4 numeric features, MllibHelper.scala:58-71) and the kept
// index of sorted position pos.
__device__ __forceinline__ void row_scalars(const DevRawBatch& b, const DevPrepared& p,
                                            const FeaturizeParams& fp, int64_t pos, bool valid,
                                            int64_t row, int32_t kidx) {
  const int64_t cap = p.cap_rows16;
  if (valid) {
    p.y[pos] = float(raw_scalar(b, 0, row));
    const double fol = double(raw_scalar(b, 1, row)), fav = double(raw_scalar(b, 2, row));
    const double fri = double(raw_scalar(b, 3, row));
    const double age = double(fp.now_ms - raw_scalar(b, 4, row));
    p.num[0 * cap + pos] = float(fol * 1e-12);
    p.num[1 * cap + pos] = float(fav * 1e-12);
    p.num[2 * cap + pos] = float(fri * 1e-12);
    p.num[3 * cap + pos] = float(age * 1e-14);
  } else {
    p.y[pos] = 0.f;
    for (int k = 0; k < 4; ++k) p.num[k * cap + pos] = 0.f;
  }
  p.perm[pos] = kidx;
}

// Flag an active feature id (LDS bitmap below lds_lim, byte flags above).
// fcache (murmur3 over a wide F only): a direct-mapped LDS cache of ids this
// workgroup already flagged, so the ~150 entries per tweet do not each store
// a byte into a 100 MB flag array -- a tweet batch touches a few thousand
// distinct ids, almost every lookup hits.
constexpr int kFlagCache = 4096;

// k_featurize (wide rows, murmur3 over F > 2^24): the cache takes the LDS
// of the id bitmap (ids < 2^16 are 0.07 % of a uniform hash over 1e8), so
// the workgroups stay at three per CU
constexpr int kFlagCacheWide = 2048;

__device__ __forceinline__ void flag_id(uint32_t* fbits, const DevPrepared& p, int64_t idx,
                                        int64_t lds_lim, uint32_t* fcache = nullptr,
                                        uint32_t cmask = kFlagCache - 1) {
  if (idx < lds_lim) {
    // hot ids are flagged early: a (broadcast) read skips the atomic
    const uint32_t bit = 1u << (idx & 31);
    if (!(fbits[idx >> 5] & bit)) atomicOr(&fbits[idx >> 5], bit);
  } else if (idx < p.flag_len) {
    if (fcache) {
      uint32_t& e = fcache[uint32_t(idx) & cmask];
      if (e != uint32_t(idx)) {
        p.flags[idx] = 1;
        e = uint32_t(idx);   // racing lanes may both store: harmless
      }
    } else {
      p.flags[idx] = 1;
    }
  }
}

__device__ __forceinline__ void flush_flag_bits(const uint32_t* fbits, const DevPrepared& p) {
  for (int i = threadIdx.x; i < kFlagWords; i += kBlock) {
    uint32_t bits = fbits[i];
    while (bits) {
      const int bit = __builtin_ctz(bits);
      bits &= bits - 1u;
      p.flags[int64_t(i) * 32 + bit] = 1;
    }
  }
}

// One wave per 16-row chunk.  Per chunk the wave first resolves the 16 rows'
// metadata (lanes 0..15), then stages the rows' bytes into LDS with up to 48
// independent aligned dword loads in flight -- one memory latency per chunk
// instead of one per bigram (byte loads from global memory may alias the
// output stores, which serialised the old per-entry loop).  The 4 lanes of a
// row then take entries j = t, t+4, ... from LDS and write 8 entries per
// lane with two 16-byte stores.  Rows too long to stage read global memory.
template <bool CACHE>
__global__ __launch_bounds__(kBlock) void k_featurize(DevRawBatch b, DevPrepared p, FeaturizeParams fp,
                                                      const uint8_t* lpage, const uint16_t* lblocks,
                                                      int64_t cmax) {
  __shared__ uint32_t fbits[CACHE ? 1 : kFlagWords];
  __shared__ uint32_t fcache_s[CACHE ? kFlagCacheWide : 1];
  uint32_t* fcache = CACHE ? fcache_s : nullptr;
  if (CACHE)
    for (int i = threadIdx.x; i < kFlagCacheWide; i += kBlock) fcache_s[i] = 0xFFFFFFFFu;
  else
    for (int i = threadIdx.x; i < kFlagWords; i += kBlock) fbits[i] = 0u;
  __shared__ uint32_t stage[kFeatWaves][kRowsPerChunk * kStageStride];
  __shared__ __attribute__((aligned(16))) uint8_t lpage_s[256];
  __shared__ __attribute__((aligned(16))) uint16_t lblk_s[kLowerLdsBlocks * 256];
  stage_lower_tables(lpage_s, lblk_s, lpage, lblocks, threadIdx.x, kBlock);
  __syncthreads();
  const LowerLds lt{lpage_s, lblk_s, lblocks};
  const int64_t n_kept = p.counters[0];
  const int lane = lane_id();
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  uint32_t* st = stage[threadIdx.x / kWave];
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * kBlock / kWave;
  const int64_t F = fp.num_text_features;
  const bool f32 = F <= 0xffffffffLL;
  const FastMod32 fm(f32 ? uint32_t(F) : 1u);
  const int64_t lds_lim = CACHE ? 0 : (p.flag_len < kFlagLds ? p.flag_len : kFlagLds);
  const int64_t cap_groups = p.cap_entries / kChunkStride;
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  for (int64_t c = fp.c_lo + wave; c < nch && c < cmax && c < fp.c_hi; c += nwaves) {
    if (p.cfast[c]) continue;            // k_featurize_narrow's chunk
    const int32_t L8 = p.clen8[c];
    const int64_t g0 = p.cbase[c];
    if (g0 + L8 > cap_groups) {
      if (lane == 0) p.counters[3] = 1;  // capacity overflow -> host raises
      continue;
    }
    // 1. row metadata (lane l resolves row l & 15), 2. stage the 16 rows
    const int64_t mpos = c * kRowsPerChunk + (lane & 15);
    const bool mvalid = mpos < n_kept;
    const int32_t mkidx = mvalid ? p.sorted[mpos] : -1;
    const StageMeta meta = stage_meta(b, mvalid, mvalid ? p.kept[mkidx] : 0);
    stage_rows(b, meta, st, lane);
    // 3. bigrams of row r, entries j = t, t+4, ...
    const int64_t pos = c * kRowsPerChunk + r;
    const bool valid = pos < n_kept;
    const int32_t kidx = __shfl(mkidx, r, kWave);
    const int64_t row = __shfl(meta.row, r, kWave);
    const StagedRow sr = staged_row(meta, st, r);
    const int64_t len = valid ? sr.rt.len : 0;
    const int64_t nz = len >= 2 ? len - 1 : len;
    auto unit = [&](int64_t j) -> uint32_t { return sr.unit(b, j, lt); };
    int32_t* out = p.idx + g0 * kChunkStride + lane * kGroup;
    const int32_t total = L8 * kGroup;
    // Each unit is read and lower-cased once: entry j's second unit j + 1 is
    // the first unit of lane t + 1 (same step) or, for t = 3, of lane t - 3
    // (next step) -- a quad DPP rotate within the row's 4 lanes.  (Each
    // entry lower-casing both of its units read 2 x 4 LDS bytes / table
    // entries per bigram of a wide row.)
    auto ua_at = [&](int32_t jj) -> uint32_t {
      const int64_t j = int64_t(jj) * kLanesPerRow + t;
      return j < len ? unit(j) : 0u;
    };
    auto quad_next = [](uint32_t x) -> uint32_t {   // lane 4r + t <- lane 4r + (t + 1) % 4
      return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x39, 0xf, 0xf, true));
    };
    uint32_t ua0 = ua_at(0);
    for (int32_t jj0 = 0; jj0 < total; jj0 += kGroup) {
      uint32_t ua[kGroup + 1];
      ua[0] = ua0;
#pragma unroll
      for (int k = 1; k <= kGroup; ++k) ua[k] = ua_at(jj0 + k);
      ua0 = ua[kGroup];
      int32_t v[kGroup];
#pragma unroll
      for (int k = 0; k < kGroup; ++k) {
        const int64_t j = int64_t(jj0 + k) * kLanesPerRow + t;
        const uint32_t nA = quad_next(ua[k]), nB = quad_next(ua[k + 1]);
        v[k] = -1;
        if (j < nz) {
          const uint32_t u0 = ua[k];
          int64_t h;
          if (len >= 2) {
            const uint32_t u1 = t < kLanesPerRow - 1 ? nA : nB;
            h = fp.hash_kind == 0 ? int64_t(31u * u0 + u1) : int64_t(murmur_term(u0, u1, 2));
          } else {
            h = fp.hash_kind == 0 ? int64_t(u0) : int64_t(murmur_term(u0, 0, 1));
          }
          const int64_t idx = term_mod(h, F, fm, f32);
          v[k] = int32_t(idx);
          flag_id(fbits, p, idx, lds_lim, fcache, kFlagCacheWide - 1);
        }
      }
      int4* dst = reinterpret_cast<int4*>(out + (jj0 >> 3) * kChunkStride);
      dst[0] = make_int4(v[0], v[1], v[2], v[3]);
      dst[1] = make_int4(v[4], v[5], v[6], v[7]);
    }
    __builtin_amdgcn_wave_barrier();   // LDS reads of this chunk precede the next staging
    if (t == 0) row_scalars(b, p, fp, pos, valid, row, kidx);
  }
  if (!CACHE) {
    __syncthreads();
    flush_flag_bits(fbits, p);
  }
}

// ---------------------------------------------------------------------------
// Narrow fast path (chunks whose 16 rows are all Latin-1 on the wire and
// hold <= kFastMaxQ bigrams per lane): each of a row's 4 lanes takes a
// CONTIGUOUS quarter of the row's bigrams (the SGD kernels only need every
// entry of a row in one of its 4 lanes), so a lane's text is one byte range:
// at most 5 dwordx4 loads, realigned with v_alignbyte, lower-cased four
// bytes per SWAR step and hashed straight from VGPRs.  No LDS staging (LDS
// holds only the flag bitmap), so occupancy is register-bound, and every
// chunk costs two memory round trips (row metadata, then text).
// ---------------------------------------------------------------------------
// idx_mode (FeaturizeParams): 0 writes every entry's hashed id; 1 (lazy)
// writes ids only for the chunks the hot-slot histogram samples -- the hybrid
// remap re-derives the rest from the text (narrow_text.h); 2 writes every id
// but no flags / numeric features (fallback when the batch cannot use the
// hybrid layout after a lazy pass).
template <bool CACHE>
__global__ __launch_bounds__(kBlock) void k_featurize_narrow(DevRawBatch b, DevPrepared p,
                                                             FeaturizeParams fp, int64_t cmax) {
  __shared__ uint32_t fbits[kFlagWords];
  __shared__ uint32_t fcache_s[CACHE ? kFlagCache : 1];
  uint32_t* fcache = CACHE ? fcache_s : nullptr;
  const bool flags = fp.idx_mode != 2;
  if (flags) {
    for (int i = threadIdx.x; i < kFlagWords; i += kBlock) fbits[i] = 0u;
    if (CACHE)
      for (int i = threadIdx.x; i < kFlagCache; i += kBlock) fcache_s[i] = 0xFFFFFFFFu;
    __syncthreads();
  }
  const int64_t n_kept = p.counters[0];
  const int lane = lane_id();
  const int t = lane % kLanesPerRow;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * kBlock / kWave;
  const NarrowHash nh(fp);
  const int64_t lds_lim = p.flag_len < kFlagLds ? p.flag_len : kFlagLds;
  const int64_t cap_groups = p.cap_entries / kChunkStride;
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  for (int64_t c = fp.c_lo + wave; c < nch && c < cmax && c < fp.c_hi; c += nwaves) {
    if (!p.cfast[c]) continue;
    const int32_t L8 = p.clen8[c];
    const int64_t g0 = p.cbase[c];
    if (g0 + L8 > cap_groups) {
      if (lane == 0) p.counters[3] = 1;  // capacity overflow -> host raises
      continue;
    }
    const bool store = fp.idx_mode != 1 || (c % kHistChunks) == 0;   // wave-uniform
    NarrowLane L;
    uint32_t a[kFastAl];
    int64_t rt;
    narrow_lane_load(b, p, c, n_kept, L, a, &rt);
    if (fp.idx_mode == 1 && lane < kRowsPerChunk) p.rtext[c * kRowsPerChunk + lane] = rt;
    int32_t* out = p.idx + g0 * kChunkStride + lane * kGroup;
#pragma unroll
    for (int g = 0; g < kFastMaxQ / kGroup; ++g) {
      if (g >= L8) break;                               // wave-uniform
      int32_t v[kGroup];
#pragma unroll
      for (int k = 0; k < kGroup; ++k) {
        const int e = g * kGroup + k;
        const int64_t idx = narrow_id(L, a, e, nh);
        v[k] = e < L.my ? int32_t(idx) : -1;
        if (flags && e < L.my) flag_id(fbits, p, idx, lds_lim, fcache);
      }
      if (store) {
        int4* dst = reinterpret_cast<int4*>(out + g * kChunkStride);
        dst[0] = make_int4(v[0], v[1], v[2], v[3]);
        dst[1] = make_int4(v[4], v[5], v[6], v[7]);
      }
    }
    if (flags && t == 0) row_scalars(b, p, fp, L.pos, L.valid, L.row, L.kidx);
  }
  if (flags) {
    __syncthreads();
    flush_flag_bits(fbits, p);
  }
}

void launch_featurize(const DevRawBatch& b, const DevPrepared& p, const FeaturizeParams& fp,
                      const uint8_t* lpage, const uint16_t* lblocks, hipStream_t s) {
  const int64_t cmax = (b.n + kRowsPerChunk - 1) / kRowsPerChunk;
  if (cmax == 0) return;
  // ~8 blocks per CU, each sweeping many chunks, so the LDS flag bitmap is
  // flushed rarely (XCD-agnostic: chunk order is length-sorted anyway)
  const int ns = prep_slices();
  for (int k = 0; k < ns; ++k) {   // chunk slices (prep_slices)
    FeaturizeParams f = fp;
    f.c_lo = cmax * k / ns;
    f.c_hi = cmax * (k + 1) / ns;
    if (f.c_hi <= f.c_lo) continue;
    int grid = ceil_div(f.c_hi - f.c_lo, kBlock / kWave);
    if (grid > 2048 * prep_grid_mult()) grid = 2048 * prep_grid_mult();
    // ids of a Java-hashed Latin-1 bigram are < 8161, always in the LDS bitmap;
    // murmur3 ids above it get the flag cache
    if (f.hash_kind == 1 && p.flag_len > kFlagLds)
      TWTML_LAUNCH(k_featurize_narrow<true>, dim3(grid), dim3(kBlock), 0, s, b, p, f, cmax);
    else
      TWTML_LAUNCH(k_featurize_narrow<false>, dim3(grid), dim3(kBlock), 0, s, b, p, f, cmax);
    // wide-row ids of murmur3 over F > 2^24 land in a flag array far beyond
    // L2 / MALL: the LDS cache drops the repeats' byte stores
    static const int wcache = [] {   // TWTML_FEAT_WCACHE=0/1 forces (A/B)
      const char* e = std::getenv("TWTML_FEAT_WCACHE");
      return e ? std::atoi(e) : -1;
    }();
    if (wcache == 1 || (wcache < 0 && f.hash_kind == 1 && p.flag_len > (int64_t(1) << 24)))
      TWTML_LAUNCH(k_featurize<true>, dim3(grid), dim3(kBlock), 0, s, b, p, f, lpage, lblocks, cmax);
    else
      TWTML_LAUNCH(k_featurize<false>, dim3(grid), dim3(kBlock), 0, s, b, p, f, lpage, lblocks, cmax);
  }
}

void launch_featurize_fast_ids(const DevRawBatch& b, const DevPrepared& p, FeaturizeParams fp, hipStream_t s) {
  const int64_t cmax = (b.n + kRowsPerChunk - 1) / kRowsPerChunk;
  if (cmax == 0) return;
  fp.idx_mode = 2;
  int grid = ceil_div(cmax, kBlock / kWave);
  if (grid > 2048) grid = 2048;
  TWTML_LAUNCH(k_featurize_narrow<false>, dim3(grid), dim3(kBlock), 0, s, b, p, fp, cmax);
}

// ---------------------------------------------------------------------------
// Active-set compaction: flags[Fh] -> sorted unique ids + slot_of, clears flags
// ---------------------------------------------------------------------------
constexpr int kFlagsPerThread = 16;
constexpr int kFlagsPerBlock = kBlock * kFlagsPerThread;  // 4096

__device__ __forceinline__ int count_bytes(uint4 v) {
  int c = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) c += ((w[i] >> (8 * k)) & 0xFF) ? 1 : 0;
  return c;
}

__global__ __launch_bounds__(kBlock) void k_compact_count(const uint8_t* flags, int64_t* ublk) {
  __shared__ int64_t scratch[kBlock / kWave];
  const int64_t base = int64_t(blockIdx.x) * kFlagsPerBlock + threadIdx.x * kFlagsPerThread;
  const uint4 v = *reinterpret_cast<const uint4*>(flags + base);
  const int64_t c = block_sum<int64_t>(count_bytes(v), scratch);
  if (threadIdx.x == 0) ublk[blockIdx.x] = c;
}

__global__ __launch_bounds__(kBlock) void k_compact_write(uint8_t* flags, const int64_t* ublk_off,
                                                          int32_t* uniq, int32_t* slot_of) {
  __shared__ int wtot[kBlock / kWave];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int64_t base = int64_t(blockIdx.x) * kFlagsPerBlock + threadIdx.x * kFlagsPerThread;
  uint4* ptr = reinterpret_cast<uint4*>(flags + base);
  const uint4 v = *ptr;
  const int c = count_bytes(v);
  int x = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  int woff = 0;
  for (int k = 0; k < w; ++k) woff += wtot[k];
  int64_t pos = ublk_off[blockIdx.x] + woff + x - c;
  if (c) {
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 4; ++k)
        if ((ws[i] >> (8 * k)) & 0xFF) {
          const int64_t id = base + i * 4 + k;
          uniq[pos] = int32_t(id);
          slot_of[id] = int32_t(pos);
          ++pos;
        }
    *ptr = make_uint4(0, 0, 0, 0);
  }
}

void launch_compact_active(const DevPrepared& p, hipStream_t s) {
  const int nb = int(p.flag_len / kFlagsPerBlock);  // flag_len is padded to 4096
  TWTML_LAUNCH(k_compact_count, dim3(nb), dim3(kBlock), 0, s, p.flags, p.ublk);
  scan_excl(p.ublk, p.ublk, nb, &p.counters[1], s);
  TWTML_LAUNCH(k_compact_write, dim3(nb), dim3(kBlock), 0, s, p.flags, p.ublk, p.uniq,
                     p.slot_of);
}

// DP active-set union: flag every id of the all-gathered per-rank lists
// (-1 pads a shorter list); the next compaction numbers the union.
__global__ __launch_bounds__(kBlock) void k_flag_ids(const int32_t* ids, int64_t n, uint8_t* flags,
                                                     int64_t flag_len) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock) {
    const int32_t id = ids[i];
    if (id >= 0 && id < flag_len) flags[id] = 1;
  }
}

void launch_flag_ids(const int32_t* ids, int64_t n, const DevPrepared& p, hipStream_t s) {
  if (n <= 0) return;
  const int grid = int(std::min<int64_t>(ceil_div(n, kBlock), 4096));
  TWTML_LAUNCH(k_flag_ids, dim3(grid), dim3(kBlock), 0, s, ids, n, p.flags, p.flag_len);
}

// ---------------------------------------------------------------------------
// Remap hashed ids to compact slots: slot = 4 + slot_of[id]; pad -> per-lane pad.
// ---------------------------------------------------------------------------
template <typename SlotT>
__global__ __launch_bounds__(kBlock) void k_remap(const int32_t* idx, const int32_t* slot_of,
                                                  SlotT* slot, int64_t entries, int64_t pad_base) {
  for (int64_t e8 = int64_t(blockIdx.x) * kBlock + threadIdx.x; e8 * 8 < entries;
       e8 += int64_t(gridDim.x) * kBlock) {
    const int4* src = reinterpret_cast<const int4*>(idx + e8 * 8);
    const int4 a = src[0], bb = src[1];
    const int32_t v[8] = {a.x, a.y, a.z, a.w, bb.x, bb.y, bb.z, bb.w};
    const SlotT pad = SlotT(pad_base + ((e8) & 63));  // (e >> 3) & 63 = lane of the group
    SlotT out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = v[k] >= 0 ? SlotT(kNumNumeric + slot_of[v[k]]) : pad;
    if constexpr (sizeof(SlotT) == 2) {
      uint4 pk;
      pk.x = uint32_t(out[0]) | (uint32_t(out[1]) << 16);
      pk.y = uint32_t(out[2]) | (uint32_t(out[3]) << 16);
      pk.z = uint32_t(out[4]) | (uint32_t(out[5]) << 16);
      pk.w = uint32_t(out[6]) | (uint32_t(out[7]) << 16);
      reinterpret_cast<uint4*>(slot)[e8] = pk;
    } else {
      uint4* dst = reinterpret_cast<uint4*>(slot + e8 * 8);
      dst[0] = make_uint4(out[0], out[1], out[2], out[3]);
      dst[1] = make_uint4(out[4], out[5], out[6], out[7]);
    }
  }
}

void launch_remap(const DevPrepared& p, int64_t entries, int64_t n_unique, bool u16, hipStream_t s) {
  if (entries == 0) return;
  const int64_t n8 = entries / 8;
  int grid = ceil_div(n8, kBlock);
  if (grid > 16384) grid = 16384;
  const int64_t pad_base = kNumNumeric + n_unique;
  if (u16)
    TWTML_LAUNCH(k_remap<uint16_t>, dim3(grid), dim3(kBlock), 0, s, p.idx, p.slot_of,
                       static_cast<uint16_t*>(p.slot), entries, pad_base);
  else
    TWTML_LAUNCH(k_remap<uint32_t>, dim3(grid), dim3(kBlock), 0, s, p.idx, p.slot_of,
                       static_cast<uint32_t*>(p.slot), entries, pad_base);
}

// ---------------------------------------------------------------------------
// Per-row duplicate merging (u16 slots, small active sets).  HashingTF gives a
// term its count; the SELL rows hold one entry per bigram occurrence, and
// short texts repeat bigrams a lot ("the ... the").  One wave per chunk walks
// its 16 rows one at a time with all 64 lanes: an LDS tag array (seen[slot] =
// row tag; tags are unique per row, so it is never cleared) elects one owner
// per distinct slot, an LDS counter array counts occurrences, and owners are
// compacted in entry order (ballot prefix) with their counts.  Chunk lengths
// shrink accordingly (clen8d); every GD iteration then touches each
// (row, term) once.
// ---------------------------------------------------------------------------
constexpr int kDedupWaves = 2;

__device__ __forceinline__ int64_t sell_addr(int r, int64_t j) {
  const int64_t m = j >> 2;
  return (m >> 3) * kChunkStride + (4 * r + int(j & 3)) * kGroup + (m & 7);
}

__global__ __launch_bounds__(kDedupWaves * kWave) void k_dedup(DevPrepared p, int64_t ns, int64_t pad_base) {
  extern __shared__ uint32_t dsm[];
  const int w = threadIdx.x / kWave, lane = lane_id();
  uint32_t* seen = dsm + int64_t(w) * 2 * ns;
  uint32_t* cnt = seen + ns;
  for (int64_t s = lane; s < ns; s += kWave) seen[s] = 0u;
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t wave = (int64_t(blockIdx.x) * kDedupWaves + w);
  const int64_t nwaves = int64_t(gridDim.x) * kDedupWaves;
  uint16_t* slot = static_cast<uint16_t*>(p.slot);
  // a row has L8 * 32 entries -> L8 / 2 per lane; rows up to kMaxRegGroups
  // groups (what the iteration kernel keeps in registers) are merged
  constexpr int kMaxPer = (kMaxRegGroups + 1) / 2;
  for (int64_t c = wave; c < nch; c += nwaves) {
    const int32_t L8 = p.clen8[c];
    const int64_t base = p.cbase[c] * kChunkStride;
    uint16_t* sl = slot + base;
    uint16_t* cn = p.cnt + base;
    if (L8 > 2 * kMaxPer) {   // very long rows: keep as they are, count 1
      for (int64_t e = lane; e < int64_t(L8) * kChunkStride; e += kWave) cn[e] = sl[e] < pad_base ? 1 : 0;
      if (lane == 0) p.clen8d[c] = L8;
      continue;
    }
    const int per = (L8 * 32 + kWave - 1) / kWave;        // entries per lane for one row
    int32_t maxn = 0;
    for (int r = 0; r < kRowsPerChunk; ++r) {
      const uint32_t tag = uint32_t(c * kRowsPerChunk + r + 1);
      uint32_t s[kMaxPer];
      bool own[kMaxPer];
#pragma unroll
      for (int i = 0; i < kMaxPer; ++i) {
        const int64_t j = lane + int64_t(kWave) * i;
        s[i] = (i < per && j < int64_t(L8) * 32) ? sl[sell_addr(r, j)] : 0xFFFFu;
        own[i] = false;
        if (s[i] < pad_base) {
          own[i] = atomicExch(&seen[s[i]], tag) != tag;
          if (own[i]) cnt[s[i]] = 0u;
        }
      }
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < kMaxPer; ++i)
        if (s[i] < pad_base) atomicAdd(&cnt[s[i]], 1u);
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
      int32_t n_own = 0;
#pragma unroll
      for (int i = 0; i < kMaxPer; ++i) {
        const uint64_t m = __ballot(own[i]);
        if (own[i]) {
          const int64_t jn = n_own + __popcll(m & ((1ull << lane) - 1ull));
          const int64_t a = sell_addr(r, jn);
          const uint32_t k = cnt[s[i]];
          sl[a] = uint16_t(s[i]);
          cn[a] = uint16_t(k < 65535u ? k : 65535u);
        }
        n_own += __popcll(m);
      }
      // pads after the merged entries (per-lane pad slot, count 0)
      for (int64_t j = n_own + lane; j < int64_t(L8) * 32; j += kWave) {
        const int64_t a = sell_addr(r, j);
        sl[a] = uint16_t(pad_base + ((4 * r + (j & 3)) & 63));
        cn[a] = 0;
      }
      maxn = n_own > maxn ? n_own : maxn;
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) p.clen8d[c] = (maxn + 31) / 32;   // 32 entries per row-group (4 lanes x 8)
  }
}

bool dedup_supported(int64_t ns) { return ns <= 8192; }

void launch_dedup(const DevPrepared& p, int64_t ns, int64_t pad_base, int64_t n_kept, hipStream_t s) {
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  if (nch == 0) return;
  int grid = int((nch + kDedupWaves - 1) / kDedupWaves);
  if (grid > 4096) grid = 4096;
  const size_t lds = size_t(kDedupWaves) * 2 * size_t(ns) * sizeof(uint32_t);
  TWTML_LAUNCH(k_dedup, dim3(grid), dim3(kDedupWaves * kWave), lds, s, p, ns, pad_base);
}

// ---------------------------------------------------------------------------
void upload_lower_tables(hipStream_t s, uint8_t** d_page, uint16_t** d_blocks) {
  TWTML_HIP_CHECK(hipMalloc(d_page, 256));
  TWTML_HIP_CHECK(hipMalloc(d_blocks, sizeof(uint16_t) * 256 * uni::kLowerNumBlocks));
  TWTML_HIP_CHECK(hipMemcpyAsync(*d_page, uni::kLowerPage, 256, hipMemcpyHostToDevice, s));
  TWTML_HIP_CHECK(hipMemcpyAsync(*d_blocks, uni::kLowerBlocks,
                                 sizeof(uint16_t) * 256 * uni::kLowerNumBlocks,
                                 hipMemcpyHostToDevice, s));
  TWTML_HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace twtml
