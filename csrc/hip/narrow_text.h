// Register-resident text of the narrow fast path, shared by the featurizer
// (featurize.hip, pass 1: active-set flags, numeric features) and the hybrid
// remap (hot_split.hip, pass 2: hot counts + cold slot codes).
//
// A "fast" chunk has 16 rows that are all Latin-1 on the wire and hold at
// most kFastMaxQ bigrams per lane.  Each of a row's 4 lanes takes a
// CONTIGUOUS quarter of the row's bigrams (the SGD kernels only need every
// entry of a row in one of its 4 lanes), so a lane's text is one byte range:
// at most 5 dwordx4 loads, realigned with v_alignbyte and lower-cased four
// bytes per SWAR step, then hashed straight from VGPRs.
//
// Re-deriving the hashed ids from the text (~160 B per tweet) in pass 2 is
// cheaper than storing them between the passes (4 B per bigram, ~600 B per
// tweet written then read back): the lazy featurizer only materialises ids
// for the sampled chunks the hot-slot histogram reads (and for chunks that
// are not fast).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "kernels.h"

namespace twtml {

// Narrow fast featurizer: bigrams per lane (row quarter) it can hold in VGPRs
constexpr int kFastMaxQ = 72;
constexpr int kFastDw = 20;     // dwords loaded per lane (80 B >= 3 + kFastMaxQ + 1)
constexpr int kFastAl = 19;     // realigned dwords (76 chars >= kFastMaxQ + 1)
static_assert(kFastAl * 4 >= kFastMaxQ + 1, "realigned window too small");
// The hot-slot histogram samples chunks c with c % kHistChunks == 0; the
// lazy featurizer writes ids for exactly those fast chunks.
constexpr int kHistChunks = 16;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mur_k(uint32_t k) { return rotl32(k * 0xCC9E2D51u, 15) * 0x1B873593u; }
__device__ __forceinline__ uint32_t mur_h(uint32_t h, uint32_t k) { return rotl32(h ^ k, 13) * 5u + 0xE6546B64u; }

// Spark-2 murmur3 (hashUnsafeBytes, seed 42) of the UTF-8 bytes of a
// 1-2 unit Java string (lone surrogates become '?').
// UTF-8 encoding of one code point, little-endian packed, byte count in *m
__device__ __forceinline__ uint32_t utf8_pack(uint32_t cp, int* m) {
  if (cp < 0x80) { *m = 1; return cp; }
  if (cp < 0x800) { *m = 2; return (0xC0u | (cp >> 6)) | ((0x80u | (cp & 0x3F)) << 8); }
  if (cp < 0x10000) {
    *m = 3;
    return (0xE0u | (cp >> 12)) | ((0x80u | ((cp >> 6) & 0x3F)) << 8) | ((0x80u | (cp & 0x3F)) << 16);
  }
  *m = 4;
  return (0xF0u | (cp >> 18)) | ((0x80u | ((cp >> 12) & 0x3F)) << 8) |
         ((0x80u | ((cp >> 6) & 0x3F)) << 16) | ((0x80u | (cp & 0x3F)) << 24);
}

// The UTF-8 bytes (at most 8) live in one 64-bit register: no private array,
// so nothing spills to scratch.
__device__ inline int32_t murmur_term(uint32_t u0, uint32_t u1, int n) {
  uint64_t bytes = 0;
  int k = 0, m = 0;
  const bool hi0 = u0 >= 0xD800 && u0 <= 0xDBFF, sur0 = u0 >= 0xD800 && u0 <= 0xDFFF;
  if (n == 2 && hi0 && u1 >= 0xDC00 && u1 <= 0xDFFF) {
    bytes = utf8_pack(0x10000u + ((u0 - 0xD800u) << 10) + (u1 - 0xDC00u), &m);
    k = m;
  } else {
    bytes = utf8_pack(sur0 ? uint32_t('?') : u0, &m);
    k = m;
    if (n == 2) {
      bytes |= uint64_t(utf8_pack((u1 >= 0xD800 && u1 <= 0xDFFF) ? uint32_t('?') : u1, &m)) << (8 * k);
      k += m;
    }
  }
  uint32_t h = 42u;
  const int aligned = k & ~3;
  if (aligned >= 4) h = mur_h(h, mur_k(uint32_t(bytes)));
  if (aligned >= 8) h = mur_h(h, mur_k(uint32_t(bytes >> 32)));
  for (int i = aligned; i < k; ++i) h = mur_h(h, mur_k(uint32_t(int32_t(int8_t(uint8_t(bytes >> (8 * i)))))));
  h ^= uint32_t(k);
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return int32_t(h);
}

// nonNegativeMod(h, F).  Hashes are 32-bit (Java hashCode / murmur3), so with
// F < 2^32 the reduction is a multiply-high (FastMod32), not a division.
__device__ __forceinline__ int64_t term_mod(int64_t h, int64_t F, const FastMod32& fm, bool f32) {
  if (h >= 0 && h < F) return h;                 // java bigrams (< 2^21) with F >= 2^21
  if (f32 && h >= -0xffffffffLL && h <= 0xffffffffLL) {
    if (h >= 0) return fm.mod(uint32_t(h));
    const uint32_t r = fm.mod(uint32_t(-h));
    return r == 0 ? 0 : F - r;
  }
  const int64_t m = h % F;
  return m < 0 ? m + F : m;
}

// Character.toLowerCase on four Latin-1 bytes: A-Z and U+00C0..U+00DE except
// U+00D7 gain 0x20.  Per byte on its low 7 bits (no carries between bytes).
__device__ __forceinline__ uint32_t lower4_latin1(uint32_t x) {
  const uint32_t hb = x & 0x80808080u;
  const uint32_t x7 = x & 0x7F7F7F7Fu;
  const uint32_t ge41 = x7 + 0x3F3F3F3Fu;              // bit 7: x7 >= 0x41
  const uint32_t gt5a = x7 + 0x25252525u;              // bit 7: x7 >= 0x5B
  const uint32_t ge40 = x7 + 0x40404040u;              // bit 7: x7 >= 0x40
  const uint32_t gt5e = x7 + 0x21212121u;              // bit 7: x7 >= 0x5F
  const uint32_t x57 = (x7 ^ 0x57575757u) + 0x7F7F7F7Fu;  // bit 7: x7 != 0x57
  const uint32_t lo = ~hb & ge41 & ~gt5a;
  const uint32_t hi = hb & ge40 & ~gt5e & x57;
  return x + (((lo | hi) & 0x80808080u) >> 2);
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&a)[kFastAl], int k) {
  return (a[k >> 2] >> (8 * (k & 3))) & 0xFFu;
}

// This lane's quarter of its row in fast chunk c: row metadata (lane l
// resolves row l & 15, then shuffles), the lowered text window in a[] (a
// caller-local array: inside a struct the compiler put it in scratch), and
// its entry count `my`.  Every lane of the wave must call it (shuffles).
struct NarrowLane {
  int32_t my;      // bigrams (entries) of this lane
  int32_t len;     // row length in units
  int32_t kidx;    // kept index of the row (-1: padding row)
  int64_t row;     // raw row id
  int64_t pos;     // sorted position 16c + r
  bool valid;
};

// Fast-chunk rows are at most 4 * kFastMaxQ + 1 units: the length fits the
// low 9 bits of the packed row-text word (offset << 9 | len) that pass 1
// leaves in p.rtext for pass 2.
constexpr int kRtextShift = 9;
static_assert(4 * kFastMaxQ + 1 < (1 << kRtextShift), "row length field too small");

__device__ __forceinline__ void narrow_lane_text(const DevRawBatch& b, int64_t o, NarrowLane& L,
                                                 uint32_t (&a)[kFastAl]);

// Pass 1: row metadata through sorted -> kept -> offsets (lane l resolves
// row l & 15, then shuffles); the packed row text word is returned in *rt.
__device__ __forceinline__ void narrow_lane_load(const DevRawBatch& b, const DevPrepared& p, int64_t c,
                                                 int64_t n_kept, NarrowLane& L, uint32_t (&a)[kFastAl],
                                                 int64_t* rt = nullptr) {
  const int lane = lane_id();
  const int r = lane / kLanesPerRow;
  const int64_t mpos = c * kRowsPerChunk + (lane & 15);
  const bool mvalid = mpos < n_kept;
  const int32_t mkidx = mvalid ? p.sorted[mpos] : -1;
  const int64_t mrow = mvalid ? p.kept[mkidx] : 0;
  const int64_t mo = mvalid ? b.offsets[mrow] : 0;
  const int64_t mlen = mvalid ? b.oend[mrow] - mo : 0;
  if (rt) *rt = (mo << kRtextShift) | mlen;
  L.pos = c * kRowsPerChunk + r;
  L.valid = L.pos < n_kept;
  L.kidx = __shfl(mkidx, r, kWave);
  L.row = __shfl(mrow, r, kWave);
  const int64_t o = __shfl(mo, r, kWave);
  L.len = L.valid ? int32_t(__shfl(mlen, r, kWave)) : 0;
  narrow_lane_text(b, o, L, a);
}

// Pass 2: the row's packed text word (pass 1 wrote it; 0 for padding rows).
__device__ __forceinline__ void narrow_lane_load_rt(const DevRawBatch& b, int64_t c, int64_t n_kept,
                                                    int64_t rt, NarrowLane& L, uint32_t (&a)[kFastAl]) {
  const int r = lane_id() / kLanesPerRow;
  L.pos = c * kRowsPerChunk + r;
  L.valid = L.pos < n_kept;
  L.kidx = -1;
  L.row = 0;
  L.len = L.valid ? int32_t(rt & ((1 << kRtextShift) - 1)) : 0;
  narrow_lane_text(b, rt >> kRtextShift, L, a);
}

__device__ __forceinline__ void narrow_lane_text(const DevRawBatch& b, int64_t o, NarrowLane& L,
                                                 uint32_t (&a)[kFastAl]) {
  const int t = lane_id() % kLanesPerRow;
  const int32_t nz = L.len >= 2 ? L.len - 1 : L.len;
  const int32_t q = (nz + kLanesPerRow - 1) / kLanesPerRow;
  const int32_t e0 = t * q;
  L.my = nz - e0 < 0 ? 0 : (nz - e0 < q ? nz - e0 : q);
  // text bytes [o + e0, o + e0 + my + 1): dword-aligned window
  const int64_t start = o + e0;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(b.text + (start & ~int64_t(3)));
  const uint32_t sh = uint32_t(start & 3);
  const int32_t need = int32_t(sh) + L.my + 1;          // bytes of the window used
  uint32_t d[kFastDw];
#pragma unroll
  for (int i = 0; i < kFastDw; i += 4) {
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (L.my > 0 && 4 * i < need) __builtin_memcpy(&v, src + i, 16);
    d[i] = v.x; d[i + 1] = v.y; d[i + 2] = v.z; d[i + 3] = v.w;
  }
  // wave-uniform bound on the characters any lane uses
  int32_t mw = L.my;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int32_t x = __shfl_xor(mw, off, kWave);
    mw = x > mw ? x : mw;
  }
  mw = __builtin_amdgcn_readfirstlane(mw);
#pragma unroll
  for (int i = 0; i < kFastAl; ++i)
    a[i] = (4 * i <= mw) ? lower4_latin1(__builtin_amdgcn_alignbyte(d[i + 1], d[i], sh)) : 0u;
}

// Hashing setup shared by both passes.  `direct`: Java hash with F > 8160,
// where a Latin-1 bigram hash (< 31*255+256) needs no reduction.
struct NarrowHash {
  int64_t F;
  FastMod32 fm;
  bool f32, direct;
  int hash_kind;
  __device__ __forceinline__ explicit NarrowHash(const FeaturizeParams& fp)
      : F(fp.num_text_features), fm(fp.num_text_features <= 0xffffffffLL ? uint32_t(fp.num_text_features) : 1u),
        f32(fp.num_text_features <= 0xffffffffLL), direct(fp.hash_kind == 0 && fp.num_text_features > 8160),
        hash_kind(fp.hash_kind) {}
};

// Hashed feature id of this lane's entry e (< L.my).
__device__ __forceinline__ int64_t narrow_id(const NarrowLane& L, const uint32_t (&a)[kFastAl], int e,
                                             const NarrowHash& nh) {
  const uint32_t u0 = byte_of(a, e), u1 = byte_of(a, e + 1);
  if (nh.direct) return L.len >= 2 ? int64_t(31u * u0 + u1) : int64_t(u0);
  const int64_t h = nh.hash_kind == 0 ? (L.len >= 2 ? int64_t(31u * u0 + u1) : int64_t(u0))
                                      : int64_t(murmur_term(u0, u1, L.len >= 2 ? 2 : 1));
  return term_mod(h, nh.F, nh.fm, nh.f32);
}

}  // namespace twtml
