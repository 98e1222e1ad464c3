// Device helpers shared by the text featurizers (featurize.hip, kmeans.hip):
// Java toLowerCase per UTF-16 unit, and LDS staging of a 16-row chunk.
//
// Staging: lane l (< 16) resolves row l's byte range; the wave then issues up
// to 48 independent aligned dword loads (3 per lane per row) before writing
// them to LDS, so a chunk costs one memory latency instead of one per bigram.
// Rows are kStageStride dwords apart (odd) so the 16 rows land in distinct
// LDS banks.  Rows longer than kStageWords dwords are left unstaged.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "kernels.h"

namespace twtml {

// BMP lowering through the generated delta tables (ASCII fast path).
__device__ __forceinline__ uint32_t lower_dev(uint32_t c, const uint8_t* page, const uint16_t* blocks) {
  if (c < 128) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
  return (c + blocks[page[c >> 8] * 256 + (c & 255)]) & 0xFFFFu;
}

// The lowering tables' first kLowerLdsBlocks delta blocks (Latin, IPA,
// Greek, Cyrillic, Armenian and the identity block every uncased page --
// CJK, Arabic, Devanagari, ... -- maps to) plus the page index, copied to
// LDS by a kernel's workgroup: a non-ASCII unit then costs two LDS reads
// instead of two dependent global loads.  Blocks beyond it stay global.
constexpr int kLowerLdsBlocks = 7;
struct LowerLds {
  const uint8_t* page;      // LDS [256]
  const uint16_t* blocks;   // LDS [kLowerLdsBlocks][256]
  const uint16_t* gblocks;  // global, all blocks
  __device__ __forceinline__ uint32_t lower(uint32_t c) const {
    return lower_any(c);
  }
  // Any unit (ASCII included: page 0's block lower-cases A-Z) without a
  // branch in the common case.  The LDS read is unconditional (clamped
  // block) and only the rare block beyond LDS reads global memory: written
  // as `blk < N ? lds[..] : global[..]` the compiler merges the two into ONE
  // flat load of a selected address -- a vector-memory round trip, waited
  // on, for every unit (measured: the k-means featurizer at 630 us).
  __device__ __forceinline__ uint32_t lower_any(uint32_t c) const {
    const uint32_t blk = page[c >> 8];
    const uint32_t i = (blk < uint32_t(kLowerLdsBlocks) ? blk : 0u) * 256u + (c & 255u);
    uint32_t d = blocks[i];
    // (a relaxed atomic load: not mergeable with the LDS load above)
    if (blk >= uint32_t(kLowerLdsBlocks))
      d = __hip_atomic_load(gblocks + (blk * 256 + (c & 255)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (c + d) & 0xFFFFu;
  }
};

// Copy the tables into the workgroup's LDS arrays (caller synchronises).
__device__ __forceinline__ void stage_lower_tables(uint8_t* page_s, uint16_t* blocks_s, const uint8_t* page,
                                                   const uint16_t* blocks, int tid, int nthreads) {
  for (int i = tid; i < 256 / 4; i += nthreads)
    reinterpret_cast<uint32_t*>(page_s)[i] = reinterpret_cast<const uint32_t*>(page)[i];
  for (int i = tid; i < kLowerLdsBlocks * 256 / 2; i += nthreads)
    reinterpret_cast<uint32_t*>(blocks_s)[i] = reinterpret_cast<const uint32_t*>(blocks)[i];
}

// Latin-1 lower-casing in closed form (narrow rows): A-Z and U+00C0..U+00DE
// except U+00D7 map to +0x20; nothing else in 0..255 changes under
// Character.toLowerCase.
__device__ __forceinline__ uint32_t lower_latin1(uint32_t c) {
  return ((c - 'A' <= 'Z' - 'A') || (c - 0xC0u <= 0xDEu - 0xC0u && c != 0xD7u)) ? c + 32u : c;
}

constexpr int kStageWords = 160;                 // 640 B per staged row (>= 280 wide units)
constexpr int kStageStride = kStageWords + 1;    // odd dword stride: rows in distinct banks

// Per-lane metadata of row (lane & 15) of a chunk whose rows are rows[0..15].
struct StageMeta {
  int64_t row, o, bytes, aligned;
  int wide, ob, ndw;   // ndw = staged dwords (0 = not staged)
};

__device__ __forceinline__ StageMeta stage_meta(const DevRawBatch& b, bool valid, int64_t row) {
  StageMeta m{row, 0, 0, 0, 0, 0, 0};
  if (valid) {
    m.o = b.offsets[row];
    m.bytes = b.oend[row] - m.o;
    m.wide = (b.flags[row] & kRowWide) ? 1 : 0;
  }
  m.aligned = m.o & ~int64_t(3);
  m.ob = int(m.o - m.aligned);
  const int ndw = int((m.ob + m.bytes + 3) >> 2);
  m.ndw = (valid && ndw <= kStageWords) ? ndw : 0;
  return m;
}

// Stage the 16 rows described by lanes 0..15's StageMeta into st.
__device__ __forceinline__ void stage_rows(const DevRawBatch& b, const StageMeta& m, uint32_t* st,
                                           int lane) {
  uint32_t tmp[kRowsPerChunk][3];
#pragma unroll
  for (int q = 0; q < kRowsPerChunk; ++q) {
    const int64_t qa = __shfl(m.aligned, q, kWave);
    const int qn = __shfl(m.ndw, q, kWave);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(b.text + qa);
#pragma unroll
    for (int k = 0; k < 3; ++k) tmp[q][k] = (lane + kWave * k < qn) ? src[lane + kWave * k] : 0u;
  }
#pragma unroll
  for (int q = 0; q < kRowsPerChunk; ++q)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (lane + kWave * k < kStageWords) st[q * kStageStride + lane + kWave * k] = tmp[q][k];
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// Lower-cased UTF-16 unit j of a row: from the staged copy if staged, else global.
struct StagedRow {
  const uint8_t* sb;   // staged bytes of the row (valid if staged)
  RowText rt;          // global view
  int staged;
  __device__ __forceinline__ uint32_t unit(const DevRawBatch& b, int64_t j, const uint8_t* lpage,
                                           const uint16_t* lblocks) const {
    if (staged) {
      if (!rt.wide) return lower_latin1(sb[j]);
      return lower_dev(uint32_t(sb[2 * j]) | (uint32_t(sb[2 * j + 1]) << 8), lpage, lblocks);
    }
    return lower_dev(row_unit(b, rt, j), lpage, lblocks);
  }
  __device__ __forceinline__ uint32_t unit(const DevRawBatch& b, int64_t j, const LowerLds& lt) const {
    if (staged) {
      if (!rt.wide) return lower_latin1(sb[j]);
      return lt.lower(uint32_t(sb[2 * j]) | (uint32_t(sb[2 * j + 1]) << 8));
    }
    return lt.lower(row_unit(b, rt, j));
  }
};

// View of row r (lanes 4r..4r+3) after stage_rows.
__device__ __forceinline__ StagedRow staged_row(const StageMeta& m, const uint32_t* st, int r) {
  StagedRow s;
  const int wide = __shfl(m.wide, r, kWave);
  s.rt = RowText{__shfl(m.o, r, kWave), __shfl(m.bytes, r, kWave) >> wide, wide};
  s.staged = __shfl(m.ndw, r, kWave) > 0 ? 1 : 0;
  s.sb = reinterpret_cast<const uint8_t*>(st + r * kStageStride) + __shfl(m.ob, r, kWave);
  return s;
}

}  // namespace twtml
