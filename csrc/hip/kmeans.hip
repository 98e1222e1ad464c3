// Streaming k-means on MI355X (KMeans.scala:100-113).
//
// Per micro-batch:
//   K3'  filter isRetweet, K1' features x = [retweetCount, followers, hashed
//        bigram counts (text_dims)] as dense fp32 rows (width padded to DP)
//   K11  StandardScaler(withMean=false, withStd=true): exact integer column
//        moments (max, then sum / sum of squares) -> sample std on the host
//   K8   assignment: distances to all k centres on the MATRIX cores --
//        v_mfma_f32_32x32x2_f32 (exact fp32 products) computes C.X^T for 32
//        centres x 32 points per wave, ||c||^2 - 2 c.x is reduced to a running
//        argmin per point (first index wins ties, as KMeans.findClosest)
//   K9   per-cluster sums: counting-sort points by label, then a segmented
//        int64 sum that flushes one atomic per (label run, column): exact
//   K10  update (one workgroup): decay, weighted centroid move, dying-
//        cluster split -- StreamingKMeansModel.update [upstream]
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "kmeans_kernels.h"
#include "text_stage.h"

namespace twtml {

// ---------------------------------------------------------------------------
// K1': dense features.  One wave per kept row; bigram counts through an LDS
// integer histogram (ds_add_u32 -- LDS float atomics are ~20x slower).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t km_lower(uint32_t c, const uint8_t* page, const uint16_t* blocks) {
  if (c < 128) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
  return (c + blocks[page[c >> 8] * 256 + (c & 255)]) & 0xFFFFu;
}

constexpr int kKmFeatWaves = 4;

__global__ __launch_bounds__(kBlock) void k_km_features(DevRawBatch b, const int64_t* kept,
                                                        const int64_t* counters, float* X, int dp,
                                                        int text_dims, const uint8_t* lpage,
                                                        const uint16_t* lblocks) {
  extern __shared__ uint32_t hist[];  // [kKmFeatWaves][text_dims]
  const int lane = lane_id(), w = threadIdx.x / kWave;
  uint32_t* h = hist + w * (text_dims > 0 ? text_dims : 1);
  const int64_t n_kept = counters[0];
  for (int64_t k = int64_t(blockIdx.x) * kKmFeatWaves + w; k < n_kept;
       k += int64_t(gridDim.x) * kKmFeatWaves) {
    const int64_t row = kept[k];
    float* xr = X + k * dp;
    if (text_dims > 0) {
      for (int j = lane; j < text_dims; j += kWave) h[j] = 0u;
      __builtin_amdgcn_wave_barrier();
      const RowText rt = row_text(b, row);
      const int64_t len = rt.len;
      const int64_t nz = len >= 2 ? len - 1 : len;
      for (int64_t j = lane; j < nz; j += kWave) {
        const uint32_t u0 = km_lower(row_unit(b, rt, j), lpage, lblocks);
        const uint32_t hsh = len >= 2 ? 31u * u0 + km_lower(row_unit(b, rt, j + 1), lpage, lblocks) : u0;
        atomicAdd(&h[hsh % uint32_t(text_dims)], 1u);
      }
      __builtin_amdgcn_wave_barrier();
      for (int j = lane; j < text_dims; j += kWave) xr[2 + j] = float(h[j]);
    }
    if (lane == 0) {
      xr[0] = float(raw_scalar(b, 0, row));   // retweetCount
      xr[1] = float(raw_scalar(b, 1, row));   // followersCount
    }
    for (int j = 2 + text_dims + lane; j < dp; j += kWave) xr[j] = 0.f;
  }
}

// Chunked variant (text_dims <= kKmChunkDims): a wave takes 16 consecutive
// kept rows, stages their text in LDS (text_stage.h), 4 lanes per row build
// the row's bigram histogram in LDS, and the wave writes the 16 contiguous
// feature rows with coalesced stores.
constexpr int kKmChunkDims = 256;

__global__ __launch_bounds__(kBlock) void k_km_features_chunk(DevRawBatch b, const int64_t* kept,
                                                              const int64_t* counters, float* X,
                                                              int dp, int text_dims,
                                                              const uint8_t* lpage,
                                                              const uint16_t* lblocks) {
  extern __shared__ uint32_t smem[];
  __shared__ __attribute__((aligned(16))) uint8_t lpage_s[256];
  __shared__ __attribute__((aligned(16))) uint16_t lblk_s[kLowerLdsBlocks * 256];
  stage_lower_tables(lpage_s, lblk_s, lpage, lblocks, threadIdx.x, kBlock);
  __syncthreads();
  const LowerLds lt{lpage_s, lblk_s, lblocks};
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int tdp = text_dims > 0 ? text_dims : 1;
  uint32_t* st = smem + w * (kRowsPerChunk * kStageStride + kRowsPerChunk * tdp);
  uint32_t* hist = st + kRowsPerChunk * kStageStride;     // [16][text_dims]
  const int64_t n_kept = counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const FastMod32 fm{static_cast<uint32_t>(tdp)};
  for (int64_t c = int64_t(blockIdx.x) * kKmFeatWaves + w; c < nch;
       c += int64_t(gridDim.x) * kKmFeatWaves) {
    const int64_t mk = c * kRowsPerChunk + (lane & 15);
    const bool mvalid = mk < n_kept;
    const int64_t mrow = mvalid ? kept[mk] : 0;
    const float mx0 = mvalid ? float(raw_scalar(b, 0, mrow)) : 0.f;   // retweetCount
    const float mx1 = mvalid ? float(raw_scalar(b, 1, mrow)) : 0.f;   // followersCount
    if (text_dims > 0) {
      const StageMeta meta = stage_meta(b, mvalid, mrow);
      for (int i = lane; i < kRowsPerChunk * text_dims; i += kWave) hist[i] = 0u;
      stage_rows(b, meta, st, lane);                // includes the fence + wave barrier
      // rows one at a time with all 64 lanes (short per-lane chains)
      for (int q = 0; q < kRowsPerChunk; ++q) {
        const StagedRow sr = staged_row(meta, st, q);
        const bool valid = c * kRowsPerChunk + q < n_kept;
        const int64_t len = valid ? sr.rt.len : 0;
        const int64_t nz = len >= 2 ? len - 1 : len;
        uint32_t* h = hist + q * text_dims;
        for (int64_t j = lane; j < nz; j += kWave) {
          const uint32_t u0 = sr.unit(b, j, lt);
          const uint32_t hsh = len >= 2 ? 31u * u0 + sr.unit(b, j + 1, lt) : u0;
          atomicAdd(&h[fm.mod(hsh)], 1u);
        }
      }
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
    }
    // 16 consecutive rows x dp floats, contiguous in X
    const int64_t k0 = c * kRowsPerChunk;
    const int nrows = int(n_kept - k0 < kRowsPerChunk ? n_kept - k0 : kRowsPerChunk);
    float* xc = X + k0 * dp;
    for (int i = lane; i < nrows * dp; i += kWave) {
      const int q = i / dp, col = i - q * dp;
      if (col < 2) continue;                      // scalar columns below
      xc[i] = col < 2 + text_dims ? float(hist[q * text_dims + col - 2]) : 0.f;
    }
    // scalar columns (lanes 0..15 own row lane & 15)
    if (lane < nrows) {
      xc[int64_t(lane) * dp + 0] = mx0;
      xc[int64_t(lane) * dp + 1] = mx1;
    }
    __builtin_amdgcn_wave_barrier();   // LDS reuse by the next chunk
  }
}

// Balanced variant (0 < text_dims <= kKmChunkDims; config 4: 62 dims).  A
// wave takes 16 kept rows; their bytes are staged back to back in the wave's
// LDS window (rows that do not fit read global memory), and the chunk's T
// bigrams -- all rows together -- are split evenly over the 64 lanes: lane L
// hashes bigrams [L T / 64, (L+1) T / 64), crossing row boundaries as its
// range does, into the rows' shared LDS histograms (ds_add_u32; ~4 lanes
// per row at a time over td bins, so same-address collisions are rare).
// Round 2's kernel hashed one row at a time with all 64 lanes (64 lanes into
// 62 bins: serialised atomics); per-row lane quarters left most lanes idle
// behind the longest row of the 16.  Every unit is lower-cased through the
// LDS delta tables (page 0's block maps A-Z), without per-kind branches,
// and h mod td is one v_mul_hi_u32 (q = mulhi(h, ceil(2^32 / td)) is exact
// for h < 2^32 / td: bigram hashes are < 2^21).
// Measured (1M wide-vocabulary tweets, td = 62): round 2's kernel 787 us;
// per-row lane quarters with lane-private histograms 732-814 us; this one
// 624 us.  PMC: issue-bound (~5300 instructions per 16 rows, 2.6 waves per
// SIMD).  Rejected: one row per lane reading global memory (TA-bound, 64
// rows' byte loads per instruction: 832 us) or LDS (64 rows' staging halves
// the occupancy: 1225 us).
// LDS per wave: the staged rows, the 16 rows' histograms as u16 count pairs
// (a row has < 2^13 bytes), row metadata: 7.1 KB at td = 62, so with the
// lower-case tables a workgroup is exactly 32 KB and 5 fit a CU (round 3's
// first cut, a 6 KB stage + u32 bins, fitted 3).
constexpr int kKmStageDw = 1216;   // staged dwords per wave (4.75 KB; wide chunks: p50 3.5 KB, p99 4.8 KB)

__host__ __device__ constexpr int km_hist_words(int td) { return (td + 1) / 2; }

__host__ __device__ constexpr int km_bal_wave_dwords(int td) {
  return kKmStageDw + kRowsPerChunk * km_hist_words(td) + kRowsPerChunk * 4 + kRowsPerChunk * 2 + kRowsPerChunk;
}

__global__ __launch_bounds__(kBlock) void k_km_features_bal(DevRawBatch b, const int64_t* kept,
                                                            const int64_t* counters, float* X, int dp,
                                                            int text_dims, const uint8_t* lpage,
                                                            const uint16_t* lblocks) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_b[];
  __shared__ __attribute__((aligned(16))) uint8_t lpage_s[256];
  __shared__ __attribute__((aligned(16))) uint16_t lblk_s[kLowerLdsBlocks * 256];
  stage_lower_tables(lpage_s, lblk_s, lpage, lblocks, threadIdx.x, kBlock);
  __syncthreads();
  const LowerLds lt{lpage_s, lblk_s, lblocks};
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int td = text_dims;
  uint32_t* st = smem_b + w * km_bal_wave_dwords(td);      // staged bytes (4-B aligned rows)
  const int hw = km_hist_words(td);
  uint32_t* hist = st + kKmStageDw;                          // [16][hw]: bin b in the half b & 1 of word b >> 1
  int32_t* meta = reinterpret_cast<int32_t*>(hist + kRowsPerChunk * hw);   // [16][4]
  int64_t* mo = reinterpret_cast<int64_t*>(meta + kRowsPerChunk * 4);       // [16] row byte offsets
  int32_t* dwe = reinterpret_cast<int32_t*>(mo + kRowsPerChunk);            // [16] staged dword ends
  const uint8_t* stb = reinterpret_cast<const uint8_t*>(st);
  const int64_t n_kept = counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const uint32_t tdu = uint32_t(td);
  // (td = 1: the magic 2^32 does not fit 32 bits; every hash lands in bin 0)
  const uint32_t mg = uint32_t((uint64_t(1) << 32) / tdu + ((uint64_t(1) << 32) % tdu ? 1u : 0u));
  const bool one = tdu == 1u;
  auto lower = [&](uint32_t c) -> uint32_t { return lt.lower_any(c); };
  for (int64_t c = int64_t(blockIdx.x) * kKmFeatWaves + w; c < nch;
       c += int64_t(gridDim.x) * kKmFeatWaves) {
    // lanes 0..15: row `lane` of the chunk
    const int64_t mk = c * kRowsPerChunk + lane;
    const bool mvalid = lane < kRowsPerChunk && mk < n_kept;
    const int64_t mrow = mvalid ? kept[mk] : 0;
    const float mx0 = mvalid ? float(raw_scalar(b, 0, mrow)) : 0.f;   // retweetCount
    const float mx1 = mvalid ? float(raw_scalar(b, 1, mrow)) : 0.f;   // followersCount
    int64_t o = 0, bytes = 0;
    int wide = 0;
    if (mvalid) {
      o = b.offsets[mrow];
      bytes = b.oend[mrow] - o;
      wide = (b.flags[mrow] & kRowWide) ? 1 : 0;
    }
    const int len = int(bytes >> wide);
    const int nz = len >= 2 ? len - 1 : len;
    const int64_t al = o & ~int64_t(3);
    const int ob = int(o - al);
    const int ndw = mvalid ? int((ob + bytes + 3) >> 2) : 0;
    // inclusive scans over lanes 0..15 (ndw: LDS placement, nz: bigram ranges)
    int sdw = ndw, snz = nz;
#pragma unroll
    for (int off = 1; off < kRowsPerChunk; off <<= 1) {
      const int a = __shfl_up(sdw, off, kWave), z = __shfl_up(snz, off, kWave);
      if ((lane & 15) >= off) { sdw += a; snz += z; }
    }
    // (a wide row staged at an odd byte would split its units across dwords)
    const bool staged = mvalid && sdw <= kKmStageDw && ndw <= 3 * kWave && !(wide && (ob & 1));
    const int dw0 = sdw - ndw;
    if (lane < kRowsPerChunk) {
      meta[4 * lane + 0] = snz - nz;                         // first bigram of the row
      meta[4 * lane + 1] = nz;
      meta[4 * lane + 2] = staged ? 4 * dw0 + ob : -1;       // staged byte offset
      meta[4 * lane + 3] = wide | (len == 1 ? 2 : 0);
      mo[lane] = o;
      dwe[lane] = staged ? sdw : dw0;                        // unstaged: an empty dword range
    }
    const int T = __shfl(snz, kRowsPerChunk - 1, kWave);
    for (int i = lane; i < kRowsPerChunk * hw; i += kWave) hist[i] = 0u;
    // stage: up to 3 dwords per lane per row, 8 rows' 24 loads in flight at a
    // time (all 16 rows' took 48 VGPRs: occupancy was VGPR-bound)
    constexpr int kHalf = kRowsPerChunk / 2;
#pragma unroll 1
    for (int h0 = 0; h0 < kRowsPerChunk; h0 += kHalf) {
      uint32_t tmp[kHalf][3];
#pragma unroll
      for (int qq = 0; qq < kHalf; ++qq) {
        const int q = h0 + qq;
        const int64_t qa = __shfl(al, q, kWave);
        const int qn = __shfl(staged ? ndw : 0, q, kWave);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(b.text + qa);
#pragma unroll
        for (int k = 0; k < 3; ++k) tmp[qq][k] = (lane + kWave * k < qn) ? src[lane + kWave * k] : 0u;
      }
      // lower-cased on the way into LDS (every dword of a row is independent
      // work here: no dependent table reads left in the bigram walk below)
#pragma unroll
      for (int qq = 0; qq < kHalf; ++qq) {
        const int q = h0 + qq;
        const int qn = __shfl(staged ? ndw : 0, q, kWave);
        const int qd = __shfl(dw0, q, kWave);
        const int qw = __shfl(wide, q, kWave);
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (lane + kWave * k < qn) {
            const uint32_t v = tmp[qq][k];
            uint32_t lv;
            if (qw) {
              lv = lt.lower_any(v & 0xFFFFu) | (lt.lower_any(v >> 16) << 16);
            } else {
              lv = 0;
#pragma unroll
              for (int y = 0; y < 4; ++y) lv |= lower_latin1((v >> (8 * y)) & 0xFFu) << (8 * y);
            }
            st[qd + lane + kWave * k] = lv;
          }
      }
    }
    const bool all_staged = __all(staged || !mvalid);
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    // this lane's bigram range and the row it starts in
    const int g0 = int((int64_t(lane) * T) >> 6), g1 = int((int64_t(lane + 1) * T) >> 6);
    int q = 0;
#pragma unroll
    for (int k = 0; k < kRowsPerChunk; ++k) q += (g0 >= __builtin_amdgcn_readlane(snz, k)) ? 1 : 0;
    auto walk = [&](auto staged_tag) {
      constexpr bool STAGED = decltype(staged_tag)::value;
      int g = g0, j = 0, rnz = 0, rb = 0, rk = 0;
      int64_t ro = 0;
      auto row = [&](int qq) {
        rnz = meta[4 * qq + 1];
        rb = meta[4 * qq + 2];
        rk = meta[4 * qq + 3];
        if (!STAGED) ro = mo[qq];
      };
      auto unit = [&](int jj) -> uint32_t {   // lower-cased unit jj of the current row
        const int wd = rk & 1;
        if (STAGED || rb >= 0)
          return wd ? uint32_t(*reinterpret_cast<const uint16_t*>(stb + rb + 2 * jj)) : uint32_t(stb[rb + jj]);
        return lower(row_unit(b, RowText{ro, 0, wd}, jj));
      };
      if (g >= g1) return;
      row(q);
      j = g - meta[4 * q + 0];
      uint32_t u0 = unit(j);
      while (true) {
        const int rq = q * hw;
        const uint32_t u1 = (rk & 2) ? 0u : unit(j + 1);
        const uint32_t h = (rk & 2) ? u0 : 31u * u0 + u1;
        const uint32_t bin = one ? 0u : h - __umulhi(h, mg) * tdu;
        __hip_atomic_fetch_add(hist + rq + int(bin >> 1), 1u << ((bin & 1u) * 16), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        if (++g >= g1) break;
        if (++j < rnz) {
          u0 = u1;                               // (a 1-unit row has rnz = 1: never here)
        } else {                                 // next row with bigrams
          do { row(++q); } while (rnz == 0);
          j = 0;
          u0 = unit(0);
        }
      }
    };
    // Staged chunks: every lane takes an equal share of the chunk's staged
    // dwords and hashes the bigrams that START in each of its dwords -- 4
    // narrow or 2 wide slots per dword, the slot's two units cut out of the
    // dword pair (d, d + 1) by one v_alignbyte -- so the walk has no
    // per-bigram cursor state and each lane has 4 independent hash -> add
    // chains per dword.  (Round 3-4: four bigram cursors per lane, ~110
    // lane-ops per bigram in the PMC counts.)  Staged bytes outside a row's
    // units (alignment head, tail) fail the slot's range check.
    auto walk_dw = [&]() {
      const int dtot = __shfl(sdw, kRowsPerChunk - 1, kWave);
      const int d0 = int((int64_t(lane) * dtot) >> 6), d1 = int((int64_t(lane + 1) * dtot) >> 6);
      if (d0 >= d1) return;
      int q = 0;
#pragma unroll
      for (int k = 0; k < kRowsPerChunk; ++k) q += (d0 >= __builtin_amdgcn_readlane(sdw, k)) ? 1 : 0;
      int rend = 0, b0 = 0, lim = 0, us = 1, one1 = 0, rq = 0;
      auto row = [&]() {
        rend = dwe[q];
        b0 = meta[4 * q + 2];
        const int rk = meta[4 * q + 3];
        us = 1 + (rk & 1);
        one1 = rk & 2;
        lim = meta[4 * q + 1] * us;   // byte span of the row's bigram starts
        rq = q * hw;
      };
      row();
      for (int d = d0; d < d1; ++d) {
        while (d >= rend) { ++q; row(); }   // (empty and unstaged rows have empty ranges)
        const uint32_t v = st[d], v2 = st[d + 1];   // (d + 1 may read the histograms: masked)
        const int pb = 4 * d - b0;                   // slot 0's byte within the row's units
        const uint32_t ub = 8u * uint32_t(us);
        const uint32_t umask = us == 1 ? 0xFFu : 0xFFFFu;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int sh = y * us;
          if (sh < 4 && unsigned(pb + sh) < unsigned(lim)) {
            const uint32_t wv = __builtin_amdgcn_alignbyte(v2, v, uint32_t(sh));
            const uint32_t u0 = wv & umask;
            const uint32_t h = one1 ? u0 : 31u * u0 + __builtin_amdgcn_ubfe(wv, ub, ub);
            const uint32_t bin = one ? 0u : h - __umulhi(h, mg) * tdu;
            __hip_atomic_fetch_add(hist + rq + int(bin >> 1), 1u << ((bin & 1u) * 16), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    };
    if (all_staged) walk_dw();
    else walk(std::false_type{});
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    // 16 consecutive rows x dp floats, contiguous in X
    const int64_t k0 = c * kRowsPerChunk;
    const int nrows = int(n_kept - k0 < kRowsPerChunk ? n_kept - k0 : kRowsPerChunk);
    float* xc = X + k0 * dp;
    int r = 0, col = lane;                        // i = r * dp + col, advanced without divisions
    while (col >= dp) { col -= dp; ++r; }
    for (int i = lane; i < nrows * dp; i += kWave) {
      if (col >= 2) {   // scalars below
        const int b = col - 2;
        xc[i] = b < td ? float((hist[r * hw + (b >> 1)] >> ((b & 1) * 16)) & 0xFFFFu) : 0.f;
      }
      col += kWave;
      while (col >= dp) { col -= dp; ++r; }
    }
    if (lane < nrows) {
      xc[int64_t(lane) * dp + 0] = mx0;
      xc[int64_t(lane) * dp + 1] = mx1;
    }
    __builtin_amdgcn_wave_barrier();   // LDS reuse by the next chunk
  }
}

void launch_km_features(const DevRawBatch& b, const int64_t* kept, const int64_t* counters,
                        float* X, int dp, int text_dims, const uint8_t* lpage,
                        const uint16_t* lblocks, int64_t max_rows, hipStream_t s) {
  if (text_dims > 0 && text_dims <= kKmChunkDims) {
    const int64_t nch = (max_rows + kRowsPerChunk - 1) / kRowsPerChunk;
    int grid = int((nch + kKmFeatWaves - 1) / kKmFeatWaves);
    if (grid < 1) grid = 1;
    if (grid > 4096) grid = 4096;
    const size_t lds = size_t(kKmFeatWaves) * size_t(km_bal_wave_dwords(text_dims)) * sizeof(uint32_t);
    TWTML_LAUNCH(k_km_features_bal, dim3(grid), dim3(kBlock), lds, s, b, kept, counters, X, dp,
                       text_dims, lpage, lblocks);
    return;
  }
  if (text_dims <= kKmChunkDims) {
    const int64_t nch = (max_rows + kRowsPerChunk - 1) / kRowsPerChunk;
    int grid = int((nch + kKmFeatWaves - 1) / kKmFeatWaves);
    if (grid < 1) grid = 1;
    if (grid > 2048) grid = 2048;
    const size_t lds = size_t(kKmFeatWaves) *
                       (size_t(kRowsPerChunk) * kStageStride + size_t(kRowsPerChunk) *
                        size_t(text_dims > 0 ? text_dims : 1)) * sizeof(uint32_t);
    TWTML_LAUNCH(k_km_features_chunk, dim3(grid), dim3(kBlock), lds, s, b, kept, counters, X,
                       dp, text_dims, lpage, lblocks);
    return;
  }
  int grid = ceil_div(max_rows > 0 ? max_rows : 1, kKmFeatWaves);
  if (grid > 8192) grid = 8192;
  const size_t lds = size_t(kKmFeatWaves) * size_t(text_dims > 0 ? text_dims : 1) * sizeof(uint32_t);
  TWTML_LAUNCH(k_km_features, dim3(grid), dim3(kBlock), lds, s, b, kept, counters, X, dp,
                     text_dims, lpage, lblocks);
}

// ---------------------------------------------------------------------------
// K11: StandardScaler moments, exact in integers.
//
// Every feature is an integer-valued float (retweet / follower counts and
// bigram counts), so the column sums are exact int64 sums -- equal in any
// summation order, on any number of DP ranks, bit for bit (the
// fp64 moment / cluster sums made DP k-means order dependent).  A column
// whose magnitudes exceed 2^30 is first scaled by 2^-s (s from the
// all-reduced column max, identical on every rank) and rounded: then
// |q| <= 2^30 and
//   sum q, and q^2 as three limbs a^2 2^32 + 2ab 2^16 + b^2 (q = a 2^16 + b)
// stay below 2^63 for any batch (< 2^31 rows).  The host combines the limbs
// in 128-bit integers: var = 2^2s (n sum q^2 - (sum q)^2) / (n (n - 1)).
// ---------------------------------------------------------------------------
static int km_cols_pow2(int d) {
  int cp = 1;
  while (cp < d && cp < kBlock) cp <<= 1;
  return cp;
}

__device__ __forceinline__ int km_shift(int64_t mx) {
  const int L = mx > 0 ? 64 - __clzll(static_cast<unsigned long long>(mx)) : 0;
  return L > kKmQBits ? L - kKmQBits : 0;
}

// q = rint(x 2^-s): exact for s == 0 (x is integer valued), deterministic else
__device__ __forceinline__ int64_t km_q(float x, int s) {
  return static_cast<int64_t>(rint(ldexp(static_cast<double>(x), -s)));
}

// thread -> (row lane rr, column j): consecutive threads read consecutive
// columns of a row (coalesced); row lanes are reduced in LDS, one 64-bit
// atomic per (block, column).
__global__ __launch_bounds__(kBlock) void k_km_colmax(const float* X, const int64_t* counters, int d, int dp,
                                                      int cp, int64_t* mx) {
  __shared__ unsigned long long red[kBlock];
  const int64_t n = counters[0];
  const int rp = kBlock / cp, rr = threadIdx.x / cp;
  for (int jb = 0; jb < d; jb += cp) {
    const int j = jb + int(threadIdx.x) % cp;
    unsigned long long m = 0ull;
    if (j < d)
      for (int64_t r = int64_t(blockIdx.x) * rp + rr; r < n; r += int64_t(gridDim.x) * rp) {
        const float a = fminf(fabsf(X[r * dp + j]), 9.2e18f);
        const unsigned long long v = static_cast<unsigned long long>(rint(static_cast<double>(a)));
        m = v > m ? v : m;
      }
    red[threadIdx.x] = m;
    __syncthreads();
    if (rr == 0 && j < d) {
      for (int q = 1; q < rp; ++q) m = red[q * cp + threadIdx.x] > m ? red[q * cp + threadIdx.x] : m;
      if (m) atomicMax(reinterpret_cast<unsigned long long*>(&mx[j]), m);
    }
    __syncthreads();
  }
}

// out[0] = n, out[1 + 4j + {0,1,2,3}] = sum q, sum a^2, sum 2ab, sum b^2
__global__ __launch_bounds__(kBlock) void k_km_moments_q(const float* X, const int64_t* counters, int d, int dp,
                                                         int cp, const int64_t* mx, int64_t* out) {
  __shared__ long long red[4][kBlock];
  const int64_t n = counters[0];
  const int rp = kBlock / cp, rr = threadIdx.x / cp;
  for (int jb = 0; jb < d; jb += cp) {
    const int j = jb + int(threadIdx.x) % cp;
    long long acc[4] = {0, 0, 0, 0};
    if (j < d) {
      const int sh = km_shift(mx[j]);
      for (int64_t r = int64_t(blockIdx.x) * rp + rr; r < n; r += int64_t(gridDim.x) * rp) {
        const int64_t q = km_q(X[r * dp + j], sh);
        const uint64_t u = static_cast<uint64_t>(q < 0 ? -q : q);
        const uint64_t a = u >> 16, b = u & 0xFFFFu;
        acc[0] += q;
        acc[1] += static_cast<long long>(a * a);
        acc[2] += static_cast<long long>(2u * a * b);
        acc[3] += static_cast<long long>(b * b);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) red[t][threadIdx.x] = acc[t];
    __syncthreads();
    if (rr == 0 && j < d) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        long long v = acc[t];
        for (int q = 1; q < rp; ++q) v += red[t][q * cp + threadIdx.x];
        if (v) atomicAdd(reinterpret_cast<unsigned long long*>(&out[1 + 4 * j + t]),
                         static_cast<unsigned long long>(v));
      }
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&out[0]),
                                                     static_cast<unsigned long long>(n));
}

static int km_moment_grid(int64_t max_rows) {
  int grid = int(max_rows / 256 + 1);
  return grid > 1024 ? 1024 : grid;
}

void launch_km_colmax(const float* X, const int64_t* counters, int d, int dp, int64_t* mx, int64_t max_rows,
                      hipStream_t s) {
  TWTML_LAUNCH(k_km_colmax, dim3(km_moment_grid(max_rows)), dim3(kBlock), 0, s, X, counters, d, dp,
                     km_cols_pow2(d), mx);
}

void launch_km_moments_q(const float* X, const int64_t* counters, int d, int dp, const int64_t* mx,
                         int64_t* out, int64_t max_rows, hipStream_t s) {
  TWTML_LAUNCH(k_km_moments_q, dim3(km_moment_grid(max_rows)), dim3(kBlock), 0, s, X, counters, d, dp,
                     km_cols_pow2(d), mx, out);
}

int km_quant_shift(int64_t mx) {
  const int L = mx > 0 ? 64 - __builtin_clzll(static_cast<unsigned long long>(mx)) : 0;
  return L > kKmQBits ? L - kKmQBits : 0;
}

// ---------------------------------------------------------------------------
// K8: assignment on the matrix cores.
//   block = 4 waves = 128 points; per 32-centre tile the tile (row-padded to
//   DP+1 floats: conflict-free column reads) is staged in LDS.  A operand =
//   centres (lane: row l&31, k = kk + l>>5), B operand = points^T (lane: point
//   l&31, same k) kept in VGPRs for the whole sweep.  D(32x32) lane l holds
//   point l&31 and centres (r&3) + 8(r>>2) + 4(l>>5), r = 0..15.
// ---------------------------------------------------------------------------
using f32x16 = __attribute__((ext_vector_type(16))) float;

// A gap between the best and second-best fp32 distance (|c|^2 - 2x.c) below
// this is within accumulated rounding (~160 ulps of |x|^2 + |c|^2 - 2|x.c|
// magnitudes): such points are re-decided in fp64 by k_km_refine.
__device__ __forceinline__ float km_tie_margin(float xn, float best) {
  return 1e-5f * (xn + fabsf(best)) + 1e-30f;
}

// Running best / second (with indices) / third distance of one point.
struct KmTop3 {
  float b1 = FLT_MAX, b2 = FLT_MAX, b3 = FLT_MAX;
  int i1 = 0, i2 = 0;
  __device__ __forceinline__ void add(float d, int c) {
    if (d < b1) { b3 = b2; b2 = b1; i2 = i1; b1 = d; i1 = c; }
    else if (d < b2) { b3 = b2; b2 = d; i2 = c; }
    else if (d < b3) b3 = d;
  }
  // Near-tie routing (refine layout: [0,R) full list, [R,2R) candidate
  // points, [2R,6R) up to 4 candidate centres per point, -1 padded; cnt[0]
  // full, cnt[1] candidate lists): when only two centres are within the
  // margin the fp64 re-decision compares just those two.
  __device__ __forceinline__ void route(int64_t p, float xn, int32_t* refine, unsigned long long* cnt,
                                        int64_t R) const {
    route_m(p, km_tie_margin(xn, b1), refine, cnt, R);
  }
  __device__ __forceinline__ void route_m(int64_t p, float m, int32_t* refine, unsigned long long* cnt,
                                          int64_t R) const {
    if (b2 - b1 > m) return;
    if (b3 - b1 <= m) {
      refine[atomicAdd(&cnt[0], 1ull)] = int32_t(p);
    } else {
      const int64_t q = int64_t(atomicAdd(&cnt[1], 1ull));
      refine[R + q] = int32_t(p);
      reinterpret_cast<int4*>(refine + 2 * R)[q] = make_int4(i1, i2, -1, -1);
    }
  }
};

template <int DP>
__global__ __launch_bounds__(kBlock) void k_km_assign_mfma(const float* X, const float* fac,
                                                           const int64_t* counters,
                                                           const float* C, const float* cnorm, int k,
                                                           int32_t* labels, int32_t* refine,
                                                           unsigned long long* refine_cnt, int64_t R) {
  constexpr int KS = DP / 2;          // MFMA k-steps
  constexpr int LD = DP + 1;          // padded LDS row
  __shared__ float ct[32 * LD];
  __shared__ float cn[32];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int64_t n = counters[0];
  if (int64_t(blockIdx.x) * 128 >= n) return;   // block-uniform
  const int64_t p = int64_t(blockIdx.x) * 128 + w * 32 + (lane & 31);
  const int half = lane >> 5;
  float xb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) xb[s] = p < n ? X[p * DP + 2 * s + half] * fac[2 * s + half] : 0.f;
  float xn = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) xn += xb[s] * xb[s];
  xn += __shfl_xor(xn, 32, kWave);
  KmTop3 t;
  for (int c0 = 0; c0 < k; c0 += 32) {
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * DP; i += kBlock) {
      const int r = i / DP, col = i % DP;
      ct[r * LD + col] = (c0 + r < k) ? C[int64_t(c0 + r) * DP + col] : 0.f;
    }
    if (threadIdx.x < 32) cn[threadIdx.x] = (c0 + int(threadIdx.x) < k) ? cnorm[c0 + threadIdx.x] : FLT_MAX;
    __syncthreads();
    f32x16 acc = {};
    const float* crow = ct + (lane & 31) * LD + half;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(crow[2 * s], xb[s], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cl = (r & 3) + 8 * (r >> 2) + 4 * half;
      t.add(cn[cl] - 2.f * acc[r], c0 + cl);
    }
  }
  // combine the two lane halves (interleaved centre sets).  Exact fp32 ties
  // fall inside the margin, so the fp64 refine settles them (first index).
  const float o1 = __shfl_xor(t.b1, 32, kWave), o2 = __shfl_xor(t.b2, 32, kWave);
  const float o3 = __shfl_xor(t.b3, 32, kWave);
  const int j1 = __shfl_xor(t.i1, 32, kWave), j2 = __shfl_xor(t.i2, 32, kWave);
  if (half == 0 && p < n) {
    t.add(o1, j1);
    t.add(o2, j2);
    t.add(o3, 0);      // can only land in third place
    labels[p] = t.i1;
    t.route(p, xn, refine, refine_cnt, R);
  }
}

// ---------------------------------------------------------------------------
// K8 on the bf16 matrix cores with split operands ("bf16x3"): x = xh + xl and
// c = ch + cl in bf16 (hi = rne(x), lo = rne(x - hi)), and x.c ~ xh.ch +
// xh.cl + xl.ch with v_mfma_f32_32x32x16_bf16 (fp32 accumulate).  Relative
// error of each product <= ~3 * 2^-18, so |dist error| <= ~1.1e-5 (|x|^2 +
// |c|^2); near ties inside a 1e-4 margin go to the fp64 refine like the fp32
// path.  3 bf16 MFMAs (K=16) replace 8 fp32 MFMAs (K=2) per 16 feature dims.
//
// No LDS and no barriers: the centres are split once per launch into
// ready-made A fragments ([tile][kb][hi|lo][lane][8 bf16], 1 KB per wave
// load, L2-resident), and each wave sweeps them for NB x 32 points held in
// VGPRs.  The epilogue keeps a sorted top-4 of packed keys -- the distance
// with its low `lbits` mantissa bits replaced by the centre index -- so an
// insertion is v_min + 3 x v_med3 with no index bookkeeping (5 VALU per
// distance with the fma and bfi, vs ~14 for compare/select chains).  The key
// quantisation (2^(lbits-23) relative) is added to the tie margin.
// ---------------------------------------------------------------------------
using bf16x8 = __attribute__((ext_vector_type(8))) short;

__device__ __forceinline__ uint16_t km_f2bf(float x) {
  uint32_t u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);   // round to nearest even
  return uint16_t(u >> 16);
}
__device__ __forceinline__ float km_bf2f(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

constexpr int kKmKeyBitsMax = 12;   // k <= 4096 on the packed-key path

// thread per (tile, kb, lane) fragment: 8 hi + 8 lo bf16; padded centres are
// zero with |c|^2 = FLT_MAX so they never win.
__global__ __launch_bounds__(kBlock) void k_km_split_bf16(const float* C, const float* cnorm, int k,
                                                          int dp, int ntiles, uint16_t* frag,
                                                          float* cnp) {
  const int KB = dp / 16;
  const int64_t nfrag = int64_t(ntiles) * KB * kWave;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nfrag;
       i += int64_t(gridDim.x) * kBlock) {
    const int lane = int(i % kWave), kb = int((i / kWave) % KB);
    const int64_t tile = i / (int64_t(kWave) * KB);
    const int64_t row = tile * 32 + (lane & 31);
    const int col0 = 16 * kb + 8 * (lane >> 5);
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = row < k ? C[row * dp + col0 + j] : 0.f;
      const uint16_t h = km_f2bf(v);
      hi[j] = short(h);
      lo[j] = short(km_f2bf(v - km_bf2f(h)));
    }
    bf16x8* f = reinterpret_cast<bf16x8*>(frag) + ((tile * KB + kb) * 2) * kWave + lane;
    f[0] = hi;
    f[kWave] = lo;
  }
  for (int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x; c < int64_t(ntiles) * 32;
       c += int64_t(gridDim.x) * kBlock)
    cnp[c] = c < k ? cnorm[c] : FLT_MAX;
}

struct KmKeys4 {           // sorted b[0] <= b[1] <= b[2] <= b[3]
  float b[4] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
  __device__ __forceinline__ void add(float key) {
    const float n3 = __builtin_amdgcn_fmed3f(b[2], b[3], key);
    const float n2 = __builtin_amdgcn_fmed3f(b[1], b[2], key);
    const float n1 = __builtin_amdgcn_fmed3f(b[0], b[1], key);
    b[0] = __builtin_amdgcn_fmed3f(b[0], key, -FLT_MAX);   // a min without fminf's canonicalize
    b[1] = n1;
    b[2] = n2;
    b[3] = n3;
  }
};

template <int DP, int NB>
__global__ __launch_bounds__(kBlock) void k_km_assign_bf16x3(const float* X, const float* fac,
                                                             const int64_t* counters,
                                                             const uint16_t* frag, const float* cnp,
                                                             int ntiles, int lbits, int32_t* labels,
                                                             int32_t* refine,
                                                             unsigned long long* refine_cnt, int64_t R) {
  static_assert(DP % 16 == 0, "bf16x3 path needs DP % 16 == 0");
  constexpr int KB = DP / 16;
  const int lane = lane_id(), h = lane >> 5;
  const int64_t n = counters[0];
  const int64_t p0 = ((int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave) * (32 * NB);
  if (p0 >= n) return;                                  // wave-uniform
  bf16x8 xh[NB][KB], xl[NB][KB];
  float xn[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int64_t p = p0 + 32 * b + (lane & 31);
    xn[b] = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int col = 16 * kb + 8 * h;
      float v[8];
      if (p < n) {
        const float4 a = *reinterpret_cast<const float4*>(X + p * DP + col);
        const float4 c = *reinterpret_cast<const float4*>(X + p * DP + col + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = v[j] * fac[col + j];
        xn[b] += x * x;
        const uint16_t hi = km_f2bf(x);
        xh[b][kb][j] = short(hi);
        xl[b][kb][j] = short(km_f2bf(x - km_bf2f(hi)));
      }
    }
    xn[b] += __shfl_xor(xn[b], 32, kWave);
  }
  const uint32_t imask = (1u << lbits) - 1u;
  KmKeys4 t[NB];
  const bf16x8* F = reinterpret_cast<const bf16x8*>(frag) + lane;
  for (int tile = 0; tile < ntiles; ++tile) {
    bf16x8 ah[KB], al[KB];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      ah[kb] = F[((int64_t(tile) * KB + kb) * 2) * kWave];
      al[kb] = F[((int64_t(tile) * KB + kb) * 2 + 1) * kWave];
    }
    float cn[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 c = *reinterpret_cast<const float4*>(cnp + tile * 32 + 8 * q + 4 * h);
      cn[4 * q] = c.x; cn[4 * q + 1] = c.y; cn[4 * q + 2] = c.z; cn[4 * q + 3] = c.w;
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      f32x16 acc = {};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[kb], xh[b][kb], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[kb], xl[b][kb], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[kb], xh[b][kb], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t idx = uint32_t(tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h);
        const float dist = fmaf(-2.f, acc[r], cn[r]);
        t[b].add(__uint_as_float((__float_as_uint(dist) & ~imask) | idx));
      }
    }
  }
  const float q = ldexpf(1.f, lbits - 21);   // 4 key quanta, relative
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __shfl_xor(t[b].b[j], 32, kWave);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[b].add(o[j]);
    const int64_t p = p0 + 32 * b + (lane & 31);
    if (h != 0 || p >= n) continue;
    const float* k4 = t[b].b;
    const int i1 = int(__float_as_uint(k4[0]) & imask);
    labels[p] = i1;
    const float m = 1e-4f * (3.f * xn[b] + fabsf(k4[0]) + cnp[i1]) + q * fabsf(k4[0]) + 1e-30f;
    if (k4[1] - k4[0] > m) continue;
    if (k4[3] - k4[0] <= m) {
      refine[atomicAdd(&refine_cnt[0], 1ull)] = int32_t(p);
    } else {
      const int64_t qn = int64_t(atomicAdd(&refine_cnt[1], 1ull));
      refine[R + qn] = int32_t(p);
      int4 cand;
      cand.x = i1;
      cand.y = int(__float_as_uint(k4[1]) & imask);
      cand.z = k4[2] - k4[0] <= m ? int(__float_as_uint(k4[2]) & imask) : -1;
      cand.w = -1;
      reinterpret_cast<int4*>(refine + 2 * R)[qn] = cand;
    }
  }
}

// The same bf16x3 assignment with the centre fragments shared through LDS
// (TWTML_KM_ASSIGN=lds; the pipelined variant below is the default).  k_km_assign_bf16x3 has every wave
// fetch every tile's fragments from L2 (8 KB per tile per wave at d = 64:
// ~4 GB of L2 reads per 1M points x 1024 centres) and wait on them right
// before its MFMAs -- 545 us at 1.8 waves/SIMD.  Here the
// workgroup's 4 waves load a tile once, cooperatively, one tile AHEAD into
// registers (2 x 16 B per thread), park it in a double-buffered LDS slot
// (one barrier per tile), and each wave reads its A operands with
// conflict-free ds_read_b128 just before the MFMAs that use them.  The
// epilogue and the near-tie routing are k_km_assign_bf16x3's: a top-4, so
// the twin / triplet centres that repeated dying-cluster splits leave behind
// go to the 2-3 candidate refine (a top-3 sent the triplets to the full
// refine: +620 us per batch on the wide profile).
template <int DP, int NB>
__global__ __launch_bounds__(kBlock) void k_km_assign_bf16x3_lds(const float* X, const float* fac,
                                                                 const int64_t* counters,
                                                                 const uint16_t* frag,
                                                                 const float* cnp, int ntiles,
                                                                 int lbits, int32_t* labels,
                                                                 int32_t* refine,
                                                                 unsigned long long* refine_cnt,
                                                                 int64_t R) {
  static_assert(DP % 16 == 0, "bf16x3 path needs DP % 16 == 0");
  constexpr int KB = DP / 16;
  constexpr int TILE_V = KB * 2 * kWave;                 // bf16x8 vectors per tile
  constexpr int PER_T = (TILE_V + kBlock - 1) / kBlock;  // per thread per tile
  __shared__ bf16x8 fs[2][TILE_V];
  __shared__ float cs[2][32];
  const int lane = lane_id(), h = lane >> 5;
  const int64_t n = counters[0];
  const int64_t pb = int64_t(blockIdx.x) * (kBlock / kWave) * (32 * NB);
  if (pb >= n) return;                                   // block-uniform
  const int64_t p0 = pb + int64_t(threadIdx.x / kWave) * (32 * NB);
  const bf16x8* F = reinterpret_cast<const bf16x8*>(frag);
  bf16x8 pre[PER_T];
  float pc = 0.f;
  auto fetch = [&](int tile) {
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int v = threadIdx.x + j * kBlock;
      if (v < TILE_V) pre[j] = F[int64_t(tile) * TILE_V + v];
    }
    if (threadIdx.x < 32) pc = cnp[tile * 32 + threadIdx.x];
  };
  auto park = [&](int buf) {
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int v = threadIdx.x + j * kBlock;
      if (v < TILE_V) fs[buf][v] = pre[j];
    }
    if (threadIdx.x < 32) cs[buf][threadIdx.x] = pc;
  };
  fetch(0);
  bf16x8 xh[NB][KB], xl[NB][KB];
  float xn[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int64_t p = p0 + 32 * b + (lane & 31);
    xn[b] = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int col = 16 * kb + 8 * h;
      float v[8];
      if (p < n) {
        const float4 a = *reinterpret_cast<const float4*>(X + p * DP + col);
        const float4 c = *reinterpret_cast<const float4*>(X + p * DP + col + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = v[j] * fac[col + j];
        xn[b] += x * x;
        const uint16_t hi = km_f2bf(x);
        xh[b][kb][j] = short(hi);
        xl[b][kb][j] = short(km_f2bf(x - km_bf2f(hi)));
      }
    }
    xn[b] += __shfl_xor(xn[b], 32, kWave);
  }
  park(0);
  __syncthreads();
  const uint32_t imask = (1u << lbits) - 1u;
  KmKeys4 t[NB];
  for (int tile = 0; tile < ntiles; ++tile) {
    const int buf = tile & 1;
    if (tile + 1 < ntiles) fetch(tile + 1);              // in flight during this tile
    f32x16 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = f32x16{};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const bf16x8 ah = fs[buf][(kb * 2) * kWave + lane];
      const bf16x8 al = fs[buf][(kb * 2 + 1) * kWave + lane];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[b][kb], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xl[b][kb], acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, xh[b][kb], acc[b], 0, 0, 0);
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int cl = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float dist = fmaf(-2.f, acc[b][r], cs[buf][cl]);
        t[b].add(__uint_as_float((__float_as_uint(dist) & ~imask) | uint32_t(tile * 32 + cl)));
      }
    }
    if (tile + 1 < ntiles) park(buf ^ 1);   // its readers finished at the last barrier
    __syncthreads();
  }
  const float q = ldexpf(1.f, lbits - 21);   // 4 key quanta, relative
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __shfl_xor(t[b].b[j], 32, kWave);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[b].add(o[j]);
    const int64_t p = p0 + 32 * b + (lane & 31);
    if (h != 0 || p >= n) continue;
    const float* k4 = t[b].b;
    const int i1 = int(__float_as_uint(k4[0]) & imask);
    labels[p] = i1;
    const float m = 1e-4f * (3.f * xn[b] + fabsf(k4[0]) + cnp[i1]) + q * fabsf(k4[0]) + 1e-30f;
    if (k4[1] - k4[0] > m) continue;
    if (k4[3] - k4[0] <= m) {
      refine[atomicAdd(&refine_cnt[0], 1ull)] = int32_t(p);
    } else {
      const int64_t qn = int64_t(atomicAdd(&refine_cnt[1], 1ull));
      refine[R + qn] = int32_t(p);
      reinterpret_cast<int4*>(refine + 2 * R)[qn] =
          make_int4(i1, int(__float_as_uint(k4[1]) & imask),
                    k4[2] - k4[0] <= m ? int(__float_as_uint(k4[2]) & imask) : -1, -1);
    }
  }
}

// bf16x3 assignment with the epilogue software-pipelined behind the next
// tile's MFMAs (the default; TWTML_KM_ASSIGN=lds selects the kernel above;
// one 32-point block per wave).  In
// k_km_assign_bf16x3_lds a wave runs its 12 dependent MFMAs, then its 16
// distance insertions, then the barrier: the matrix pipe idles during the
// wave's VALU and the VALU during its MFMAs unless the SIMD's other waves
// happen to be out of phase.  Here the MFMAs of tile t and the insertions of
// tile t-1 (accumulator and centre norms held in registers across the
// barrier) sit in one basic block, interleaved by sched_group_barrier: ~10
// VALU per MFMA fill its dependency shadow.  Two accumulators and two norm
// sets (32 VGPRs) are the price.
template <int DP>
__global__ __launch_bounds__(kBlock) void k_km_assign_bf16x3_pipe(const float* X, const float* fac,
                                                                  const int64_t* counters,
                                                                  const uint16_t* frag,
                                                                  const float* cnp, int ntiles,
                                                                  int lbits, int32_t* labels,
                                                                  int32_t* refine,
                                                                  unsigned long long* refine_cnt,
                                                                  int64_t R) {
  static_assert(DP % 16 == 0, "bf16x3 path needs DP % 16 == 0");
  constexpr int KB = DP / 16;
  constexpr int TILE_V = KB * 2 * kWave;
  constexpr int PER_T = (TILE_V + kBlock - 1) / kBlock;
  __shared__ bf16x8 fs[2][TILE_V];
  __shared__ float cs[2][32];
  const int lane = lane_id(), h = lane >> 5;
  const int64_t n = counters[0];
  const int64_t pb = int64_t(blockIdx.x) * (kBlock / kWave) * 32;
  if (pb >= n) return;                                   // block-uniform
  const int64_t p = pb + int64_t(threadIdx.x / kWave) * 32 + (lane & 31);
  const bf16x8* F = reinterpret_cast<const bf16x8*>(frag);
  bf16x8 pre[PER_T];
  float pc = 0.f;
  auto fetch = [&](int tile) {
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int v = threadIdx.x + j * kBlock;
      if (TILE_V % kBlock == 0 || v < TILE_V) pre[j] = F[int64_t(tile) * TILE_V + v];
    }
    pc = cnp[tile * 32 + (threadIdx.x & 31)];   // branch-free: keeps the loop body one block
  };
  auto park = [&](int buf) {
#pragma unroll
    for (int j = 0; j < PER_T; ++j) {
      const int v = threadIdx.x + j * kBlock;
      if (TILE_V % kBlock == 0 || v < TILE_V) fs[buf][v] = pre[j];
    }
    cs[buf][threadIdx.x & 31] = pc;   // 8 lanes store each (identical) norm
  };
  fetch(0);
  bf16x8 xh[KB], xl[KB];
  float xn = 0.f;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int col = 16 * kb + 8 * h;
    float v[8];
    if (p < n) {
      const float4 a = *reinterpret_cast<const float4*>(X + p * DP + col);
      const float4 c = *reinterpret_cast<const float4*>(X + p * DP + col + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = v[j] * fac[col + j];
      xn += x * x;
      const uint16_t hi = km_f2bf(x);
      xh[kb][j] = short(hi);
      xl[kb][j] = short(km_f2bf(x - km_bf2f(hi)));
    }
  }
  xn += __shfl_xor(xn, 32, kWave);
  const uint32_t imask = (1u << lbits) - 1u;
  KmKeys4 t;
  auto mfma_tile = [&](int tile, f32x16& acc, float (&cn)[16]) {
    const int buf = tile & 1;
    acc = f32x16{};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const bf16x8 ah = fs[buf][(kb * 2) * kWave + lane];
      const bf16x8 al = fs[buf][(kb * 2 + 1) * kWave + lane];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh[kb], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xl[kb], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, xh[kb], acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 c = *reinterpret_cast<const float4*>(&cs[buf][8 * q + 4 * h]);
      cn[4 * q] = c.x; cn[4 * q + 1] = c.y; cn[4 * q + 2] = c.z; cn[4 * q + 3] = c.w;
    }
  };
  auto epi = [&](int tile, const f32x16& acc, const float (&cn)[16]) {
    const uint32_t base = uint32_t(tile * 32 + 4 * h);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float dist = fmaf(-2.f, acc[r], cn[r]);
      t.add(__uint_as_float((__float_as_uint(dist) & ~imask) | (base + uint32_t((r & 3) + 8 * (r >> 2)))));
    }
  };
  // 12 MFMAs (d = 64) with the previous tile's ~130 VALU spread between them.
  // The empty asm pins the insertions ahead of the barrier (pure arithmetic
  // is otherwise sunk past it, next to the following tile's epilogue).
  auto interleave = [&] {
    asm volatile("" : "+v"(t.b[0]), "+v"(t.b[1]), "+v"(t.b[2]), "+v"(t.b[3]));
#pragma unroll
    for (int i = 0; i < 3 * KB; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);   // then up to 10 VALU
    }
  };
  f32x16 acc0, acc1;
  float cn0[16], cn1[16];
  park(0);
  if (ntiles > 1) fetch(1);
  __syncthreads();
  mfma_tile(0, acc0, cn0);
  if (ntiles > 1) park(1);
  __syncthreads();
  int tile = 1;
  for (; tile + 1 < ntiles; tile += 2) {
    fetch(tile + 1);
    mfma_tile(tile, acc1, cn1);
    epi(tile - 1, acc0, cn0);
    interleave();
    park(0);   // tile + 1 (even); tile - 1's readers passed the last barrier
    __syncthreads();
    const bool more = tile + 2 < ntiles;
    if (more) fetch(tile + 2);
    mfma_tile(tile + 1, acc0, cn0);
    epi(tile, acc1, cn1);
    interleave();
    if (more) park(1);
    __syncthreads();
  }
  if (tile < ntiles) {
    mfma_tile(tile, acc1, cn1);
    epi(tile - 1, acc0, cn0);
    interleave();
    epi(tile, acc1, cn1);
  } else {
    epi(tile - 1, acc0, cn0);
  }
  const float q = ldexpf(1.f, lbits - 21);   // 4 key quanta, relative
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = __shfl_xor(t.b[j], 32, kWave);
#pragma unroll
  for (int j = 0; j < 4; ++j) t.add(o[j]);
  if (h != 0 || p >= n) return;
  const float* k4 = t.b;
  const int i1 = int(__float_as_uint(k4[0]) & imask);
  labels[p] = i1;
  const float m = 1e-4f * (3.f * xn + fabsf(k4[0]) + cnp[i1]) + q * fabsf(k4[0]) + 1e-30f;
  if (k4[1] - k4[0] > m) return;
  if (k4[3] - k4[0] <= m) {
    refine[atomicAdd(&refine_cnt[0], 1ull)] = int32_t(p);
  } else {
    const int64_t qn = int64_t(atomicAdd(&refine_cnt[1], 1ull));
    refine[R + qn] = int32_t(p);
    reinterpret_cast<int4*>(refine + 2 * R)[qn] =
        make_int4(i1, int(__float_as_uint(k4[1]) & imask),
                  k4[2] - k4[0] <= m ? int(__float_as_uint(k4[2]) & imask) : -1, -1);
  }
}

// Generic fallback (any width): one thread per point, scalar fp32.
__global__ __launch_bounds__(kBlock) void k_km_assign_scalar(const float* X, const float* fac,
                                                             const int64_t* counters,
                                                             const float* C, const float* cnorm, int k,
                                                             int dp, int32_t* labels, int32_t* refine,
                                                             unsigned long long* refine_cnt, int64_t R) {
  const int64_t n = counters[0];
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < n; p += int64_t(gridDim.x) * kBlock) {
    KmTop3 t;
    float xn = 0.f;
    for (int j = 0; j < dp; ++j) xn += (X[p * dp + j] * fac[j]) * (X[p * dp + j] * fac[j]);
    for (int c = 0; c < k; ++c) {
      float dot = 0.f;
      for (int j = 0; j < dp; ++j) dot += C[int64_t(c) * dp + j] * (X[p * dp + j] * fac[j]);
      t.add(cnorm[c] - 2.f * dot, c);
    }
    labels[p] = t.i1;
    t.route(p, xn, refine, refine_cnt, R);
  }
}

// fp64 re-decision among a short candidate list (2-3 centres; typically the
// two halves of a just-split cluster, 1e-14 apart -- invisible in fp32):
// thread per point, first index on exact ties.
__global__ __launch_bounds__(kBlock) void k_km_refine_cand(const float* X, const double* fac,
                                                           const int32_t* refine,
                                                           const unsigned long long* refine_cnt,
                                                           const double* centers, int d, int dp,
                                                           int64_t R, int32_t* labels) {
  const int64_t np = int64_t(refine_cnt[1]);
  for (int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x; q < np; q += int64_t(gridDim.x) * kBlock) {
    const int64_t p = refine[R + q];
    const int4 c4 = reinterpret_cast<const int4*>(refine + 2 * R)[q];
    const int cand[4] = {c4.x, c4.y, c4.z, c4.w};
    const float* x = X + p * dp;
    double best = DBL_MAX;
    int bi = 0x7fffffff;
    for (int i = 0; i < 4 && cand[i] >= 0; ++i) {
      const double* c = centers + int64_t(cand[i]) * d;
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double t = double(x[j]) * fac[j] - c[j];
        s += t * t;
      }
      if (s < best || (s == best && cand[i] < bi)) { best = s; bi = cand[i]; }
    }
    labels[p] = bi;
  }
}

// fp64 re-decision when three or more centres are within the margin: one
// wave per point, direct sum of squared differences against all fp64
// centres, first index on exact ties.
__global__ __launch_bounds__(kBlock) void k_km_refine(const float* X, const double* fac,
                                                      const int32_t* refine,
                                                      const unsigned long long* refine_cnt,
                                                      const double* centers, int k, int d, int dp,
                                                      int32_t* labels) {
  const int lane = lane_id();
  const int64_t nref = int64_t(*refine_cnt);
  for (int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; q < nref;
       q += int64_t(gridDim.x) * (kBlock / kWave)) {
    const int64_t p = refine[q];
    const float* x = X + p * dp;
    double best = DBL_MAX;
    int bi = 0x7fffffff;
    for (int c = lane; c < k; c += kWave) {
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double t = double(x[j]) * fac[j] - centers[int64_t(c) * d + j];
        s += t * t;
      }
      if (s < best) { best = s; bi = c; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ob = __shfl_xor(best, off, kWave);
      const int oi = __shfl_xor(bi, off, kWave);
      if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) labels[p] = bi;
  }
}

void launch_km_assign(const float* X, const float* f32, const double* f64, const int64_t* counters,
                      const float* C, const float* cnorm, const double* centers, int k, int d, int dp,
                      int32_t* labels, int32_t* refine, unsigned long long* refine_cnt,
                      uint16_t* frag, float* cnp, int64_t max_rows, bool mfma, bool bf16,
                      hipStream_t s) {
  TWTML_HIP_CHECK(hipMemsetAsync(refine_cnt, 0, 2 * sizeof(unsigned long long), s));
  const int grid_m = int(max_rows / 128 + 1);
  const int64_t R = max_rows;
  bool done = false;
  const int ntiles = (k + 31) / 32;
  int lbits = 1;
  while ((1 << lbits) < ntiles * 32) ++lbits;
  if (mfma && bf16 && dp >= 16 && dp <= 128 && lbits <= kKmKeyBitsMax) {
    int gs = int((int64_t(ntiles) * (dp / 16) * kWave + kBlock - 1) / kBlock);
    TWTML_LAUNCH(k_km_split_bf16, dim3(gs < 1024 ? gs : 1024), dim3(kBlock), 0, s, C, cnorm, k,
                       dp, ntiles, frag, cnp);
#define KM_BF16L(DPV, NBV)                                                                         \
  case DPV: {                                                                                      \
    const int64_t waves = (max_rows + 32 * NBV - 1) / (32 * NBV);                                  \
    TWTML_LAUNCH((k_km_assign_bf16x3_lds<DPV, NBV>), dim3(int((waves + 3) / 4)), dim3(kBlock), \
                       0, s, X, f32, counters, frag, cnp, ntiles, lbits, labels, refine, refine_cnt, \
                       R);                                                                         \
    done = true;                                                                                   \
    break;                                                                                         \
  }
#define KM_BF16(DPV, NBV)                                                                          \
  case DPV: {                                                                                      \
    const int64_t waves = (max_rows + 32 * NBV - 1) / (32 * NBV);                                  \
    TWTML_LAUNCH((k_km_assign_bf16x3<DPV, NBV>), dim3(int((waves + 3) / 4)), dim3(kBlock), 0, \
                       s, X, f32, counters, frag, cnp, ntiles, lbits, labels, refine, refine_cnt, R); \
    done = true;                                                                                   \
    break;                                                                                         \
  }
    // TWTML_KM_ASSIGN: pipe (default: the lds kernel with its epilogue
    // software-pipelined behind the next tile's MFMAs), lds (one 32-point
    // block per wave, 4 waves per SIMD at d = 64), lds2 (two blocks per wave,
    // 2 waves per SIMD), reg (per-wave L2 fragment loads, the round-2 kernel)
    // -- for A/B runs; all four are bitwise identical
    // (tests/test_gpu_kmeans.py).  Measured at k = 1024, d = 64, 1M points:
    // round 3 reg 572 us, lds2 538, lds 462; round 5 (overlapped with the
    // next batch's decode, profiles/r5/kernels_kmeans_*.txt) lds 440, pipe 424.
    static const int variant = [] {
      const char* e = std::getenv("TWTML_KM_ASSIGN");
      if (e && std::strcmp(e, "reg") == 0) return 0;
      if (e && std::strcmp(e, "lds2") == 0) return 2;
      if (e && std::strcmp(e, "lds") == 0) return 1;
      return 3;
    }();
#define KM_BF16P(DPV)                                                                              \
  case DPV: {                                                                                      \
    const int64_t waves = (max_rows + 31) / 32;                                                    \
    TWTML_LAUNCH((k_km_assign_bf16x3_pipe<DPV>), dim3(int((waves + 3) / 4)), dim3(kBlock),   \
                       0, s, X, f32, counters, frag, cnp, ntiles, lbits, labels, refine, refine_cnt, \
                       R);                                                                         \
    done = true;                                                                                   \
    break;                                                                                         \
  }
    if (variant == 3) {
      switch (dp) { KM_BF16P(16) KM_BF16P(32) KM_BF16P(64) KM_BF16P(128) default: break; }
    } else if (variant == 0) {
      switch (dp) { KM_BF16(16, 2) KM_BF16(32, 2) KM_BF16(64, 2) KM_BF16(128, 1) default: break; }
    } else if (variant == 2) {
      switch (dp) { KM_BF16L(16, 2) KM_BF16L(32, 2) KM_BF16L(64, 2) KM_BF16L(128, 1) default: break; }
    } else {
      switch (dp) { KM_BF16L(16, 1) KM_BF16L(32, 1) KM_BF16L(64, 1) KM_BF16L(128, 1) default: break; }
    }
#undef KM_BF16
#undef KM_BF16L
#undef KM_BF16P
  }
  if (mfma && !done) {
#define KM_MFMA(DPV)                                                                                \
  case DPV:                                                                                         \
    TWTML_LAUNCH(k_km_assign_mfma<DPV>, dim3(grid_m), dim3(kBlock), 0, s, X, f32, counters, C, \
                       cnorm, k, labels, refine, refine_cnt, R);                                    \
    done = true;                                                                                    \
    break;
    switch (dp) { KM_MFMA(2) KM_MFMA(4) KM_MFMA(8) KM_MFMA(16) KM_MFMA(32) KM_MFMA(64) KM_MFMA(128) default: break; }
#undef KM_MFMA
  }
  int grid = int(max_rows / kBlock + 1);
  if (grid > 4096) grid = 4096;
  if (!done)
    TWTML_LAUNCH(k_km_assign_scalar, dim3(grid), dim3(kBlock), 0, s, X, f32, counters, C, cnorm,
                       k, dp, labels, refine, refine_cnt, R);
  const int grid_r = grid < 1024 ? grid : 1024;
  TWTML_LAUNCH(k_km_refine_cand, dim3(grid_r), dim3(kBlock), 0, s, X, f64, refine, refine_cnt,
                     centers, d, dp, R, labels);
  TWTML_LAUNCH(k_km_refine, dim3(grid_r), dim3(kBlock), 0, s, X, f64, refine, refine_cnt,
                     centers, k, d, dp, labels);
}

// ---------------------------------------------------------------------------
// K9: counting sort by label + segmented sums with one atomic per label run.
//
// Labels are heavily skewed (most points fall in a few clusters), so global
// per-point atomics serialise on a handful of addresses.  The histogram and
// the scatter are privatised per block in LDS, and each wave first "peels"
// its dominant labels with ballots: one LDS atomic per distinct label per
// round, lane ranks from popcounts.  Blocks then reserve one global range
// per (block, label).
// ---------------------------------------------------------------------------
constexpr int kKmChunk = 4096;      // points per block pass (multiple of kBlock)
constexpr int kKmLdsBins = 8192;    // k limit for the LDS-privatised path

// Returns this lane's rank among the points with the same label in cnt[label].
__device__ __forceinline__ uint32_t km_peel_add(uint32_t* cnt, int label, bool active) {
  const int lane = lane_id();
  uint64_t rem = __ballot(active);
  uint32_t mine = 0;
  for (int it = 0; it < 4 && rem; ++it) {
    const int leader = __builtin_ctzll(rem);
    const int L = __shfl(label, leader, kWave);
    const uint64_t mask = __ballot(active && label == L) & rem;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&cnt[L], uint32_t(__popcll(mask)));
    base = __shfl(base, leader, kWave);
    if ((mask >> lane) & 1ull) mine = base + uint32_t(__popcll(mask & ((1ull << lane) - 1ull)));
    rem &= ~mask;
  }
  if ((rem >> lane) & 1ull) mine = atomicAdd(&cnt[label], 1u);
  return mine;
}

__global__ __launch_bounds__(kBlock) void k_km_label_hist(const int32_t* labels, const int64_t* counters,
                                                          int k, int64_t* hist) {
  extern __shared__ uint32_t cnt[];
  const int64_t n = counters[0];
  for (int c = threadIdx.x; c < k; c += kBlock) cnt[c] = 0u;
  __syncthreads();
  for (int64_t base = int64_t(blockIdx.x) * kKmChunk; base < n; base += int64_t(gridDim.x) * kKmChunk)
    for (int i = threadIdx.x; i < kKmChunk; i += kBlock) {
      const int64_t p = base + i;
      km_peel_add(cnt, p < n ? labels[p] : 0, p < n);
    }
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += kBlock)
    if (cnt[c]) atomicAdd(reinterpret_cast<unsigned long long*>(&hist[c]), (unsigned long long)cnt[c]);
}

__global__ __launch_bounds__(kBlock) void k_km_label_scatter(const int32_t* labels, const int64_t* counters,
                                                             int k, int64_t* cursor, int32_t* order) {
  extern __shared__ uint32_t sh[];
  uint32_t* cnt = sh;          // [k]
  uint32_t* rbase = sh + k;    // [k] reserved global base per label
  const int64_t n = counters[0];
  for (int64_t base = int64_t(blockIdx.x) * kKmChunk; base < n; base += int64_t(gridDim.x) * kKmChunk) {
    for (int c = threadIdx.x; c < k; c += kBlock) cnt[c] = 0u;
    __syncthreads();
    for (int i = threadIdx.x; i < kKmChunk; i += kBlock) {
      const int64_t p = base + i;
      km_peel_add(cnt, p < n ? labels[p] : 0, p < n);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < k; c += kBlock) {
      const uint32_t m = cnt[c];
      rbase[c] = m ? uint32_t(atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[c]),
                                        (unsigned long long)m)) : 0u;
      cnt[c] = 0u;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kKmChunk; i += kBlock) {
      const int64_t p = base + i;
      const int lab = p < n ? labels[p] : 0;
      const uint32_t r = km_peel_add(cnt, lab, p < n);
      if (p < n) order[rbase[lab] + r] = int32_t(p);
    }
    __syncthreads();
  }
}

// k > kKmLdsBins: plain global atomics
__global__ __launch_bounds__(kBlock) void k_km_label_hist_g(const int32_t* labels, const int64_t* counters,
                                                            int64_t* hist) {
  const int64_t n = counters[0];
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < n; p += int64_t(gridDim.x) * kBlock)
    atomicAdd(reinterpret_cast<unsigned long long*>(&hist[labels[p]]), 1ull);
}

__global__ __launch_bounds__(kBlock) void k_km_label_scatter_g(const int32_t* labels, const int64_t* counters,
                                                               int64_t* cursor, int32_t* order) {
  const int64_t n = counters[0];
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < n; p += int64_t(gridDim.x) * kBlock) {
    const int64_t pos = int64_t(atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[labels[p]]), 1ull));
    order[pos] = int32_t(p);
  }
}

constexpr int kSegRows = 1024;
// k * d + k sums up to this many go through an LDS copy per workgroup
constexpr int kSegLdsSums = 4096;

// Per-cluster sums of the quantized features (km_q) and counts, int64:
// exact, so every rank / grid / order gives the same bits.  thread = (row
// lane rr, column j); walks rows rr, rr+RP, ... of its chunk in label order
// and flushes its running sum whenever the label changes.  LDS: flushes go to
// the workgroup's LDS copy (ds_add_u64), added to the global sums once at the
// end -- with few clusters (the reference's k = 3) every workgroup's flushes
// would otherwise hit the same handful of global atomics.
template <bool LDS>
__global__ __launch_bounds__(kBlock) void k_km_segsum(const float* X, const int64_t* mx,
                                                      const int32_t* labels,
                                                      const int32_t* order, const int64_t* counters,
                                                      int k, int d, int dp, int cols_pow2, int64_t* sums) {
  extern __shared__ unsigned long long lsum[];   // LDS: [k * d] sums, then [k] counts
  const int64_t n = counters[0];
  const int nsum = k * d + k;
  auto* gsum = reinterpret_cast<unsigned long long*>(sums);
  if (LDS) {
    for (int i = threadIdx.x; i < nsum; i += kBlock) lsum[i] = 0ull;
    __syncthreads();
  }
  auto flush = [&](int cur, int j, long long acc, long long cnt) {
    unsigned long long* dst = LDS ? lsum : gsum;
    if (j < d && acc) atomicAdd(&dst[cur * d + j], static_cast<unsigned long long>(acc));
    if (j == 0) atomicAdd(&dst[k * d + cur], static_cast<unsigned long long>(cnt));
  };
  const int rp = kBlock / cols_pow2;               // rows per pass
  const int rr = threadIdx.x / cols_pow2;
  for (int64_t base = int64_t(blockIdx.x) * kSegRows; base < n; base += int64_t(gridDim.x) * kSegRows)
  for (int j = threadIdx.x % cols_pow2; j < d; j += cols_pow2) {   // column passes (d > 256)
    const int64_t end = base + kSegRows < n ? base + kSegRows : n;
    const int sh = km_shift(mx[j]);
    int cur = -1;
    long long acc = 0, cnt = 0;
    for (int64_t q = base + rr; q < end; q += rp) {
      const int32_t p = order[q];
      const int lab = labels[p];
      if (lab != cur) {
        if (cur >= 0) flush(cur, j, acc, cnt);
        cur = lab; acc = 0; cnt = 0;
      }
      acc += km_q(X[int64_t(p) * dp + j], sh);
      cnt += 1;
    }
    if (cur >= 0) flush(cur, j, acc, cnt);
  }
  if (LDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < nsum; i += kBlock) {
      const unsigned long long v = lsum[i];
      if (v) atomicAdd(&gsum[i], v);
    }
  }
}

void launch_km_cluster_sums(const float* X, const int64_t* mx, const int32_t* labels,
                            const int64_t* counters, int k,
                            int d, int dp, int64_t* hist, int32_t* order, int64_t* sums,
                            int64_t max_rows, hipStream_t s,
                            void (*scan)(const int64_t*, int64_t*, int64_t, int64_t*, hipStream_t)) {
  TWTML_HIP_CHECK(hipMemsetAsync(hist, 0, sizeof(int64_t) * size_t(k + 1), s));
  if (k <= kKmLdsBins) {
    int grid = int((max_rows + kKmChunk - 1) / kKmChunk);
    grid = grid < 1 ? 1 : (grid > 1024 ? 1024 : grid);
    TWTML_LAUNCH(k_km_label_hist, dim3(grid), dim3(kBlock), sizeof(uint32_t) * size_t(k), s,
                       labels, counters, k, hist);
    scan(hist, hist, k, nullptr, s);
    TWTML_LAUNCH(k_km_label_scatter, dim3(grid), dim3(kBlock), 2 * sizeof(uint32_t) * size_t(k), s,
                       labels, counters, k, hist, order);
  } else {
    int grid = int(max_rows / kBlock + 1);
    if (grid > 4096) grid = 4096;
    TWTML_LAUNCH(k_km_label_hist_g, dim3(grid), dim3(kBlock), 0, s, labels, counters, hist);
    scan(hist, hist, k, nullptr, s);
    TWTML_LAUNCH(k_km_label_scatter_g, dim3(grid), dim3(kBlock), 0, s, labels, counters, hist, order);
  }
  int g2 = int(max_rows / kSegRows + 1);
  if (g2 > 4096) g2 = 4096;
  if (k * d + k <= kSegLdsSums)
    TWTML_LAUNCH(k_km_segsum<true>, dim3(g2), dim3(kBlock), sizeof(int64_t) * size_t(k * d + k), s, X, mx,
                       labels, order, counters, k, d, dp, km_cols_pow2(d), sums);
  else
    TWTML_LAUNCH(k_km_segsum<false>, dim3(g2), dim3(kBlock), 0, s, X, mx, labels, order, counters, k, d,
                       dp, km_cols_pow2(d), sums);
}

// the all-reduced integer sums -> the fp64 sums of the SCALED features
// (factor_j 2^s_j sum q) and the counts the update reads
__global__ void k_km_sums_f64(const int64_t* si, const int64_t* mx, const double* fac, int k, int d,
                              double* sums, double* counts) {
  const int64_t total = int64_t(k) * d + k;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    if (i < int64_t(k) * d) {
      const int j = int(i % d);
      sums[i] = ldexp(static_cast<double>(si[i]), km_shift(mx[j])) * fac[j];
    } else {
      counts[i - int64_t(k) * d] = static_cast<double>(si[i]);
    }
  }
}

void launch_km_sums_f64(const int64_t* si, const int64_t* mx, const double* fac, int k, int d, double* sums,
                        double* counts, hipStream_t s) {
  int grid = int((int64_t(k) * d + k + kBlock - 1) / kBlock);
  if (grid > 8192) grid = 8192;
  TWTML_LAUNCH(k_km_sums_f64, dim3(grid), dim3(kBlock), 0, s, si, mx, fac, k, d, sums, counts);
}

// ---------------------------------------------------------------------------
// K10: StreamingKMeansModel.update (fp64): weights + per-cluster blend
// factors (one workgroup), centre blend (grid, elementwise), dying-cluster
// split (one workgroup), fp32 centre copy + norms (wave per centre).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_km_weights(double* weights, const double* counts, int k,
                                                     double decay, int points_unit, double* blend) {
  __shared__ double red_v[16];
  __shared__ double total;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  {
    double s = 0.0;
    for (int c = t; c < k; c += 1024) s += counts[c];
    s = wave_sum(s);
    if (lane == 0) red_v[w] = s;
    __syncthreads();
    if (t == 0) {
      double tot = 0.0;
      for (int q = 0; q < 16; ++q) tot += red_v[q];
      total = tot;
    }
    __syncthreads();
  }
  const double discount = points_unit ? pow(decay, total) : decay;
  for (int c = t; c < k; c += 1024) {
    const double cnt = counts[c];
    double wgt = weights[c] * discount;
    double lam = -1.0, a = 0.0;           // lam < 0: cluster untouched this batch
    if (cnt > 0.0) {
      const double upd = wgt + cnt;
      lam = cnt / (upd > 1e-16 ? upd : 1e-16);
      a = lam / cnt;
      wgt = upd;
    }
    weights[c] = wgt;
    blend[c] = lam;
    blend[k + c] = a;
  }
}

// c <- (1 - lam) c + (lam / n) sum   (BLAS.scal + BLAS.axpy order)
__global__ void k_km_blend(double* centers, const double* sums, const double* blend, int k, int d) {
  const int64_t total = int64_t(k) * d;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(i / d);
    const double lam = blend[c];
    if (lam >= 0.0) centers[i] = (1.0 - lam) * centers[i] + blend[k + c] * sums[i];
  }
}

__global__ __launch_bounds__(1024) void k_km_split(double* centers, double* weights, int k, int d) {
  __shared__ double red_v[2][16];
  __shared__ int red_i[2][16];
  __shared__ int sel[2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  {
    // dying-cluster check: argmax / argmin of the weights, first index on ties
    // (Scala maxBy/minBy) -- strided scan, then wave and block reductions
    double vmax = -DBL_MAX, vmin = DBL_MAX;
    int imax = 0x7fffffff, imin = 0x7fffffff;
    for (int c = t; c < k; c += 1024) {
      const double v = weights[c];
      if (v > vmax) { vmax = v; imax = c; }
      if (v < vmin) { vmin = v; imin = c; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double om = __shfl_xor(vmax, off, kWave), on = __shfl_xor(vmin, off, kWave);
      const int jm = __shfl_xor(imax, off, kWave), jn = __shfl_xor(imin, off, kWave);
      if (om > vmax || (om == vmax && jm < imax)) { vmax = om; imax = jm; }
      if (on < vmin || (on == vmin && jn < imin)) { vmin = on; imin = jn; }
    }
    if (lane == 0) { red_v[0][w] = vmax; red_i[0][w] = imax; red_v[1][w] = vmin; red_i[1][w] = imin; }
    __syncthreads();
    if (t == 0) {
      for (int q = 1; q < 16; ++q) {
        if (red_v[0][q] > red_v[0][0] || (red_v[0][q] == red_v[0][0] && red_i[0][q] < red_i[0][0])) {
          red_v[0][0] = red_v[0][q]; red_i[0][0] = red_i[0][q];
        }
        if (red_v[1][q] < red_v[1][0] || (red_v[1][q] == red_v[1][0] && red_i[1][q] < red_i[1][0])) {
          red_v[1][0] = red_v[1][q]; red_i[1][0] = red_i[1][q];
        }
      }
      sel[0] = red_i[0][0];
      sel[1] = red_i[1][0];
    }
    __syncthreads();
  }
  if (t == 0) {
    const int largest = sel[0], smallest = sel[1];
    const double maxw = weights[largest], minw = weights[smallest];
    if (minw < 1e-8 * maxw) {
      const double wv = (maxw + minw) / 2.0;
      weights[largest] = wv;
      weights[smallest] = wv;
      for (int j = 0; j < d; ++j) {
        const double x = centers[int64_t(largest) * d + j];
        const double pp = 1e-14 * (fabs(x) > 1.0 ? fabs(x) : 1.0);
        centers[int64_t(largest) * d + j] = x + pp;
        centers[int64_t(smallest) * d + j] = x - pp;
      }
    }
  }
}

// wave per centre: fp32 copy (row padded to dp) + squared norm
__global__ __launch_bounds__(kBlock) void k_km_centers32(const double* centers, int k, int d, int dp,
                                                         float* c32, float* cnorm) {
  const int lane = lane_id();
  for (int64_t c = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; c < k;
       c += int64_t(gridDim.x) * (kBlock / kWave)) {
    float nrm = 0.f;
    for (int j = lane; j < dp; j += kWave) {
      const float v = j < d ? float(centers[c * d + j]) : 0.f;
      c32[c * dp + j] = v;
      nrm += v * v;
    }
    nrm = wave_sum(nrm);
    if (lane == 0) cnorm[c] = nrm;
  }
}

void launch_km_centers32(const double* centers, int k, int d, int dp, float* c32, float* cnorm,
                         hipStream_t s) {
  int grid = (k + 3) / 4;
  if (grid > 4096) grid = 4096;
  TWTML_LAUNCH(k_km_centers32, dim3(grid), dim3(kBlock), 0, s, centers, k, d, dp, c32, cnorm);
}

void launch_km_update(double* centers, double* weights, const double* sums, const double* counts,
                      int k, int d, double decay, bool points_unit, double* blend, float* c32,
                      float* cnorm, int dp, hipStream_t s) {
  TWTML_LAUNCH(k_km_weights, dim3(1), dim3(1024), 0, s, weights, counts, k, decay,
                     points_unit ? 1 : 0, blend);
  int grid = int((int64_t(k) * d + kBlock - 1) / kBlock);
  if (grid > 8192) grid = 8192;
  TWTML_LAUNCH(k_km_blend, dim3(grid), dim3(kBlock), 0, s, centers, sums, blend, k, d);
  TWTML_LAUNCH(k_km_split, dim3(1), dim3(1024), 0, s, centers, weights, k, d);
  launch_km_centers32(centers, k, d, dp, c32, cnorm, s);
}

}  // namespace twtml
