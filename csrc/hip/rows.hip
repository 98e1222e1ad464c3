// Row normalisation of a raw batch on the device, before the filter:
//
//   * full case mapping of the rows whose lower-casing is not one UTF-16
//     unit per unit (U+0130 -> "i" U+0307, Greek capital sigma with the
//     Final_Sigma context, astral cased letters), i.e. Java's / Python's
//     String.toLowerCase as MllibHelper.featurizeText applies it
//     (spark/src/main/scala/com/giorgioinf/twtml/spark/MllibHelper.scala:45).
//     Every other unit is lowered per unit by the featurizer, and lowering is
//     idempotent, so only these rows are rewritten here (to their lowered
//     UTF-16 text; the featurizer's per-unit pass leaves it unchanged).
//   * UTF-16 batches (raw ingest, no host packing): rows whose units are all
//     < 256 are narrowed to one byte per unit so the featurizer's Latin-1
//     fast path (and the lazy-id remap) takes them.
//
// One wave per 64 rows; lane l owns row l's extents, and the wave walks the
// wide rows among them (ballot) together, 64 units per step.  Rewritten rows
// are relocated (their start / end are written to out_s / out_e, the text
// stays where it is):
//   narrowed row with wire bytes [o, e)  -> tail + 2 o        (<= (e - o) / 2 bytes)
//   lowered special row                  -> lower_base + 2 o  (<= 2 (e - o) bytes:
//       a unit that grows (U+0130, 2 units) takes 2 wire bytes in every
//       encoding, every other unit keeps one unit)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "../common/unicode_tables.h"
#include "common.h"
#include "kernels.h"

namespace twtml {

namespace {

__device__ __forceinline__ bool is_high(uint32_t u) { return u >= 0xD800u && u <= 0xDBFFu; }
__device__ __forceinline__ bool is_low(uint32_t u) { return u >= 0xDC00u && u <= 0xDFFFu; }

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int32_t(uint32_t(v)), l));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int32_t(uint32_t(uint64_t(v) >> 32)), l));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// High surrogates of the astral code points that have a lower-case mapping
// (uni::kSuppHigh: Deseret, Osage, Old Hungarian, Warang Citi, Medefaidrin, Adlam).
__device__ __forceinline__ bool supp_high_mapped(uint32_t u) {
  return u == 0xD801u || u == 0xD803u || u == 0xD806u || u == 0xD81Bu || u == 0xD83Au;
}

struct RowNorm {
  uint8_t* text;
  const int64_t* wire_off;   // [n + 1] wire byte offsets (relocation regions)
  const int64_t* cur_s;      // current extents (cesu rows already expanded)
  const int64_t* cur_e;
  uint8_t* flags;
  int64_t* out_s;
  int64_t* out_e;
  int64_t n;
  int64_t tail, lower_base;
  int32_t narrow;
  int32_t flagged_only;      // scan only rows the decoder flagged kRowSpecial
  DevCaseTables ct;
  int64_t* stats;            // [0] lowered rows, [1] narrowed rows (nullable)
};

__device__ __forceinline__ uint32_t unit_at(const uint8_t* text, int64_t o, int64_t i) {
  const uint8_t* p = text + o + 2 * i;   // wide rows may start at any byte
  if ((o & 1) == 0) return *reinterpret_cast<const uint16_t*>(p);   // one load when aligned
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8);
}

constexpr int kScanRows = 8;   // wide rows whose pass-1 loads are in flight together

// 0 = neither, 1 = case-ignorable, 2 = cased (unicode_tables.h kCaseRanges):
// BMP code points from the 2-bit table (one load), astral ones by binary
// search of the ranges
__device__ int case_class(const DevCaseTables& ct, uint32_t cp) {
  if (cp < 0x10000u) return int((ct.bmp_class[cp >> 4] >> (2 * (cp & 15u))) & 3u);
  int lo = 0, hi = ct.n_ranges - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t* r = ct.case_ranges + 3 * mid;
    if (cp < r[0]) hi = mid - 1;
    else if (cp > r[1]) lo = mid + 1;
    else return int(r[2]);
  }
  return 0;
}

__device__ uint32_t lower_astral(const DevCaseTables& ct, uint32_t cp) {
  int lo = 0, hi = ct.n_supp - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t k = ct.supp_lower[2 * mid];
    if (k == cp) return ct.supp_lower[2 * mid + 1];
    if (k < cp) lo = mid + 1; else hi = mid - 1;
  }
  return cp;
}

// Final_Sigma (Unicode SpecialCasing): preceded by a cased letter (skipping
// case-ignorables) and not followed by one.
__device__ bool final_sigma(const RowNorm& a, int64_t o, int64_t len, int64_t i) {
  int64_t j = i - 1;
  int cls = 0;
  bool found = false;
  while (j >= 0) {
    const uint32_t u = unit_at(a.text, o, j);
    uint32_t cp = u;
    int64_t step = 1;
    if (is_low(u) && j > 0) {
      const uint32_t h = unit_at(a.text, o, j - 1);
      if (is_high(h)) { cp = 0x10000u + ((h - 0xD800u) << 10) + (u - 0xDC00u); step = 2; }
    }
    cls = case_class(a.ct, cp);
    if (cls != 1) { found = true; break; }
    j -= step;
  }
  if (!(found && cls == 2)) return false;
  int64_t k = i + 1;
  while (k < len) {
    const uint32_t u = unit_at(a.text, o, k);
    uint32_t cp = u;
    int64_t step = 1;
    if (is_high(u) && k + 1 < len) {
      const uint32_t l = unit_at(a.text, o, k + 1);
      if (is_low(l)) { cp = 0x10000u + ((u - 0xD800u) << 10) + (l - 0xDC00u); step = 2; }
    }
    const int c2 = case_class(a.ct, cp);
    if (c2 != 1) return c2 != 2;
    k += step;
  }
  return true;
}

// One wide row [o, o + 2 len) (wire offset w0) given its wave-reduced max
// unit bits `orv` and special test: narrowed (UTF-16 batches, every unit <
// 256) or fully lower-cased (special) into its relocation region, else kept.
// Wave-uniform arguments; every lane returns the same extents.
struct RowOut {
  int64_t s0, s1;
  bool narrowed, lowered;
};

__device__ __forceinline__ RowOut normalize_row(const RowNorm& a, int64_t o, int64_t len, int64_t w0, uint32_t orv,
                                                bool special) {
  const int lane = lane_id();
  const uint64_t below = (uint64_t(1) << lane) - 1;
  RowOut out{o, o + 2 * len, false, false};
  if (a.narrow && orv < 256u) {
    uint8_t* dst = a.text + a.tail + 2 * w0;
    for (int64_t i = lane; i < len; i += kWave) dst[i] = uint8_t(unit_at(a.text, o, i));
    out.s0 = a.tail + 2 * w0;
    out.s1 = out.s0 + len;
    out.narrowed = true;
  } else if (special) {
    uint16_t* dst = reinterpret_cast<uint16_t*>(a.text + a.lower_base + 2 * w0);
    int64_t k = 0;
    for (int64_t i0 = 0; i0 < len; i0 += kWave) {
      const int64_t i = i0 + lane;
      const bool valid = i < len;
      const uint32_t u = valid ? unit_at(a.text, o, i) : 0u;
      const bool two = valid && u == 0x130u;
      const uint64_t bm = __ballot(two);
      const int64_t pos = k + lane + __popcll(bm & below);
      if (valid) {
        if (two) {
          dst[pos] = 0x0069u;
          dst[pos + 1] = 0x0307u;
        } else if (u == 0x3A3u) {
          dst[pos] = final_sigma(a, o, len, i) ? 0x03C2u : 0x03C3u;
        } else if (is_high(u) && i + 1 < len && is_low(unit_at(a.text, o, i + 1))) {
          const uint32_t cp = 0x10000u + ((u - 0xD800u) << 10) + (unit_at(a.text, o, i + 1) - 0xDC00u);
          dst[pos] = uint16_t(0xD800u + ((lower_astral(a.ct, cp) - 0x10000u) >> 10));
        } else if (is_low(u) && i > 0 && is_high(unit_at(a.text, o, i - 1))) {
          const uint32_t cp = 0x10000u + ((unit_at(a.text, o, i - 1) - 0xD800u) << 10) + (u - 0xDC00u);
          dst[pos] = uint16_t(0xDC00u + ((lower_astral(a.ct, cp) - 0x10000u) & 0x3FFu));
        } else {
          dst[pos] = uint16_t(u);   // per-unit lowering: the featurizer
        }
      }
      k += std::min<int64_t>(kWave, len - i0) + __popcll(bm);
    }
    out.s0 = a.lower_base + 2 * w0;
    out.s1 = out.s0 + 2 * k;
    out.lowered = true;
  }
  return out;
}

// Special-unit test of unit i of a row (pass 1).
__device__ __forceinline__ bool special_unit(const uint8_t* text, int64_t o, int64_t len, int64_t i, uint32_t u) {
  bool sp = u == 0x130u || u == 0x3A3u;
  if (is_high(u) && i + 1 < len && supp_high_mapped(u)) sp |= is_low(unit_at(text, o, i + 1));
  return sp;
}

__global__ __launch_bounds__(256) void k_row_normalize(RowNorm a) {
  const int lane = lane_id();
  const int64_t wave = (int64_t(blockIdx.x) * 256 + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * 256 / kWave;
  for (int64_t g = wave; g * kWave < a.n; g += nwaves) {
    const int64_t r = g * kWave + lane;
    const bool in = r < a.n;
    uint8_t fl = in ? a.flags[r] : 0;
    int64_t s0 = in ? a.cur_s[r] : 0, s1 = in ? a.cur_e[r] : 0;
    const int64_t wo = in ? a.wire_off[r] : 0;
    uint64_t m = __ballot(in && (fl & kRowWide) && (!a.flagged_only || (fl & kRowSpecial)));
    fl = uint8_t(fl & ~kRowSpecial);
    int n_low = 0, n_nar = 0;
    while (m) {
      // pass 1 over up to kScanRows wide rows at once (their unit loads all
      // in flight together: one row at a time left this kernel latency-bound,
      // a memory round trip per row): max unit (narrowing) and special units
      int nr = 0;
      int ls[kScanRows];
      int64_t os[kScanRows], lens[kScanRows];
      int64_t lmax = 0;
#pragma unroll
      for (int q = 0; q < kScanRows; ++q) {
        ls[q] = -1;
        os[q] = 0;
        lens[q] = 0;
        if (m) {
          const int l = __builtin_ctzll(m);
          m &= m - 1;
          ls[q] = l;
          os[q] = readlane64(s0, l);
          lens[q] = (readlane64(s1, l) - os[q]) >> 1;
          lmax = std::max(lmax, lens[q]);
          ++nr;
        }
      }
      uint32_t orq[kScanRows];
      bool spq[kScanRows];
#pragma unroll
      for (int q = 0; q < kScanRows; ++q) {
        orq[q] = 0;
        spq[q] = false;
      }
      for (int64_t i0 = 0; i0 < lmax; i0 += kWave) {
        const int64_t i = i0 + lane;
        uint32_t u[kScanRows];
#pragma unroll
        for (int q = 0; q < kScanRows; ++q) u[q] = i < lens[q] ? unit_at(a.text, os[q], i) : 0u;
#pragma unroll
        for (int q = 0; q < kScanRows; ++q) {
          orq[q] |= u[q];
          spq[q] |= special_unit(a.text, os[q], lens[q], i, u[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < kScanRows; ++q) {
        if (q >= nr) break;   // wave-uniform; q is a constant after unrolling (no scratch arrays)
        const int l = ls[q];
        const RowOut ro = normalize_row(a, os[q], lens[q], readlane64(wo, l), wave_or(orq[q]), __any(spq[q]));
        n_nar += ro.narrowed ? 1 : 0;
        n_low += ro.lowered ? 1 : 0;
        if (lane == l) {
          s0 = ro.s0;
          s1 = ro.s1;
          if (ro.narrowed) fl = uint8_t(fl & ~kRowWide);
        }
      }
    }
    if (in) {
      a.out_s[r] = s0;
      a.out_e[r] = s1;
      a.flags[r] = fl;
    }
    if (a.stats && lane == 0 && (n_low | n_nar)) {
      if (n_low) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stats[0]), (unsigned long long)n_low);
      if (n_nar) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stats[1]), (unsigned long long)n_nar);
    }
  }
}

// The decoder's kRowSpecial rows (UTF-8 batches), one wave per listed row:
// every special row of the batch is walked at once.  (Walked by the wave of
// its 64-row group, k_row_normalize's flagged_only pass, a group's special
// rows ran one after another -- each Final_Sigma test a chain of dependent
// loads -- and the ~0.3 % of rows that are special set that kernel's span:
// ~115 us under overlap for ~42 MB of row extents it rewrote unchanged.)
__global__ __launch_bounds__(256) void k_row_special(RowNorm a, const int32_t* list) {
  const int lane = lane_id();
  const int64_t wave = (int64_t(blockIdx.x) * 256 + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * 256 / kWave;
  const int64_t cnt = a.stats[2] < a.n ? a.stats[2] : a.n;   // <= one entry per row
  int n_low = 0, n_nar = 0;
  for (int64_t j = wave; j < cnt; j += nwaves) {
    const int64_t r = list[j];
    if (r < 0 || r >= a.n) continue;   // the list holds row indices of this batch (wave-uniform)
    const int64_t o = a.cur_s[r], len = (a.cur_e[r] - o) >> 1, w0 = a.wire_off[r];
    uint32_t orq = 0;
    bool spq = false;
    for (int64_t i = lane; i < len; i += kWave) {
      const uint32_t u = unit_at(a.text, o, i);
      orq |= u;
      spq |= special_unit(a.text, o, len, i, u);
    }
    const RowOut ro = normalize_row(a, o, len, w0, wave_or(orq), __any(spq));
    n_nar += ro.narrowed ? 1 : 0;
    n_low += ro.lowered ? 1 : 0;
    if (lane == 0) {
      uint8_t fl = uint8_t(a.flags[r] & ~kRowSpecial);
      if (ro.narrowed) fl = uint8_t(fl & ~kRowWide);
      a.out_s[r] = ro.s0;
      a.out_e[r] = ro.s1;
      a.flags[r] = fl;
    }
  }
  if (lane == 0 && (n_low | n_nar)) {
    if (n_low) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stats[0]), (unsigned long long)n_low);
    if (n_nar) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stats[1]), (unsigned long long)n_nar);
  }
}

}  // namespace

// The class of a code point by binary search of kCaseRanges (the device
// lookup for astral code points, and the source of the BMP table).
static int host_case_class(uint32_t cp) {
  int lo = 0, hi = uni::kNumCaseRanges - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < uni::kCaseRanges[mid][0]) hi = mid - 1;
    else if (cp > uni::kCaseRanges[mid][1]) lo = mid + 1;
    else return int(uni::kCaseRanges[mid][2]);
  }
  return 0;
}

void upload_case_tables(DevCaseTables* ct) {
  uint32_t* sl = nullptr;
  uint32_t* cr = nullptr;
  uint32_t* bc = nullptr;
  std::vector<uint32_t> bmp(4096, 0u);
  for (uint32_t cp = 0; cp < 0x10000u; ++cp) bmp[cp >> 4] |= uint32_t(host_case_class(cp)) << (2 * (cp & 15u));
  TWTML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&sl), sizeof(uni::kSuppLower)));
  TWTML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&cr), sizeof(uni::kCaseRanges)));
  TWTML_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&bc), bmp.size() * sizeof(uint32_t)));
  TWTML_HIP_CHECK(hipMemcpy(sl, uni::kSuppLower, sizeof(uni::kSuppLower), hipMemcpyHostToDevice));
  TWTML_HIP_CHECK(hipMemcpy(cr, uni::kCaseRanges, sizeof(uni::kCaseRanges), hipMemcpyHostToDevice));
  TWTML_HIP_CHECK(hipMemcpy(bc, bmp.data(), bmp.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  TWTML_HIP_CHECK(hipDeviceSynchronize());   // landed before any engine stream reads them
  ct->supp_lower = sl;
  ct->case_ranges = cr;
  ct->bmp_class = bc;
  ct->n_supp = uni::kNumSuppLower;
  ct->n_ranges = uni::kNumCaseRanges;
}

void free_case_tables(DevCaseTables* ct) {
  if (ct->supp_lower) (void)hipFree(const_cast<uint32_t*>(ct->supp_lower));
  if (ct->case_ranges) (void)hipFree(const_cast<uint32_t*>(ct->case_ranges));
  if (ct->bmp_class) (void)hipFree(const_cast<uint32_t*>(ct->bmp_class));
  *ct = DevCaseTables{};
}

void launch_row_normalize(uint8_t* text, const int64_t* wire_off, const int64_t* cur_s, const int64_t* cur_e,
                          uint8_t* flags, int64_t* out_s, int64_t* out_e, int64_t n, int64_t tail,
                          int64_t lower_base, bool narrow, const DevCaseTables& ct, int64_t* stats,
                          hipStream_t s, bool flagged_only) {
  if (n <= 0) return;
  RowNorm a{text, wire_off, cur_s, cur_e, flags, out_s, out_e, n, tail, lower_base, narrow ? 1 : 0,
            flagged_only ? 1 : 0, ct, stats};
  const int grid = int(std::min<int64_t>((n + 255) / 256, 4096));
  TWTML_LAUNCH(k_row_normalize, dim3(grid), dim3(256), 0, s, a);
}

void launch_row_special(uint8_t* text, const int64_t* wire_off, int64_t* cur_s, int64_t* cur_e,
                        uint8_t* flags, const int32_t* special, int64_t n, int64_t tail, int64_t lower_base,
                        const DevCaseTables& ct, int64_t* stats, hipStream_t s) {
  if (n <= 0) return;
  RowNorm a{text, wire_off, cur_s, cur_e, flags, cur_s, cur_e, n, tail, lower_base, 1, 1, ct, stats};
  // the list length is on the device: a grid of up to 4096 waves (one row
  // each for the ~3K special rows of a wide 1M-row batch), the rest stride
  const int grid = int(std::min<int64_t>((n + 255) / 256, 1024));
  TWTML_LAUNCH(k_row_special, dim3(grid), dim3(256), 0, s, a, special);
}

}  // namespace twtml
