// See unicode_lower.h.  Semantics follow CPython's str.lower (full case
// mapping + handle_capital_sigma), which is what the fp64 oracle uses; the
// tables in csrc/common/unicode_tables.h are derived from str.lower itself.
#include "unicode_lower.h"

#include <algorithm>

#include "../common/unicode_tables.h"

namespace twtml {

uint16_t lower_unit(uint16_t c) {
  if (c < 128) return (c >= 'A' && c <= 'Z') ? uint16_t(c + 32) : c;
  return uint16_t(c + uni::kLowerBlocks[uni::kLowerPage[c >> 8]][c & 0xFF]);
}

static inline bool is_high(uint16_t c) { return c >= 0xD800 && c <= 0xDBFF; }
static inline bool is_low(uint16_t c) { return c >= 0xDC00 && c <= 0xDFFF; }

static bool supp_high_has_mapping(uint16_t hi) {
  return std::binary_search(uni::kSuppHigh, uni::kSuppHigh + uni::kNumSuppHigh, hi);
}

bool row_needs_special(const uint16_t* s, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint16_t c = s[i];
    if (c < 0x130) continue;
    if (c == 0x0130 || c == 0x03A3) return true;
    if (is_high(c) && i + 1 < n && is_low(s[i + 1]) && supp_high_has_mapping(c)) return true;
  }
  return false;
}

static uint32_t lower_cp(uint32_t cp) {
  if (cp < 0x10000) return lower_unit(uint16_t(cp));
  int lo = 0, hi = uni::kNumSuppLower - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t k = uni::kSuppLower[mid][0];
    if (k == cp) return uni::kSuppLower[mid][1];
    if (k < cp) lo = mid + 1; else hi = mid - 1;
  }
  return cp;
}

// 0 = neither, 1 = case-ignorable, 2 = cased (and not case-ignorable)
static int case_class(uint32_t cp) {
  int lo = 0, hi = uni::kNumCaseRanges - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < uni::kCaseRanges[mid][0]) hi = mid - 1;
    else if (cp > uni::kCaseRanges[mid][1]) lo = mid + 1;
    else return int(uni::kCaseRanges[mid][2]);
  }
  return 0;
}

static void decode(const uint16_t* s, size_t n, std::vector<uint32_t>& cps) {
  cps.clear();
  for (size_t i = 0; i < n; ++i) {
    const uint16_t c = s[i];
    if (is_high(c) && i + 1 < n && is_low(s[i + 1])) {
      cps.push_back(0x10000u + ((uint32_t(c) - 0xD800u) << 10) + (uint32_t(s[i + 1]) - 0xDC00u));
      ++i;
    } else {
      cps.push_back(c);  // lone surrogates pass through as themselves
    }
  }
}

static void put_cp(uint32_t cp, std::vector<uint16_t>& out) {
  if (cp < 0x10000) {
    out.push_back(uint16_t(cp));
  } else {
    cp -= 0x10000;
    out.push_back(uint16_t(0xD800 + (cp >> 10)));
    out.push_back(uint16_t(0xDC00 + (cp & 0x3FF)));
  }
}

void lower_full(const uint16_t* s, size_t n, std::vector<uint16_t>& out) {
  thread_local std::vector<uint32_t> cps;
  decode(s, n, cps);
  const size_t m = cps.size();
  for (size_t i = 0; i < m; ++i) {
    const uint32_t c = cps[i];
    if (c == 0x0130) {             // LATIN CAPITAL LETTER I WITH DOT ABOVE -> "i̇"
      out.push_back(0x0069);
      out.push_back(0x0307);
    } else if (c == 0x03A3) {      // GREEK CAPITAL SIGMA: Final_Sigma context
      ptrdiff_t j = ptrdiff_t(i) - 1;
      int cls = 0;
      for (; j >= 0; --j) {
        cls = case_class(cps[j]);
        if (cls != 1) break;
      }
      bool final_sigma = j >= 0 && cls == 2;
      if (final_sigma && i + 1 < m) {
        size_t k = i + 1;
        int cls2 = 0;
        for (; k < m; ++k) {
          cls2 = case_class(cps[k]);
          if (cls2 != 1) break;
        }
        final_sigma = (k == m) || cls2 != 2;
      }
      out.push_back(final_sigma ? 0x03C2 : 0x03C3);
    } else {
      put_cp(lower_cp(c), out);
    }
  }
}

void lower_simple(const uint16_t* s, size_t n, uint16_t* out) {
  for (size_t i = 0; i < n; ++i) out[i] = lower_unit(s[i]);
}

size_t count_special_rows(const uint16_t* text, const int64_t* offsets, size_t nrows) {
  size_t cnt = 0;
  for (size_t r = 0; r < nrows; ++r)
    cnt += row_needs_special(text + offsets[r], size_t(offsets[r + 1] - offsets[r])) ? 1 : 0;
  return cnt;
}

size_t prelower_special_rows(const uint16_t* text, const int64_t* offsets, size_t nrows,
                             std::vector<uint16_t>& out_text, std::vector<int64_t>& out_offsets) {
  out_text.clear();
  out_offsets.assign(nrows + 1, 0);
  out_text.reserve(size_t(offsets[nrows]) + 16);
  size_t changed = 0;
  for (size_t r = 0; r < nrows; ++r) {
    const uint16_t* s = text + offsets[r];
    const size_t n = size_t(offsets[r + 1] - offsets[r]);
    if (row_needs_special(s, n)) {
      lower_full(s, n, out_text);
      ++changed;
    } else {
      out_text.insert(out_text.end(), s, s + n);
    }
    out_offsets[r + 1] = int64_t(out_text.size());
  }
  return changed;
}

}  // namespace twtml
