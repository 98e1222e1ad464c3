// CPU bigram featurizer (K1 on the host) for the local[N] engine.
//
// Same output as the fp64 oracle (oracle/featurize.py) but in C++: for each
// kept row, lower-case (unicode_lower), take text.sliding(2) over UTF-16
// units and hash each term (Java String.hashCode or Spark-2 murmur3), mod F.
// Duplicates are kept; the Python side sums them into CSR counts.
#include "../common/host_threads.h"
#include "featurize_cpu.h"

#include <algorithm>
#include <thread>
#include <vector>

#include "unicode_lower.h"

namespace twtml {

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t mix_k1(uint32_t k1) { return rotl32(k1 * 0xCC9E2D51u, 15) * 0x1B873593u; }
static inline uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  return rotl32(h1 ^ k1, 13) * 5u + 0xE6546B64u;
}
static inline uint32_t fmix(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16; h1 *= 0x85EBCA6Bu; h1 ^= h1 >> 13; h1 *= 0xC2B2AE35u; h1 ^= h1 >> 16;
  return h1;
}

int32_t murmur3_spark(const uint8_t* b, int n, uint32_t seed) {
  uint32_t h1 = seed;
  const int aligned = n - n % 4;
  for (int i = 0; i < aligned; i += 4) {
    const uint32_t k = uint32_t(b[i]) | (uint32_t(b[i + 1]) << 8) | (uint32_t(b[i + 2]) << 16) |
                       (uint32_t(b[i + 3]) << 24);
    h1 = mix_h1(h1, mix_k1(k));
  }
  for (int i = aligned; i < n; ++i) h1 = mix_h1(h1, mix_k1(uint32_t(int32_t(int8_t(b[i])))));
  return int32_t(fmix(h1, uint32_t(n)));
}

// UTF-8 bytes of a 1- or 2-unit Java string (lone surrogate -> '?').
static int term_utf8(const uint16_t* u, int n, uint8_t* out) {
  int k = 0;
  auto put = [&](uint32_t cp) {
    if (cp < 0x80) out[k++] = uint8_t(cp);
    else if (cp < 0x800) { out[k++] = uint8_t(0xC0 | (cp >> 6)); out[k++] = uint8_t(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out[k++] = uint8_t(0xE0 | (cp >> 12)); out[k++] = uint8_t(0x80 | ((cp >> 6) & 0x3F));
      out[k++] = uint8_t(0x80 | (cp & 0x3F));
    } else {
      out[k++] = uint8_t(0xF0 | (cp >> 18)); out[k++] = uint8_t(0x80 | ((cp >> 12) & 0x3F));
      out[k++] = uint8_t(0x80 | ((cp >> 6) & 0x3F)); out[k++] = uint8_t(0x80 | (cp & 0x3F));
    }
  };
  for (int i = 0; i < n; ++i) {
    const uint16_t c = u[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && u[i + 1] >= 0xDC00 && u[i + 1] <= 0xDFFF) {
      put(0x10000u + ((uint32_t(c) - 0xD800u) << 10) + (uint32_t(u[i + 1]) - 0xDC00u));
      ++i;
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      put('?');
    } else {
      put(c);
    }
  }
  return k;
}

int64_t term_index(const uint16_t* u, int n, int64_t F, int hash_kind) {
  int64_t h;
  if (hash_kind == 0) {
    int32_t j = 0;
    for (int i = 0; i < n; ++i) j = int32_t(uint32_t(j) * 31u + u[i]);
    h = j;
  } else {
    uint8_t buf[16];
    const int k = term_utf8(u, n, buf);
    h = murmur3_spark(buf, k, 42u);
  }
  int64_t m = h % F;
  return m < 0 ? m + F : m;
}

void featurize_rows_cpu(const uint16_t* text, const int64_t* offsets, const int64_t* rows,
                        size_t nrows, int64_t F, int hash_kind, std::vector<int64_t>& indptr,
                        std::vector<int64_t>& indices, int nthreads) {
  indptr.assign(nrows + 1, 0);
  int T = nthreads > 0 ? nthreads : host_threads();
  T = std::max(1, std::min<int>(T, int((nrows + 1023) / 1024)));
  std::vector<std::vector<int64_t>> part(T);
  std::vector<size_t> r0(T + 1);
  for (int t = 0; t <= T; ++t) r0[t] = nrows * size_t(t) / size_t(T);
  auto work = [&](int t) {
    std::vector<uint16_t> low;
    for (size_t i = r0[t]; i < r0[t + 1]; ++i) {
      const int64_t r = rows[i];
      const uint16_t* s = text + offsets[r];
      const size_t n = size_t(offsets[r + 1] - offsets[r]);
      low.clear();
      if (row_needs_special(s, n)) {
        lower_full(s, n, low);
      } else {
        low.resize(n);
        lower_simple(s, n, low.data());
      }
      const size_t m = low.size();
      auto& out = part[t];
      if (m >= 2) {
        for (size_t j = 0; j + 1 < m; ++j) out.push_back(term_index(&low[j], 2, F, hash_kind));
      } else if (m == 1) {
        out.push_back(term_index(&low[0], 1, F, hash_kind));
      }
      indptr[i + 1] = int64_t(out.size());
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  size_t total = 0;
  for (int t = 0; t < T; ++t) {
    for (size_t i = r0[t]; i < r0[t + 1]; ++i) indptr[i + 1] += int64_t(total);
    total += part[t].size();
  }
  indices.resize(total);
  size_t pos = 0;
  for (int t = 0; t < T; ++t) {
    std::copy(part[t].begin(), part[t].end(), indices.begin() + pos);
    pos += part[t].size();
  }
}

}  // namespace twtml
