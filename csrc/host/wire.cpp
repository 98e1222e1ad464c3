#include "../common/host_threads.h"
#include "wire.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

namespace twtml {

namespace {

// Encoding of a row and its wire bytes.
uint8_t row_kind(const uint16_t* t, int64_t len, int64_t* bytes) {
  uint16_t acc = 0;
  for (int64_t i = 0; i < len; ++i) acc |= t[i];
  if (acc < 256) {
    *bytes = len;
    return 0;
  }
  int64_t c = 0;
  for (int64_t i = 0; i < len; ++i) c += cesu_len(t[i]);
  if (c < 2 * len) {
    *bytes = c;
    return kWireCesu;
  }
  *bytes = 2 * len;
  return kWireWide;
}

template <typename F>
void parallel_chunks(int64_t n, int threads, F&& fn) {
  if (threads <= 0) threads = std::min(16, host_threads());
  const int64_t min_rows = 16384;
  int T = int(std::min<int64_t>(std::min(threads, 64), (n + min_rows - 1) / min_rows));
  if (T < 1) T = 1;
  std::vector<std::thread> pool;
  for (int c = 1; c < T; ++c) pool.emplace_back([&, c] { fn(c, T); });
  fn(0, T);
  for (auto& th : pool) th.join();
}

}  // namespace

int64_t wire_pack(const uint16_t* text, const int64_t* offsets, const uint8_t* is_rt, int64_t n,
                  uint8_t* out, int64_t out_cap, int64_t* out_offsets, uint8_t* flags, int threads) {
  out_offsets[0] = 0;
  if (n <= 0) return 0;
  // Pass 1: encoding per row, chunk-local byte offsets; pass 2: globalise + copy.
  // Wide rows need no alignment (the device assembles units from byte pairs).
  std::vector<int64_t> chunk_bytes(64 + 1, 0);
  int used = 1;
  parallel_chunks(n, threads, [&](int c, int T) {
    used = T;
    const int64_t r0 = n * c / T, r1 = n * (c + 1) / T;
    int64_t pos = 0;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t len = offsets[r + 1] - offsets[r];
      int64_t nb = 0;
      const uint8_t kind = row_kind(text + offsets[r], len, &nb);
      flags[r] = uint8_t((is_rt[r] ? kWireRetweet : 0) | kind);
      out_offsets[r + 1] = pos + nb;   // chunk-local end
      pos = out_offsets[r + 1];
    }
    chunk_bytes[size_t(c) + 1] = pos;
  });
  for (int c = 0; c < used; ++c) chunk_bytes[size_t(c) + 1] += chunk_bytes[size_t(c)];
  const int64_t total = chunk_bytes[size_t(used)];
  if (total > out_cap) throw std::length_error("wire_pack: output buffer too small");
  parallel_chunks(n, threads, [&](int c, int T) {
    const int64_t r0 = n * c / T, r1 = n * (c + 1) / T;
    const int64_t base = chunk_bytes[size_t(c)];
    for (int64_t r = r0; r < r1; ++r) out_offsets[r + 1] += base;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t o = r == r0 ? base : out_offsets[r];
      const uint16_t* src = text + offsets[r];
      const int64_t len = offsets[r + 1] - offsets[r];
      uint8_t* dst = out + o;
      if (flags[r] & kWireWide) {
        for (int64_t i = 0; i < len; ++i) {
          dst[2 * i] = uint8_t(src[i] & 0xFF);
          dst[2 * i + 1] = uint8_t(src[i] >> 8);
        }
      } else if (flags[r] & kWireCesu) {
        for (int64_t i = 0; i < len; ++i) {
          const uint32_t u = src[i];
          if (u < 0x80) {
            *dst++ = uint8_t(u);
          } else if (u < 0x800) {
            *dst++ = uint8_t(0xC0 | (u >> 6));
            *dst++ = uint8_t(0x80 | (u & 0x3F));
          } else {
            *dst++ = uint8_t(0xE0 | (u >> 12));
            *dst++ = uint8_t(0x80 | ((u >> 6) & 0x3F));
            *dst++ = uint8_t(0x80 | (u & 0x3F));
          }
        }
      } else {
        for (int64_t i = 0; i < len; ++i) dst[i] = uint8_t(src[i]);
      }
    }
  });
  return total;
}

namespace {
int64_t row_units(const uint8_t* w, int64_t nb, uint8_t fl) {
  if (fl & kWireWide) return nb >> 1;
  if (!(fl & kWireCesu)) return nb;
  int64_t u = 0;
  for (int64_t i = 0; i < nb; ++i) u += (w[i] & 0xC0) != 0x80;
  return u;
}
}  // namespace

int64_t wire_units(const uint8_t* wire, const int64_t* woff, const uint8_t* flags, int64_t n) {
  int64_t u = 0;
  for (int64_t r = 0; r < n; ++r) u += row_units(wire + woff[r], woff[r + 1] - woff[r], flags[r]);
  return u;
}

void wire_unpack(const uint8_t* wire, const int64_t* woff, const uint8_t* flags, int64_t n,
                 uint16_t* text, int64_t* offsets, uint8_t* is_rt) {
  offsets[0] = 0;
  for (int64_t r = 0; r < n; ++r) {
    const uint8_t fl = flags[r];
    const int64_t nb = woff[r + 1] - woff[r];
    const uint8_t* src = wire + woff[r];
    uint16_t* dst = text + offsets[r];
    int64_t len = 0;
    if (fl & kWireWide) {
      len = nb >> 1;
      for (int64_t i = 0; i < len; ++i) dst[i] = uint16_t(src[2 * i] | (uint16_t(src[2 * i + 1]) << 8));
    } else if (fl & kWireCesu) {
      for (int64_t i = 0; i < nb;) {
        const uint32_t b0 = src[i];
        uint32_t u;
        if (b0 < 0x80) {
          u = b0;
          i += 1;
        } else if (b0 < 0xE0) {
          u = ((b0 & 0x1F) << 6) | (src[i + 1] & 0x3F);
          i += 2;
        } else {
          u = ((b0 & 0x0F) << 12) | ((src[i + 1] & 0x3F) << 6) | (src[i + 2] & 0x3F);
          i += 3;
        }
        dst[len++] = uint16_t(u);
      }
    } else {
      len = nb;
      for (int64_t i = 0; i < len; ++i) dst[i] = src[i];
    }
    offsets[r + 1] = offsets[r] + len;
    is_rt[r] = fl & kWireRetweet;
  }
}

namespace {
inline bool hi_sur(uint32_t u) { return u >= 0xD800u && u <= 0xDBFFu; }
inline bool lo_sur(uint32_t u) { return u >= 0xDC00u && u <= 0xDFFFu; }

// Encodes one row; out == nullptr only counts.
int64_t utf8_row(const uint16_t* t, int64_t len, uint8_t* out) {
  int64_t b = 0;
  for (int64_t i = 0; i < len; ++i) {
    const uint32_t u = t[i];
    if (u < 0x80u) {
      if (out) out[b] = uint8_t(u);
      b += 1;
    } else if (u < 0x800u) {
      if (out) {
        out[b] = uint8_t(0xC0u | (u >> 6));
        out[b + 1] = uint8_t(0x80u | (u & 0x3Fu));
      }
      b += 2;
    } else if (hi_sur(u) && i + 1 < len && lo_sur(t[i + 1])) {
      const uint32_t cp = 0x10000u + ((u - 0xD800u) << 10) + (uint32_t(t[i + 1]) - 0xDC00u);
      if (out) {
        out[b] = uint8_t(0xF0u | (cp >> 18));
        out[b + 1] = uint8_t(0x80u | ((cp >> 12) & 0x3Fu));
        out[b + 2] = uint8_t(0x80u | ((cp >> 6) & 0x3Fu));
        out[b + 3] = uint8_t(0x80u | (cp & 0x3Fu));
      }
      b += 4;
      ++i;
    } else {
      if (out) {
        out[b] = uint8_t(0xE0u | (u >> 12));
        out[b + 1] = uint8_t(0x80u | ((u >> 6) & 0x3Fu));
        out[b + 2] = uint8_t(0x80u | (u & 0x3Fu));
      }
      b += 3;
    }
  }
  return b;
}
}  // namespace

int64_t utf8_encode(const uint16_t* text, const int64_t* offsets, int64_t n, uint8_t* out, int64_t out_cap,
                    int64_t* out_offsets, int threads) {
  out_offsets[0] = 0;
  if (n <= 0) return 0;
  std::vector<int64_t> chunk_bytes(64 + 1, 0);
  int used = 1;
  parallel_chunks(n, threads, [&](int c, int T) {
    used = T;
    const int64_t r0 = n * c / T, r1 = n * (c + 1) / T;
    int64_t pos = 0;
    for (int64_t r = r0; r < r1; ++r) {
      pos += utf8_row(text + offsets[r], offsets[r + 1] - offsets[r], nullptr);
      out_offsets[r + 1] = pos;   // chunk-local end
    }
    chunk_bytes[size_t(c) + 1] = pos;
  });
  for (int c = 0; c < used; ++c) chunk_bytes[size_t(c) + 1] += chunk_bytes[size_t(c)];
  const int64_t total = chunk_bytes[size_t(used)];
  if (total > out_cap) throw std::length_error("utf8_encode: output buffer too small");
  parallel_chunks(n, threads, [&](int c, int T) {
    const int64_t r0 = n * c / T, r1 = n * (c + 1) / T;
    const int64_t base = chunk_bytes[size_t(c)];
    for (int64_t r = r0; r < r1; ++r) out_offsets[r + 1] += base;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t o = r == r0 ? base : out_offsets[r];
      utf8_row(text + offsets[r], offsets[r + 1] - offsets[r], out + o);
    }
  });
  return total;
}

}  // namespace twtml
