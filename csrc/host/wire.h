// Compact host->device wire format of a raw tweet batch.
//
// PCIe is the bound once the GPU pipeline is fast (a 1M-tweet batch is ~280 MB
// as UTF-16), and most tweet text is Latin-1.  Each row is stored as one of
//   narrow  1 byte per UTF-16 unit (every unit < 256)
//   cesu    every UTF-16 *unit* as 1-3 UTF-8-style bytes (< 0x80: 1, < 0x800:
//           2, else 3 -- surrogates encoded one by one, CESU-8 style, so any
//           unit sequence, lone surrogates included, round-trips exactly);
//           chosen when smaller than UTF-16 (mostly-ASCII text with a few
//           non-Latin-1 characters: ~0.6 of the UTF-16 bytes on tweets)
//   wide    UTF-16LE, 2 bytes per unit, any alignment
// The device expands cesu rows to wide ones after the H2D.  Per-row flags
// byte: bit0 = isRetweet, bit1 = wide, bit2 = cesu.  Offsets are byte
// offsets [n+1].
#pragma once
#include <cstdint>

namespace twtml {

constexpr uint8_t kWireRetweet = 1;
constexpr uint8_t kWireWide = 2;
constexpr uint8_t kWireCesu = 4;

// Bytes of one UTF-16 unit in the cesu encoding.
inline int cesu_len(uint16_t u) { return u < 0x80 ? 1 : (u < 0x800 ? 2 : 3); }

// Upper bound of the packed size for `units` UTF-16 units in `rows` rows
// (a row is cesu only when that is smaller than its UTF-16 bytes).
inline int64_t wire_bound(int64_t units, int64_t rows) { (void)rows; return 2 * units + 64; }

// Packs rows [0, n); returns the total byte count.  `threads` <= 0: auto.
int64_t wire_pack(const uint16_t* text, const int64_t* offsets, const uint8_t* is_rt, int64_t n,
                  uint8_t* out, int64_t out_cap, int64_t* out_offsets, uint8_t* flags, int threads);

// Inverse (tests / debugging): unit offsets + UTF-16 text.
void wire_unpack(const uint8_t* wire, const int64_t* woff, const uint8_t* flags, int64_t n,
                 uint16_t* text, int64_t* offsets, uint8_t* is_rt);

// Total UTF-16 units of a packed batch.
int64_t wire_units(const uint8_t* wire, const int64_t* woff, const uint8_t* flags, int64_t n);

// UTF-16 -> UTF-8 (what a network receiver holds: tweet JSON is UTF-8).
// Surrogate pairs become 4-byte sequences; a lone surrogate is encoded as a
// 3-byte sequence (WTF-8), so every unit sequence round-trips exactly through
// the device decoder.  Two passes over row chunks (`threads` <= 0: auto);
// out needs utf8_bound(units) bytes, out_offsets [n+1] byte offsets.
inline int64_t utf8_bound(int64_t units) { return 3 * units + 64; }
int64_t utf8_encode(const uint16_t* text, const int64_t* offsets, int64_t n, uint8_t* out, int64_t out_cap,
                    int64_t* out_offsets, int threads);

}  // namespace twtml
