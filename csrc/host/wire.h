// Compact host->device wire format of a raw tweet batch.
//
// PCIe is the bound once the GPU pipeline is fast (a 1M-tweet batch is ~280 MB
// as UTF-16), and most tweet text is Latin-1.  Each row is stored either
// narrow (1 byte per UTF-16 unit, every unit < 256) or wide (UTF-16LE, 2
// bytes per unit, any alignment).  Per-row flags byte: bit0 = isRetweet,
// bit1 = wide.  Offsets are byte offsets [n+1]; a row has
// (off[r+1] - off[r]) >> wide units.
#pragma once
#include <cstdint>

namespace twtml {

constexpr uint8_t kWireRetweet = 1;
constexpr uint8_t kWireWide = 2;

// Upper bound of the packed size for `units` UTF-16 units in `rows` rows.
inline int64_t wire_bound(int64_t units, int64_t rows) { (void)rows; return 2 * units + 64; }

// Packs rows [0, n); returns the total byte count.  `threads` <= 0: auto.
int64_t wire_pack(const uint16_t* text, const int64_t* offsets, const uint8_t* is_rt, int64_t n,
                  uint8_t* out, int64_t out_cap, int64_t* out_offsets, uint8_t* flags, int threads);

// Inverse (tests / debugging): unit offsets + UTF-16 text.
void wire_unpack(const uint8_t* wire, const int64_t* woff, const uint8_t* flags, int64_t n,
                 uint16_t* text, int64_t* offsets, uint8_t* is_rt);

// Total UTF-16 units of a packed batch.
int64_t wire_units(const int64_t* woff, const uint8_t* flags, int64_t n);

}  // namespace twtml
