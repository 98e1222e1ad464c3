// Java/Python-compatible lower-casing of UTF-16 text (host side).
//
// The reference lower-cases every original tweet before hashing its
// bigrams (spark/.../MllibHelper.scala:43-45).  The GPU featurizer lowers
// per UTF-16 unit through a table; rows whose lowering is NOT per-unit
// (U+0130 expands to two units, U+03A3 depends on context, astral cased
// letters need the surrogate pair) are detected here and rewritten on the
// host before the batch leaves for the device.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace twtml {

// Simple per-unit lowercase of a BMP code unit (table driven).
uint16_t lower_unit(uint16_t c);

// True when lower_unit() applied per unit would NOT equal full lowering.
bool row_needs_special(const uint16_t* s, size_t n);

// Full lowering (Python str.lower / Java toLowerCase semantics) of one row.
void lower_full(const uint16_t* s, size_t n, std::vector<uint16_t>& out);

// Per-unit lowering (valid when !row_needs_special).
void lower_simple(const uint16_t* s, size_t n, uint16_t* out);

// Rewrite the special rows of a batch with their full lowering.  Rows that
// need no special handling are copied unchanged (the device lowers them).
// Returns the number of rewritten rows; out_text/out_offsets are resized.
size_t prelower_special_rows(const uint16_t* text, const int64_t* offsets, size_t nrows,
                             std::vector<uint16_t>& out_text, std::vector<int64_t>& out_offsets);

// Count special rows without rewriting (fast scan).
size_t count_special_rows(const uint16_t* text, const int64_t* offsets, size_t nrows);

}  // namespace twtml
