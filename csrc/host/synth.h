// Synthetic tweet source (the stand-in for the Twitter sample stream).
//
// The reference ingests the live statuses/sample stream through
// TwitterUtils.createStream (spark/.../LinearRegression.scala:44); that API
// no longer exists, so the engine generates tweet-shaped records
//  deterministically from (seed, record index): any
// slice of the stream can be regenerated on any thread or rank, which makes
// multi-threaded generation and DP sharding reproducible.
#pragma once
#include <cstddef>
#include <cstdint>

namespace twtml {

struct SynthParams {
  uint64_t seed = 1;
  double retweet_fraction = 0.6;   // P(isRetweet)
  int64_t rt_lo = 0;               // clamp range of the original's retweet count
  int64_t rt_hi = 100000;
  double rt_base = 150.0;          // retweet_count = base + slope*log10(1+followers)
  double rt_slope = 90.0;          //                 + keyword score + N(0, noise)
  double rt_noise = 120.0;
  double rt_tail = 0.15;           // P(heavy-tail count: log-uniform up to rt_hi)
  int32_t min_len = 20;            // text length in UTF-16 units
  int32_t max_len = 280;
  double unicode_fraction = 0.08;  // P(tweet contains non-ASCII words/emoji)
  double special_fraction = 0.002; // P(tweet contains U+0130 / U+03A3 edge cases)
  int64_t now_ms = 1700000000000LL;
  int64_t max_age_ms = 7LL * 24 * 3600 * 1000;
  // 0: the ~300-word toy vocabulary (1.4K active bigrams per batch);
  // 1: a realistic multi-script vocabulary of `vocab_size` generated words
  //    (Latin, accented Latin-1, Cyrillic, Greek, CJK, kana, Hangul, Arabic,
  //    Devanagari, Thai, Hebrew) plus fresh @handles, hashtags and URL slugs
  int32_t vocab = 0;
  int32_t vocab_size = 50000;
};

// Generate rows [start, start+n) of the stream into caller buffers.
// text_cap is the capacity of `text` in units; returns the number of units
// written, or -(needed) if the capacity is too small (nothing valid then).
// offsets has n+1 entries (offsets[0] = 0), is_rt n, scalars 5*n (row-major
// [field][n]: retweet_count, followers, favourites, friends, created_at_ms).
int64_t synth_generate(const SynthParams& p, uint64_t start, size_t n, uint16_t* text,
                       size_t text_cap, int64_t* offsets, uint8_t* is_rt, int64_t* scalars,
                       int nthreads);

// Upper bound of units for n rows (max_len + slack per row).
size_t synth_max_units(const SynthParams& p, size_t n);

}  // namespace twtml
