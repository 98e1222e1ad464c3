#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace twtml {

// Spark 2.x Murmur3_x86_32.hashUnsafeBytes (signed result).
int32_t murmur3_spark(const uint8_t* b, int n, uint32_t seed);

// Index of a 1- or 2-unit term: hash_kind 0 = Java hashCode, 1 = murmur3.
int64_t term_index(const uint16_t* u, int n, int64_t F, int hash_kind);

// Bigram hash indices (duplicates kept) of rows[] of a ragged UTF-16 batch.
void featurize_rows_cpu(const uint16_t* text, const int64_t* offsets, const int64_t* rows,
                        size_t nrows, int64_t F, int hash_kind, std::vector<int64_t>& indptr,
                        std::vector<int64_t>& indices, int nthreads);

}  // namespace twtml
