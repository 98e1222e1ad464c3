// Launchers of the streaming k-means kernels (kmeans.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace twtml {

void launch_km_features(const DevRawBatch& b, const int64_t* kept, const int64_t* counters,
                        float* X, int dp, int text_dims, const uint8_t* lpage,
                        const uint16_t* lblocks, int64_t max_rows, hipStream_t s);
// Exact integer scaler moments (kmeans.hip K11): column max |x| (atomic max
// into mx[d], all-reduced MAX), then n and per column sum q, sum a^2, sum 2ab,
// sum b^2 of the quantized features q = rint(x 2^-s), s = km_quant_shift(mx)
// (out[1 + 4 d], all-reduced SUM).  X itself stays unscaled; the factors are
// computed on the host and every consumer multiplies on load.
constexpr int kKmQBits = 30;   // |q| <= 2^30: every int64 sum / limb fits any batch
int km_quant_shift(int64_t mx);
void launch_km_colmax(const float* X, const int64_t* counters, int d, int dp, int64_t* mx, int64_t max_rows,
                      hipStream_t s);
void launch_km_moments_q(const float* X, const int64_t* counters, int d, int dp, const int64_t* mx,
                         int64_t* out, int64_t max_rows, hipStream_t s);
// MFMA (bf16x3 or fp32) or scalar argmin; near-ties re-decided in fp64
// against `centers` (refine: scratch of 6 * max_rows ints; refine_cnt: 2
// device counters; frag / cnp: bf16x3 scratch of km_frag_elems(k, dp) u16 and
// round_up(k, 32) floats)
void launch_km_assign(const float* X, const float* f32, const double* f64, const int64_t* counters,
                      const float* C, const float* cnorm, const double* centers, int k, int d, int dp,
                      int32_t* labels, int32_t* refine, unsigned long long* refine_cnt,
                      uint16_t* frag, float* cnp, int64_t max_rows, bool mfma, bool bf16,
                      hipStream_t s);
inline size_t km_frag_elems(int k, int dp) { return size_t((k + 31) / 32) * 32 * size_t(dp) * 2; }
// per-cluster int64 sums of q ([k][d]) then counts ([k]) into sums[k d + k]
void launch_km_cluster_sums(const float* X, const int64_t* mx, const int32_t* labels,
                            const int64_t* counters, int k,
                            int d, int dp, int64_t* hist, int32_t* order, int64_t* sums,
                            int64_t max_rows, hipStream_t s,
                            void (*scan)(const int64_t*, int64_t*, int64_t, int64_t*, hipStream_t));
// all-reduced integer sums -> fp64 sums of the scaled features + counts
void launch_km_sums_f64(const int64_t* si, const int64_t* mx, const double* fac, int k, int d, double* sums,
                        double* counts, hipStream_t s);
void launch_km_update(double* centers, double* weights, const double* sums, const double* counts,
                      int k, int d, double decay, bool points_unit, double* blend, float* c32,
                      float* cnorm, int dp, hipStream_t s);
void launch_km_centers32(const double* centers, int k, int d, int dp, float* c32, float* cnorm,
                         hipStream_t s);

// from featurize.hip
void launch_filter_only(const DevRawBatch& b, const DevPrepared& p, const FeaturizeParams& fp,
                        hipStream_t s);
void scan_excl_launch(const int64_t* in, int64_t* out, int64_t n, int64_t* total, hipStream_t s);

}  // namespace twtml
