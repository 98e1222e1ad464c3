// Launchers of the streaming k-means kernels (kmeans.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace twtml {

void launch_km_features(const DevRawBatch& b, const int64_t* kept, const int64_t* counters,
                        float* X, int dp, int text_dims, const uint8_t* lpage,
                        const uint16_t* lblocks, int64_t max_rows, hipStream_t s);
void launch_km_moments(const float* X, const int64_t* counters, int d, int dp, int mode,
                       const double* sum_n, double* out, int64_t max_rows, hipStream_t s);
// scaler factors (X itself stays unscaled; consumers multiply on load)
void launch_km_factor(int d, int dp, bool scale, const double* sum_n, const double* m2,
                      double* std_out, double* f64, float* f32, hipStream_t s);
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
void launch_km_cluster_sums(const float* X, const double* f64, const int32_t* labels,
                            const int64_t* counters, int k,
                            int d, int dp, int64_t* hist, int32_t* order, double* sums,
                            double* counts, int64_t max_rows, hipStream_t s,
                            void (*scan)(const int64_t*, int64_t*, int64_t, int64_t*, hipStream_t));
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
