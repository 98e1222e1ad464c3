// Streaming k-means on MI355X (KMeans.scala:100-113).
//
// Per micro-batch:
//   K3'  filter isRetweet, K1' features x = [retweetCount, followers, hashed
//        bigram counts (text_dims)] as dense fp32 rows (width padded to DP)
//   K11  StandardScaler(withMean=false, withStd=true): two-pass column
//        moments in fp64 (mean, then centred M2 -> sample std), scale in place
//   K8   assignment: distances to all k centres on the MATRIX cores --
//        v_mfma_f32_32x32x2_f32 (exact fp32 products) computes C.X^T for 32
//        centres x 32 points per wave, ||c||^2 - 2 c.x is reduced to a running
//        argmin per point (first index wins ties, as KMeans.findClosest)
//   K9   per-cluster sums: counting-sort points by label, then a segmented
//        sum that flushes one fp64 atomic per (label run, column)
//   K10  update (one workgroup): decay, weighted centroid move, dying-
//        cluster split -- StreamingKMeansModel.update [upstream]
#include <hip/hip_runtime.h>

#include <cfloat>

#include "common.h"
#include "kernels.h"
#include "kmeans_kernels.h"

namespace twtml {

// ---------------------------------------------------------------------------
// K1': dense features.  One wave per kept row; bigram counts through an LDS
// integer histogram (ds_add_u32 -- LDS float atomics are ~20x slower).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t km_lower(uint32_t c, const uint8_t* page, const uint16_t* blocks) {
  if (c < 128) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
  return (c + blocks[page[c >> 8] * 256 + (c & 255)]) & 0xFFFFu;
}

constexpr int kKmFeatWaves = 4;

__global__ __launch_bounds__(kBlock) void k_km_features(DevRawBatch b, const int64_t* kept,
                                                        const int64_t* counters, float* X, int dp,
                                                        int text_dims, const uint8_t* lpage,
                                                        const uint16_t* lblocks) {
  extern __shared__ uint32_t hist[];  // [kKmFeatWaves][text_dims]
  const int lane = lane_id(), w = threadIdx.x / kWave;
  uint32_t* h = hist + w * (text_dims > 0 ? text_dims : 1);
  const int64_t n_kept = counters[0];
  for (int64_t k = int64_t(blockIdx.x) * kKmFeatWaves + w; k < n_kept;
       k += int64_t(gridDim.x) * kKmFeatWaves) {
    const int64_t row = kept[k];
    float* xr = X + k * dp;
    if (text_dims > 0) {
      for (int j = lane; j < text_dims; j += kWave) h[j] = 0u;
      __builtin_amdgcn_wave_barrier();
      const int64_t o = b.offsets[row];
      const int64_t len = b.offsets[row + 1] - o;
      const int64_t nz = len >= 2 ? len - 1 : len;
      for (int64_t j = lane; j < nz; j += kWave) {
        const uint32_t u0 = km_lower(b.text[o + j], lpage, lblocks);
        const uint32_t hsh = len >= 2 ? 31u * u0 + km_lower(b.text[o + j + 1], lpage, lblocks) : u0;
        atomicAdd(&h[hsh % uint32_t(text_dims)], 1u);
      }
      __builtin_amdgcn_wave_barrier();
      for (int j = lane; j < text_dims; j += kWave) xr[2 + j] = float(h[j]);
    }
    if (lane == 0) {
      xr[0] = float(b.scalars[0 * b.n + row]);   // retweetCount
      xr[1] = float(b.scalars[1 * b.n + row]);   // followersCount
    }
    for (int j = 2 + text_dims + lane; j < dp; j += kWave) xr[j] = 0.f;
  }
}

void launch_km_features(const DevRawBatch& b, const int64_t* kept, const int64_t* counters,
                        float* X, int dp, int text_dims, const uint8_t* lpage,
                        const uint16_t* lblocks, int64_t max_rows, hipStream_t s) {
  int grid = ceil_div(max_rows > 0 ? max_rows : 1, kKmFeatWaves);
  if (grid > 8192) grid = 8192;
  const size_t lds = size_t(kKmFeatWaves) * size_t(text_dims > 0 ? text_dims : 1) * sizeof(uint32_t);
  hipLaunchKernelGGL(k_km_features, dim3(grid), dim3(kBlock), lds, s, b, kept, counters, X, dp,
                     text_dims, lpage, lblocks);
}

// ---------------------------------------------------------------------------
// K11: column moments (fp64).  mode 0: sums -> out[1+j] (+ n in out[0]);
// mode 1: centred squares -> out[j] using mean = sum_n[1+j] / sum_n[0].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_km_moments(const float* X, const int64_t* counters,
                                                       int d, int dp, int mode, const double* sum_n,
                                                       double* out) {
  const int64_t n = counters[0];
  // thread -> (row lane, column); columns strided over the block
  for (int j0 = 0; j0 < d; j0 += kBlock) {
    const int j = j0 + int(threadIdx.x);
    if (j >= d) continue;
    const double mean = mode == 1 && sum_n[0] > 0 ? sum_n[1 + j] / sum_n[0] : 0.0;
    double acc = 0.0;
    for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
      const double v = double(X[r * dp + j]) - mean;
      acc += mode == 0 ? v : v * v;
    }
    atomicAdd(&out[(mode == 0 ? 1 : 0) + j], acc);
  }
  if (mode == 0 && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&out[0], double(n));
}

void launch_km_moments(const float* X, const int64_t* counters, int d, int dp, int mode,
                       const double* sum_n, double* out, int64_t max_rows, hipStream_t s) {
  int grid = int(max_rows / 64 + 1);
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(k_km_moments, dim3(grid), dim3(kBlock), 0, s, X, counters, d, dp, mode, sum_n, out);
}

// factor_j = std_j != 0 ? 1/std_j : 0 with std = sqrt(M2/(n-1)), n < 2 -> 0
__global__ void k_km_scale(float* X, const int64_t* counters, int d, int dp, const double* sum_n,
                           const double* m2, double* factor_out) {
  const int64_t n = counters[0];
  const double cnt = sum_n[0];
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n * dp;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int j = int(i % dp);
    if (j >= d) continue;
    const double var = cnt > 1.0 ? m2[j] / (cnt - 1.0) : 0.0;
    const double sd = sqrt(var);
    const double f = sd != 0.0 ? 1.0 / sd : 0.0;
    X[i] = float(double(X[i]) * f);
  }
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < d; j += blockDim.x) {
      const double var = cnt > 1.0 ? m2[j] / (cnt - 1.0) : 0.0;
      factor_out[j] = sqrt(var);
    }
}

void launch_km_scale(float* X, const int64_t* counters, int d, int dp, const double* sum_n,
                     const double* m2, double* std_out, int64_t max_rows, hipStream_t s) {
  int grid = int((max_rows * dp) / 1024 + 1);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(k_km_scale, dim3(grid), dim3(kBlock), 0, s, X, counters, d, dp, sum_n, m2, std_out);
}

// ---------------------------------------------------------------------------
// K8: assignment on the matrix cores.
//   block = 4 waves = 128 points; per 32-centre tile the tile (row-padded to
//   DP+1 floats: conflict-free column reads) is staged in LDS.  A operand =
//   centres (lane: row l&31, k = kk + l>>5), B operand = points^T (lane: point
//   l&31, same k) kept in VGPRs for the whole sweep.  D(32x32) lane l holds
//   point l&31 and centres (r&3) + 8(r>>2) + 4(l>>5), r = 0..15.
// ---------------------------------------------------------------------------
using f32x16 = __attribute__((ext_vector_type(16))) float;

// A gap between the best and second-best fp32 distance (|c|^2 - 2x.c) below
// this is within accumulated rounding (~160 ulps of |x|^2 + |c|^2 - 2|x.c|
// magnitudes): such points are re-decided in fp64 by k_km_refine.
__device__ __forceinline__ float km_tie_margin(float xn, float best) {
  return 1e-5f * (xn + fabsf(best)) + 1e-30f;
}

template <int DP>
__global__ __launch_bounds__(kBlock) void k_km_assign_mfma(const float* X, const int64_t* counters,
                                                           const float* C, const float* cnorm, int k,
                                                           int32_t* labels, int32_t* refine,
                                                           unsigned long long* refine_cnt) {
  constexpr int KS = DP / 2;          // MFMA k-steps
  constexpr int LD = DP + 1;          // padded LDS row
  __shared__ float ct[32 * LD];
  __shared__ float cn[32];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int64_t n = counters[0];
  if (int64_t(blockIdx.x) * 128 >= n) return;   // block-uniform
  const int64_t p = int64_t(blockIdx.x) * 128 + w * 32 + (lane & 31);
  const int half = lane >> 5;
  float xb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) xb[s] = p < n ? X[p * DP + 2 * s + half] : 0.f;
  float xn = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) xn += xb[s] * xb[s];
  xn += __shfl_xor(xn, 32, kWave);
  float best = FLT_MAX, second = FLT_MAX;
  int bidx = 0;
  for (int c0 = 0; c0 < k; c0 += 32) {
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * DP; i += kBlock) {
      const int r = i / DP, col = i % DP;
      ct[r * LD + col] = (c0 + r < k) ? C[int64_t(c0 + r) * DP + col] : 0.f;
    }
    if (threadIdx.x < 32) cn[threadIdx.x] = (c0 + int(threadIdx.x) < k) ? cnorm[c0 + threadIdx.x] : FLT_MAX;
    __syncthreads();
    f32x16 acc = {};
    const float* crow = ct + (lane & 31) * LD + half;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(crow[2 * s], xb[s], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cl = (r & 3) + 8 * (r >> 2) + 4 * half;
      const float dist = cn[cl] - 2.f * acc[r];
      if (dist < best) { second = best; best = dist; bidx = c0 + cl; }
      else if (dist < second) second = dist;
    }
  }
  // combine the two lane halves (interleaved centre sets); ties -> lower index
  const float ob = __shfl_xor(best, 32, kWave);
  const float os = __shfl_xor(second, 32, kWave);
  const int oi = __shfl_xor(bidx, 32, kWave);
  if (ob < best || (ob == best && oi < bidx)) {
    second = fminf(os, best);
    best = ob; bidx = oi;
  } else {
    second = fminf(second, ob);
  }
  if (half == 0 && p < n) {
    labels[p] = bidx;
    if (second - best <= km_tie_margin(xn, best)) refine[atomicAdd(refine_cnt, 1ull)] = int32_t(p);
  }
}

// Generic fallback (any width): one thread per point, scalar fp32.
__global__ __launch_bounds__(kBlock) void k_km_assign_scalar(const float* X, const int64_t* counters,
                                                             const float* C, const float* cnorm, int k,
                                                             int dp, int32_t* labels, int32_t* refine,
                                                             unsigned long long* refine_cnt) {
  const int64_t n = counters[0];
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < n; p += int64_t(gridDim.x) * kBlock) {
    float best = FLT_MAX, second = FLT_MAX, xn = 0.f;
    int bi = 0;
    for (int j = 0; j < dp; ++j) xn += X[p * dp + j] * X[p * dp + j];
    for (int c = 0; c < k; ++c) {
      float dot = 0.f;
      for (int j = 0; j < dp; ++j) dot += C[int64_t(c) * dp + j] * X[p * dp + j];
      const float dist = cnorm[c] - 2.f * dot;
      if (dist < best) { second = best; best = dist; bi = c; }
      else if (dist < second) second = dist;
    }
    labels[p] = bi;
    if (second - best <= km_tie_margin(xn, best)) refine[atomicAdd(refine_cnt, 1ull)] = int32_t(p);
  }
}

// fp64 re-decision of near-ties (e.g. the two halves of a just-split cluster
// differ by 1e-14 relative, invisible in fp32): one wave per flagged point,
// direct sum of squared differences against the fp64 centres, first index
// on exact ties.
__global__ __launch_bounds__(kBlock) void k_km_refine(const float* X, const int32_t* refine,
                                                      const unsigned long long* refine_cnt,
                                                      const double* centers, int k, int d, int dp,
                                                      int32_t* labels) {
  const int lane = lane_id();
  const int64_t nref = int64_t(*refine_cnt);
  for (int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave; q < nref;
       q += int64_t(gridDim.x) * (kBlock / kWave)) {
    const int64_t p = refine[q];
    const float* x = X + p * dp;
    double best = DBL_MAX;
    int bi = 0x7fffffff;
    for (int c = lane; c < k; c += kWave) {
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double t = double(x[j]) - centers[int64_t(c) * d + j];
        s += t * t;
      }
      if (s < best) { best = s; bi = c; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ob = __shfl_xor(best, off, kWave);
      const int oi = __shfl_xor(bi, off, kWave);
      if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) labels[p] = bi;
  }
}

void launch_km_assign(const float* X, const int64_t* counters, const float* C, const float* cnorm,
                      const double* centers, int k, int d, int dp, int32_t* labels, int32_t* refine,
                      unsigned long long* refine_cnt, int64_t max_rows, bool mfma, hipStream_t s) {
  TWTML_HIP_CHECK(hipMemsetAsync(refine_cnt, 0, sizeof(unsigned long long), s));
  const int grid_m = int(max_rows / 128 + 1);
  bool done = false;
  if (mfma) {
#define KM_MFMA(DPV)                                                                                \
  case DPV:                                                                                         \
    hipLaunchKernelGGL(k_km_assign_mfma<DPV>, dim3(grid_m), dim3(kBlock), 0, s, X, counters, C,     \
                       cnorm, k, labels, refine, refine_cnt);                                       \
    done = true;                                                                                    \
    break;
    switch (dp) { KM_MFMA(2) KM_MFMA(4) KM_MFMA(8) KM_MFMA(16) KM_MFMA(32) KM_MFMA(64) KM_MFMA(128) default: break; }
#undef KM_MFMA
  }
  int grid = int(max_rows / kBlock + 1);
  if (grid > 4096) grid = 4096;
  if (!done)
    hipLaunchKernelGGL(k_km_assign_scalar, dim3(grid), dim3(kBlock), 0, s, X, counters, C, cnorm, k,
                       dp, labels, refine, refine_cnt);
  hipLaunchKernelGGL(k_km_refine, dim3(grid), dim3(kBlock), 0, s, X, refine, refine_cnt, centers, k,
                     d, dp, labels);
}

// ---------------------------------------------------------------------------
// K9: counting sort by label + segmented sums with one atomic per label run.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_km_label_hist(const int32_t* labels, const int64_t* counters,
                                                          int64_t* hist) {
  const int64_t n = counters[0];
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < n; p += int64_t(gridDim.x) * kBlock)
    atomicAdd(reinterpret_cast<unsigned long long*>(&hist[labels[p]]), 1ull);
}

__global__ __launch_bounds__(kBlock) void k_km_label_scatter(const int32_t* labels, const int64_t* counters,
                                                             int64_t* cursor, int32_t* order) {
  const int64_t n = counters[0];
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < n; p += int64_t(gridDim.x) * kBlock) {
    const int64_t pos = int64_t(atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[labels[p]]), 1ull));
    order[pos] = int32_t(p);
  }
}

constexpr int kSegRows = 1024;

// thread = (row lane rr, column j); walks rows rr, rr+RP, ... of its chunk in
// label order; flushes its running sum whenever the label changes.
__global__ __launch_bounds__(kBlock) void k_km_segsum(const float* X, const int32_t* labels,
                                                      const int32_t* order, const int64_t* counters,
                                                      int d, int dp, int cols_pow2, double* sums,
                                                      double* counts) {
  const int64_t n = counters[0];
  const int rp = kBlock / cols_pow2;               // rows per pass
  const int rr = threadIdx.x / cols_pow2;
  for (int64_t base = int64_t(blockIdx.x) * kSegRows; base < n; base += int64_t(gridDim.x) * kSegRows)
  for (int j = threadIdx.x % cols_pow2; j < d; j += cols_pow2) {   // column passes (d > 256)
    const int64_t end = base + kSegRows < n ? base + kSegRows : n;
    int cur = -1;
    double acc = 0.0, cnt = 0.0;
    for (int64_t q = base + rr; q < end; q += rp) {
      const int32_t p = order[q];
      const int lab = labels[p];
      if (lab != cur) {
        if (cur >= 0) {
          if (j < d) atomicAdd(&sums[int64_t(cur) * d + j], acc);
          if (j == 0) atomicAdd(&counts[cur], cnt);
        }
        cur = lab; acc = 0.0; cnt = 0.0;
      }
      if (j < d) acc += double(X[int64_t(p) * dp + j]);
      cnt += 1.0;
    }
    if (cur >= 0) {
      if (j < d) atomicAdd(&sums[int64_t(cur) * d + j], acc);
      if (j == 0) atomicAdd(&counts[cur], cnt);
    }
  }
}

void launch_km_cluster_sums(const float* X, const int32_t* labels, const int64_t* counters, int k,
                            int d, int dp, int64_t* hist, int32_t* order, double* sums,
                            double* counts, int64_t max_rows, hipStream_t s,
                            void (*scan)(const int64_t*, int64_t*, int64_t, int64_t*, hipStream_t)) {
  TWTML_HIP_CHECK(hipMemsetAsync(hist, 0, sizeof(int64_t) * size_t(k + 1), s));
  int grid = int(max_rows / kBlock + 1);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(k_km_label_hist, dim3(grid), dim3(kBlock), 0, s, labels, counters, hist);
  scan(hist, hist, k, nullptr, s);
  hipLaunchKernelGGL(k_km_label_scatter, dim3(grid), dim3(kBlock), 0, s, labels, counters, hist, order);
  int cp = 1;
  while (cp < d && cp < kBlock) cp <<= 1;
  int g2 = int(max_rows / kSegRows + 1);
  if (g2 > 4096) g2 = 4096;
  hipLaunchKernelGGL(k_km_segsum, dim3(g2), dim3(kBlock), 0, s, X, labels, order, counters, d, dp, cp,
                     sums, counts);
}

// ---------------------------------------------------------------------------
// K10: StreamingKMeansModel.update (one workgroup, fp64).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_km_update(double* centers, double* weights, const double* sums,
                                                    const double* counts, int k, int d, double decay,
                                                    int points_unit, float* c32, float* cnorm, int dp) {
  __shared__ double total;
  const int t = threadIdx.x;
  if (t == 0) {
    double s = 0.0;
    for (int c = 0; c < k; ++c) s += counts[c];
    total = s;
  }
  __syncthreads();
  const double discount = points_unit ? pow(decay, total) : decay;
  for (int c = t; c < k; c += 1024) {
    const double cnt = counts[c];
    double wgt = weights[c] * discount;
    if (cnt > 0.0) {
      const double upd = wgt + cnt;
      const double lam = cnt / (upd > 1e-16 ? upd : 1e-16);
      for (int j = 0; j < d; ++j)
        centers[int64_t(c) * d + j] = (1.0 - lam) * centers[int64_t(c) * d + j] + (lam / cnt) * sums[int64_t(c) * d + j];
      wgt = upd;
    }
    weights[c] = wgt;
  }
  __syncthreads();
  if (t == 0) {
    // dying-cluster check: argmax / argmin of the weights, first index on ties
    // (Scala maxBy/minBy); a sequential scan -- k is at most a few thousand
    int largest = 0, smallest = 0;
    for (int c = 1; c < k; ++c) {
      if (weights[c] > weights[largest]) largest = c;
      if (weights[c] < weights[smallest]) smallest = c;
    }
    const double maxw = weights[largest], minw = weights[smallest];
    if (minw < 1e-8 * maxw) {
      const double wv = (maxw + minw) / 2.0;
      weights[largest] = wv;
      weights[smallest] = wv;
      for (int j = 0; j < d; ++j) {
        const double x = centers[int64_t(largest) * d + j];
        const double pp = 1e-14 * (fabs(x) > 1.0 ? fabs(x) : 1.0);
        centers[int64_t(largest) * d + j] = x + pp;
        centers[int64_t(smallest) * d + j] = x - pp;
      }
    }
  }
  __syncthreads();
  for (int c = t; c < k; c += 1024) {
    float nrm = 0.f;
    for (int j = 0; j < dp; ++j) {
      const float v = j < d ? float(centers[int64_t(c) * d + j]) : 0.f;
      c32[int64_t(c) * dp + j] = v;
      nrm += v * v;
    }
    cnorm[c] = nrm;
  }
}

void launch_km_update(double* centers, double* weights, const double* sums, const double* counts,
                      int k, int d, double decay, bool points_unit, float* c32, float* cnorm, int dp,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_km_update, dim3(1), dim3(1024), 0, s, centers, weights, sums, counts, k, d,
                     decay, points_unit ? 1 : 0, c32, cnorm, dp);
}

__global__ void k_km_centers32(const double* centers, int k, int d, int dp, float* c32, float* cnorm) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < k; c += gridDim.x * blockDim.x) {
    float nrm = 0.f;
    for (int j = 0; j < dp; ++j) {
      const float v = j < d ? float(centers[int64_t(c) * d + j]) : 0.f;
      c32[int64_t(c) * dp + j] = v;
      nrm += v * v;
    }
    cnorm[c] = nrm;
  }
}

void launch_km_centers32(const double* centers, int k, int d, int dp, float* c32, float* cnorm,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_km_centers32, dim3((k + 255) / 256), dim3(256), 0, s, centers, k, d, dp, c32, cnorm);
}

}  // namespace twtml
