// Streaming linear regression (StreamingLinearRegressionWithSGD) on MI355X.
//
// One GradientDescent iteration (SURVEY §2.2 U5-U7, §3.2 hot loop):
//   r_i = x_i . w - y_i          (LeastSquaresGradient, U6)
//   g   = sum_i r_i x_i          (treeAggregate -> here LDS-privatised scatter)
//   w  -= (step / sqrt(i)) g / m (SimpleUpdater, U7)
//   stop when ||dw|| < tol * max(||w||, 1) once two updates exist.
//
// The model works in the batch's *compact active space*: slots 0..3 are the
// numeric features (F..F+3), slots 4.. the text features touched by the
// batch (sorted feature ids), followed by 64 zero-weight pad slots.  Untouched
// features have exactly zero gradient, so the compact iteration is exactly
// the full-width one; ||w|| adds the constant norm of the untouched part.
//
// k_sgd_iter: each workgroup stages the compact fp32 weights in LDS
// (typically 4-16K slots -> 16-64 KB), streams its SELL-64 chunks (one row per
// lane, 16-byte slot loads), gathers w from LDS, and scatters r into an LDS
// gradient (ds_add_f32) -- the hot bigram range never touches global
// atomics.  The workgroup flushes its non-zero gradient slots once.  At
// iteration 1 the same pass yields the prequential predictions and batch
// statistics (K4 + K7 fused: output op #1 uses the weights before training).
// k_sgd_update (one workgroup): fp64 master update + norms + convergence flag;
// every later kernel of the batch early-exits once the flag is set.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace twtml {

constexpr int kLdsBytes = 160 * 1024;

int sgd_lds_limit_slots() { return kLdsBytes / (2 * int(sizeof(float))); }

template <typename SlotT>
struct SlotLoad;

template <>
struct SlotLoad<uint16_t> {
  __device__ __forceinline__ static void load(const uint16_t* p, uint32_t (&s)[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    s[0] = v.x & 0xFFFF; s[1] = v.x >> 16; s[2] = v.y & 0xFFFF; s[3] = v.y >> 16;
    s[4] = v.z & 0xFFFF; s[5] = v.z >> 16; s[6] = v.w & 0xFFFF; s[7] = v.w >> 16;
  }
};

template <>
struct SlotLoad<uint32_t> {
  __device__ __forceinline__ static void load(const uint32_t* p, uint32_t (&s)[8]) {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0];
    const uint4 b = reinterpret_cast<const uint4*>(p)[1];
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
  }
};

template <typename SlotT, bool STATS, bool SAMPLE, bool LDS>
__global__ __launch_bounds__(kBlock) void k_sgd_iter(DevSgd d, DevPrepared p, SgdParams sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double red_scratch[kBlock / kWave];
  if (d.state[0] != 0.0) return;  // converged / finished: whole batch is a no-op
  const int64_t ns = d.ns;
  float* wl = lds;
  float* gl = lds + (LDS ? ns : 0);
  const float* w = LDS ? wl : d.wc32;
  float* g = LDS ? gl : d.g32;
  if (LDS) {
    for (int64_t s = threadIdx.x; s < ns; s += kBlock) {
      wl[s] = d.wc32[s];
      gl[s] = 0.f;
    }
    __syncthreads();
  }
  const int lane = lane_id();
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kChunk - 1) / kChunk;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  const SlotT* slot = static_cast<const SlotT*>(p.slot);
  const float w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];

  float gn0 = 0.f, gn1 = 0.f, gn2 = 0.f, gn3 = 0.f, loss = 0.f;
  double msum = 0.0;
  double st_n = 0, st_y = 0, st_y2 = 0, st_p = 0, st_p2 = 0, st_e2 = 0;

  for (int64_t c = wave; c < nch; c += nwaves) {
    const int32_t L8 = p.clen8[c];
    const SlotT* sl = slot + p.cbase[c] * kChunkStride + lane * kGroup;
    float dot = 0.f;
    for (int32_t q = 0; q < L8; ++q) {
      uint32_t s[8];
      SlotLoad<SlotT>::load(sl + int64_t(q) * kChunkStride, s);
#pragma unroll
      for (int k = 0; k < 8; ++k) dot += w[s[k]];
    }
    const int64_t q0 = c * kChunk + lane;
    const float n0 = p.num[(c * 4 + 0) * kChunk + lane], n1 = p.num[(c * 4 + 1) * kChunk + lane];
    const float n2 = p.num[(c * 4 + 2) * kChunk + lane], n3 = p.num[(c * 4 + 3) * kChunk + lane];
    dot += n0 * w0 + n1 * w1 + n2 * w2 + n3 * w3;
    const bool valid = q0 < n_kept;
    const float y = p.y[q0];
    bool in = valid;
    if (SAMPLE && valid)
      in = sample_uniform(uint64_t(42 + sp.iteration), uint64_t(sp.row_offset + p.perm[q0])) <
           sp.fraction;
    const float r = in ? dot - y : 0.f;
    if (STATS && valid) {
      const double pr = round_half_away(double(dot));
      if (sp.want_pred) d.pred_out[p.perm[q0]] = float(pr);
      const double yd = double(y), e = yd - pr;
      st_n += 1.0; st_y += yd; st_y2 += yd * yd; st_p += pr; st_p2 += pr * pr; st_e2 += e * e;
    }
    if (__any(r != 0.f)) {
      for (int32_t q = 0; q < L8; ++q) {
        uint32_t s[8];
        SlotLoad<SlotT>::load(sl + int64_t(q) * kChunkStride, s);
        if (r != 0.f) {
#pragma unroll
          for (int k = 0; k < 8; ++k) atomicAdd(&g[s[k]], r);
        }
      }
    }
    gn0 += r * n0; gn1 += r * n1; gn2 += r * n2; gn3 += r * n3;
    loss += r * r;
    msum += in ? 1.0 : 0.0;
  }

  // --- workgroup reductions of the scalar partials -> one atomic each
  const double b0 = block_sum<double>(gn0, red_scratch);
  const double b1 = block_sum<double>(gn1, red_scratch);
  const double b2 = block_sum<double>(gn2, red_scratch);
  const double b3 = block_sum<double>(gn3, red_scratch);
  const double bl = block_sum<double>(0.5 * double(loss), red_scratch);
  double bm = 0.0;
  if (SAMPLE) bm = block_sum<double>(msum, red_scratch);
  double bs[6] = {0, 0, 0, 0, 0, 0};
  if (STATS) {
    bs[0] = block_sum<double>(st_n, red_scratch);
    bs[1] = block_sum<double>(st_y, red_scratch);
    bs[2] = block_sum<double>(st_y2, red_scratch);
    bs[3] = block_sum<double>(st_p, red_scratch);
    bs[4] = block_sum<double>(st_p2, red_scratch);
    bs[5] = block_sum<double>(st_e2, red_scratch);
  }
  if (threadIdx.x == 0) {
    atomicAdd(&d.g32[0], float(b0));
    atomicAdd(&d.g32[1], float(b1));
    atomicAdd(&d.g32[2], float(b2));
    atomicAdd(&d.g32[3], float(b3));
    atomicAdd(&d.g32[ns], float(bl));
    if (SAMPLE) atomicAdd(&d.red64[1], bm);
    if (STATS)
      for (int k = 0; k < 6; ++k) atomicAdd(&d.stats[k], bs[k]);
  }
  if (LDS) {
    __syncthreads();
    const int64_t hi = kNumNumeric + d.n_unique;  // pads are never flushed
    for (int64_t s = kNumNumeric + threadIdx.x; s < hi; s += kBlock) {
      const float v = gl[s];
      if (v != 0.f) atomicAdd(&d.g32[s], v);
    }
  }
}

template <typename SlotT, bool LDS>
static void launch_iter_t(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, int grid,
                          size_t lds, hipStream_t s) {
  const bool stats = sp.iteration == 1;
  const bool sample = sp.sample != 0;
  if (stats && sample)
    hipLaunchKernelGGL((k_sgd_iter<SlotT, true, true, LDS>), dim3(grid), dim3(kBlock), lds, s, d, p, sp);
  else if (stats)
    hipLaunchKernelGGL((k_sgd_iter<SlotT, true, false, LDS>), dim3(grid), dim3(kBlock), lds, s, d, p, sp);
  else if (sample)
    hipLaunchKernelGGL((k_sgd_iter<SlotT, false, true, LDS>), dim3(grid), dim3(kBlock), lds, s, d, p, sp);
  else
    hipLaunchKernelGGL((k_sgd_iter<SlotT, false, false, LDS>), dim3(grid), dim3(kBlock), lds, s, d, p, sp);
}

void launch_sgd_iter(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, int64_t /*groups*/,
                     bool u16, int grid, hipStream_t s) {
  const bool lds_ok = d.ns <= sgd_lds_limit_slots() - 64;
  const size_t lds = lds_ok ? size_t(2 * d.ns) * sizeof(float) : 0;
  if (u16) {
    if (lds_ok) launch_iter_t<uint16_t, true>(d, p, sp, grid, lds, s);
    else launch_iter_t<uint16_t, false>(d, p, sp, grid, lds, s);
  } else {
    if (lds_ok) launch_iter_t<uint32_t, true>(d, p, sp, grid, lds, s);
    else launch_iter_t<uint32_t, false>(d, p, sp, grid, lds, s);
  }
}

// ---------------------------------------------------------------------------
// SimpleUpdater + convergence test (one workgroup, fp64 master weights).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_sgd_update(DevSgd d, SgdParams sp) {
  __shared__ double scratch[16];
  if (d.state[0] != 0.0) return;
  const int tid = threadIdx.x;
  const int64_t hi = kNumNumeric + d.n_unique;
  const double m = sp.sample ? d.red64[1] : d.state[5];
  const double loss = double(d.g32[d.ns]);
  double ds = 0.0, ws = 0.0;
  if (m > 0.0) {
    const double alpha = sp.step_size / sqrt(double(sp.iteration));
    for (int64_t s = tid; s < hi; s += 1024) {
      const double step = alpha * (double(d.g32[s]) / m);
      const double wn = d.wc64[s] - step;
      d.wc64[s] = wn;
      d.wc32[s] = float(wn);
      d.g32[s] = 0.f;
      ds += step * step;
      ws += wn * wn;
    }
  } else {
    for (int64_t s = tid; s < hi; s += 1024) d.g32[s] = 0.f;
  }
  // block reduce (1024 threads = 16 waves)
  ds = wave_sum(ds);
  ws = wave_sum(ws);
  const int w = tid / kWave;
  if (lane_id() == 0) scratch[w] = ds;
  __syncthreads();
  double dsum = 0.0;
  for (int k = 0; k < 16; ++k) dsum += scratch[k];
  __syncthreads();
  if (lane_id() == 0) scratch[w] = ws;
  __syncthreads();
  double wsum = 0.0;
  for (int k = 0; k < 16; ++k) wsum += scratch[k];
  if (tid == 0) {
    if (m > 0.0) {
      d.loss_hist[sp.iteration] = loss / m;
      const double nupd = d.state[2] + 1.0;
      d.state[2] = nupd;
      double rest = d.state[4] - d.state[6];
      if (rest < 0.0) rest = 0.0;
      const double wnorm = sqrt(wsum + rest);
      if (nupd >= 2.0 && sqrt(dsum) < sp.tol * (wnorm > 1.0 ? wnorm : 1.0)) {
        d.state[0] = 1.0;
        d.state[1] = 1.0;
      }
    }
    d.state[3] = double(sp.iteration);
    if (sp.iteration >= sp.num_iterations) d.state[0] = 1.0;
    d.g32[d.ns] = 0.f;
    d.red64[0] = 0.0;
    d.red64[1] = 0.0;
  }
}

void launch_sgd_update(const DevSgd& d, const SgdParams& sp, hipStream_t s) {
  hipLaunchKernelGGL(k_sgd_update, dim3(1), dim3(1024), 0, s, d, sp);
}

// ---------------------------------------------------------------------------
// Gather / scatter between full-width fp64 weights and the compact space.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_gather_w(DevSgd d, const int32_t* uniq) {
  __shared__ double scratch[kBlock / kWave];
  double acc = 0.0;
  for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < d.ns;
       s += int64_t(gridDim.x) * kBlock) {
    double v = 0.0;
    if (s < kNumNumeric) v = d.w64[d.F + s];
    else if (s < kNumNumeric + d.n_unique) v = d.w64[uniq[s - kNumNumeric]];
    d.wc64[s] = v;
    d.wc32[s] = float(v);
    d.g32[s] = 0.f;
    acc += v * v;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) atomicAdd(&d.state[6], acc);
}

__global__ __launch_bounds__(kBlock) void k_norm2(const double* v, int64_t n, double* out) {
  __shared__ double scratch[kBlock / kWave];
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    acc += v[i] * v[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) atomicAdd(out, acc);
}

__global__ __launch_bounds__(kBlock) void k_scatter_w(DevSgd d, const int32_t* uniq) {
  for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < kNumNumeric + d.n_unique;
       s += int64_t(gridDim.x) * kBlock) {
    if (s < kNumNumeric) d.w64[d.F + s] = d.wc64[s];
    else d.w64[uniq[s - kNumNumeric]] = d.wc64[s];
  }
}

void launch_gather_w(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  int grid = ceil_div(d.ns, kBlock);
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(k_gather_w, dim3(grid), dim3(kBlock), 0, s, d, p.uniq);
}

void launch_norm2(const double* v, int64_t n, double* out, hipStream_t s) {
  int grid = ceil_div(n, kBlock * 8);
  if (grid > 1024) grid = 1024;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_norm2, dim3(grid), dim3(kBlock), 0, s, v, n, out);
}

void launch_scatter_w(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  int grid = ceil_div(kNumNumeric + d.n_unique, kBlock);
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(k_scatter_w, dim3(grid), dim3(kBlock), 0, s, d, p.uniq);
}

}  // namespace twtml

namespace twtml {
__global__ void k_batch_init(double* state, double m_global) { state[5] = m_global; }
void launch_batch_init(double* state, double m_global, hipStream_t s) {
  hipLaunchKernelGGL(k_batch_init, dim3(1), dim3(1), 0, s, state, m_global);
}
}  // namespace twtml
