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
// k_sgd_iter_lds (the hot kernel): a 1024-thread workgroup stages the compact
// fp32 weights in LDS, streams its SELL-16x4 chunks (4 lanes per row, the
// row's slots kept in VGPRs between the forward gather and the backward
// scatter), and accumulates the gradient in LDS as 64-bit FIXED POINT with
// ds_add_u64.  Measured on gfx950 (tools/ubench_lds_atomics.hip): ds_add_f32
// costs ~170 LDS cycles per wave-instruction, ds_add_u64 ~12 and ds_read_b32
// ~8, so integer accumulation is ~14x faster -- and exact, so a workgroup's
// partial gradient is independent of the order rows are added in.  Each
// workgroup flushes its non-zero slots once (fp64 global atomics).  At
// iteration 1 the same pass yields the prequential predictions and batch
// statistics (K4 + K7 fused: output op #1 uses the weights before training).
// k_sgd_update (one workgroup): fp64 master update + norms + convergence
// flag; every later kernel of the batch early-exits once the flag is set.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace twtml {

// Fixed-point scale of the LDS gradient: residuals are added as
// round(r * 2^24) (resolution 6e-8, finer than fp32 for |r| > 1).  |r| is
// clamped (at most 2^26, tighter when a workgroup sees more entries, see
// sgd_fix_limit) so a workgroup's int64 slot sums cannot overflow; a clamp
// raises the overflow flag (state[7]) and the host reports it.
constexpr float kFixScale = 16777216.0f;        // 2^24
constexpr double kFixInv = 1.0 / 16777216.0;
constexpr float kFixClamp = 67108864.0f;        // 2^26

// Iteration record i (k_sgd_update -> convergence test) and the sampled row
// count of iteration i (double-buffered by parity: iteration i+1's count is
// zeroed while iteration i's is still being read).
__device__ __forceinline__ double* sgd_rec(const DevSgd& d, int it) { return d.itrec + int64_t(it) * kRecStride; }
__device__ __forceinline__ double* sgd_red_m(const DevSgd& d, int it) { return d.red64 + 2 * (it & 1) + 1; }

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

__device__ __forceinline__ void unpack4(const uint2 v, uint32_t (&s)[4]) {
  s[0] = v.x & 0xFFFF; s[1] = v.x >> 16; s[2] = v.y & 0xFFFF; s[3] = v.y >> 16;
}

__device__ __forceinline__ void unpack8(const uint4 v, uint32_t (&s)[8]) {
  s[0] = v.x & 0xFFFF; s[1] = v.x >> 16; s[2] = v.y & 0xFFFF; s[3] = v.y >> 16;
  s[4] = v.z & 0xFFFF; s[5] = v.z >> 16; s[6] = v.w & 0xFFFF; s[7] = v.w >> 16;
}

// Per-row epilogue shared by both iteration kernels: residual, stats, preds.
struct RowAcc {
  float gn0 = 0.f, gn1 = 0.f, gn2 = 0.f, gn3 = 0.f, loss = 0.f;
  double msum = 0.0;
  double st[6] = {0, 0, 0, 0, 0, 0};
};

// Row-level inputs (numeric features + label), loadable ahead of the dot.
struct RowIn {
  float n0, n1, n2, n3, y;
};

__device__ __forceinline__ RowIn row_in(const DevPrepared& p, int64_t pos) {
  const int64_t cap = p.cap_rows16;
  return RowIn{p.num[0 * cap + pos], p.num[1 * cap + pos], p.num[2 * cap + pos],
               p.num[3 * cap + pos], p.y[pos]};
}

template <bool STATS, bool SAMPLE>
__device__ __forceinline__ float row_residual(float dot, const RowIn& ri, int64_t pos, int t,
                                              const DevSgd& d, const DevPrepared& p,
                                              const SgdParams& sp, int64_t n_kept, float w0, float w1,
                                              float w2, float w3, RowAcc& acc) {
  const bool valid = pos < n_kept;
  const float n0 = ri.n0, n1 = ri.n1, n2 = ri.n2, n3 = ri.n3;
  dot += n0 * w0 + n1 * w1 + n2 * w2 + n3 * w3;
  const float y = ri.y;
  bool in = valid;
  if (SAMPLE && valid)
    in = sample_uniform(uint64_t(42 + sp.iteration), uint64_t(sp.row_offset + p.perm[pos])) <
         sp.fraction;
  const float r = in ? dot - y : 0.f;
  if (t == 0) {  // one lane per row owns the row-level accumulators
    if (STATS && valid) {
      const double pr = round_half_away(double(dot));
      if (sp.want_pred) d.pred_out[p.perm[pos]] = float(pr);
      const double yd = double(y), e = yd - pr;
      acc.st[0] += 1.0; acc.st[1] += yd; acc.st[2] += yd * yd;
      acc.st[3] += pr; acc.st[4] += pr * pr; acc.st[5] += e * e;
    }
    acc.gn0 += r * n0; acc.gn1 += r * n1; acc.gn2 += r * n2; acc.gn3 += r * n3;
    acc.loss += r * r;
    acc.msum += in ? 1.0 : 0.0;
  }
  return r;
}

template <bool STATS, bool SAMPLE>
__device__ __forceinline__ float row_residual(float dot, int64_t pos, int t, const DevSgd& d,
                                              const DevPrepared& p, const SgdParams& sp,
                                              int64_t n_kept, float w0, float w1, float w2,
                                              float w3, RowAcc& acc) {
  return row_residual<STATS, SAMPLE>(dot, row_in(p, pos), pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
}

template <bool STATS, bool SAMPLE>
__device__ __forceinline__ void flush_scalars(const DevSgd& d, const RowAcc& acc, double* scratch, int it) {
  const double b0 = block_sum<double>(acc.gn0, scratch);
  const double b1 = block_sum<double>(acc.gn1, scratch);
  const double b2 = block_sum<double>(acc.gn2, scratch);
  const double b3 = block_sum<double>(acc.gn3, scratch);
  const double bl = block_sum<double>(0.5 * double(acc.loss), scratch);
  double bm = 0.0;
  if (SAMPLE) bm = block_sum<double>(acc.msum, scratch);
  double bs[6] = {0, 0, 0, 0, 0, 0};
  if (STATS)
    for (int k = 0; k < 6; ++k) bs[k] = block_sum<double>(acc.st[k], scratch);
  if (threadIdx.x == 0) {
    atomicAdd(&d.g64[0], b0);
    atomicAdd(&d.g64[1], b1);
    atomicAdd(&d.g64[2], b2);
    atomicAdd(&d.g64[3], b3);
    atomicAdd(&d.g64[d.ns], bl);
    if (SAMPLE) atomicAdd(sgd_red_m(d, it), bm);
    if (STATS)
      for (int k = 0; k < 6; ++k) atomicAdd(&d.stats[k], bs[k]);
  }
}

// Workgroup epilogue without contended atomics.  Every workgroup writes one
// partial row (plain stores) that k_sgd_reduce sums in a fixed order:
//   cols 0..3 numeric gradients, 4..hi-1 text slots, hi..ns-1 pads (0),
//   ns loss, ns+1 sampled row count, ns+2..ns+7 batch stats (STATS).
// (256 workgroups adding into the same fp64 addresses serialise at the
// memory-side atomic units: ~10-20 us per launch on MI355X, measured.)
constexpr int kPartVals = 12;

template <bool STATS, bool SAMPLE>
__device__ __forceinline__ void part_scalars(const DevSgd& d, const RowAcc& acc,
                                             double (*wsc)[kPartVals], double* prow) {
  double v[kPartVals] = {0.0, 0.0, 0.0, 0.0, 0.0, acc.msum, acc.st[0], acc.st[1], acc.st[2],
                         acc.st[3], acc.st[4], acc.st[5]};
  constexpr int nv = STATS ? kPartVals : (SAMPLE ? 6 : 5);
  const int w = threadIdx.x / kWave;
  // the per-lane fp32 partials reduce on the VALU (DPP); fp64 from here on
  v[0] = double(wave_sum_f32(acc.gn0));
  v[1] = double(wave_sum_f32(acc.gn1));
  v[2] = double(wave_sum_f32(acc.gn2));
  v[3] = double(wave_sum_f32(acc.gn3));
  v[4] = 0.5 * double(wave_sum_f32(acc.loss));
#pragma unroll
  for (int k = 5; k < nv; ++k) v[k] = wave_sum(v[k]);
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < nv; ++k) wsc[w][k] = v[k];
  }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < kPartVals) {
    double t = 0.0;
    if (tid < nv)
      for (int k = 0; k < int(blockDim.x) / kWave; ++k) t += wsc[k][tid];
    prow[tid < kNumNumeric ? int64_t(tid) : d.ns + (tid - kNumNumeric)] = t;
  }
}

// Text-slot columns of a partial row: the REP fixed-point replicas summed
// (+ the hot total of a hot slot).
template <int REP>
__device__ __forceinline__ double part_slot(const unsigned long long* gl, int64_t s) {
  long long v = 0;
#pragma unroll
  for (int k = 0; k < REP; ++k) v += (long long)gl[s * REP + k];
  return double(v) * kFixInv;
}

float sgd_fix_limit(int64_t entries_per_wg) {
  const double e = double(entries_per_wg < 1 ? 1 : entries_per_wg);
  const double lim = std::min(double(kFixClamp) * double(kFixScale), 4.611686018427388e18 / e);
  return float(lim * 0.999);
}

__device__ __forceinline__ unsigned long long to_fix(float r, bool& clamped, float lim) {
  float v = r * kFixScale;
  if (fabsf(v) > lim) {
    clamped = true;
    v = v > 0.f ? lim : -lim;
  }
  return (unsigned long long)(long long)__float2ll_rn(v);
}

// ---------------------------------------------------------------------------
// Fast path: u16 slots, LDS weights + REP replicated fixed-point gradients.
// ---------------------------------------------------------------------------
constexpr int kIterBlock = 1024;

// CNT: entries carry HashingTF term counts (p.cnt, merged duplicates, chunk
// lengths p.clen8d); otherwise every entry counts once.
// Convergence after update `it`, evaluated by one wave (lane-parallel loads,
// fixed-order DPP reduction): identical in every caller.
__device__ bool sgd_converged_wave(const DevSgd& d, int it, double tol) {
  const double* rec = sgd_rec(d, it);
  const int nw = int(rec[2]);
  double ds = 0.0, ws = 0.0;
  for (int k = lane_id(); k < nw; k += kWave) {
    ds += rec[kRecHead + 2 * k];
    ws += rec[kRecHead + 2 * k + 1];
  }
  ds = wave_sum(ds);
  ws = wave_sum(ws);
  if (!(rec[1] > 0.0) || rec[0] < 2.0) return false;   // no update this iteration / first update
  double rest = d.state[4] - d.state[6];
  if (rest < 0.0) rest = 0.0;
  const double wnorm = sqrt(ws + rest);
  return sqrt(ds) < tol * (wnorm > 1.0 ? wnorm : 1.0);
}

// Iteration-kernel prologue: true when the batch is finished (the caller
// returns).  Called by every thread; `flag` is a workgroup-shared int.
// Also publishes the verdict for update i-1 to the host (zero-copy pinned
// memory, initialised to -1 by the host): the host polls it to stop
// enqueueing iterations, without a per-iteration event in the stream.
__device__ bool sgd_stop(const DevSgd& d, const SgdParams& sp, int* flag) {
  if (threadIdx.x < kWave) {
    const bool done = d.state[0] != 0.0;
    bool stop = done;
    if (!done && sp.iteration > 1) {
      stop = sgd_converged_wave(d, sp.iteration - 1, sp.tol);
      if (stop && blockIdx.x == 0 && threadIdx.x == 0) {
        d.state[0] = 1.0;
        d.state[1] = 1.0;
      }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && d.host_flags && sp.iteration > 1) {
      __hip_atomic_store(&d.host_flags[sp.iteration - 1], stop ? 1.0 : 0.0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (threadIdx.x == 0) *flag = stop ? 1 : 0;
  }
  __syncthreads();
  return *flag != 0;
}

template <bool STATS, bool SAMPLE, int REP, bool CNT>
__global__ __launch_bounds__(kIterBlock) void k_sgd_iter_lds(DevSgd d, DevPrepared p, SgdParams sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double wsc[kIterBlock / kWave][kPartVals];
  __shared__ int stop_flag;
  if (sgd_stop(d, sp, &stop_flag)) return;  // converged / finished: the rest of the batch is a no-op
  const int64_t ns = d.ns;        // multiple of 64
  float* wl = lds;
  unsigned long long* gl = reinterpret_cast<unsigned long long*>(lds + ns);
  for (int64_t s = threadIdx.x; s < ns; s += kIterBlock) wl[s] = d.wc32[s];
  for (int64_t s = threadIdx.x; s < ns * REP; s += kIterBlock) gl[s] = 0ull;
  __syncthreads();
  const int lane = lane_id();
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  const int rep = lane % REP;
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t wave = int64_t(blockIdx.x) * (kIterBlock / kWave) +
                       __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);   // wave-uniform
  const int64_t nwaves = int64_t(gridDim.x) * (kIterBlock / kWave);
  const uint16_t* slot = static_cast<const uint16_t*>(p.slot);
  const float w0 = wl[0], w1 = wl[1], w2 = wl[2], w3 = wl[3];
  RowAcc acc;
  bool clamped = false;

  // chunk metadata for 64 chunks at a time in lanes (see k_sgd_iter_hyb)
  const int32_t* __restrict__ clen = CNT ? p.clen8d : p.clen8;
  int32_t md_l8 = 0;
  int64_t md_cb = 0;
  int k = 0;
  for (int64_t c = wave; c < nch; c += nwaves, ++k) {
    if ((k & (kWave - 1)) == 0) {
      const int64_t cc = c + int64_t(lane) * nwaves;
      md_l8 = cc < nch ? clen[cc] : 0;
      md_cb = cc < nch ? p.cbase[cc] : 0;
    }
    const int kl = k & (kWave - 1);
    const int32_t L8 = __builtin_amdgcn_readlane(md_l8, kl);
    const int64_t cb = int64_t(uint32_t(__builtin_amdgcn_readlane(int32_t(md_cb), kl))) |
                       (int64_t(__builtin_amdgcn_readlane(int32_t(md_cb >> 32), kl)) << 32);
    const int64_t off = cb * kChunkStride + lane * kGroup;
    const uint16_t* sl = slot + off;
    const int64_t pos = c * kRowsPerChunk + r;
    const RowIn ri = row_in(p, pos);
    if (L8 <= kMaxRegGroups) {
      uint4 v[kMaxRegGroups];
      uint4 cv[CNT ? kMaxRegGroups : 1];
#pragma unroll
      for (int g = 0; g < kMaxRegGroups; ++g)
        if (g < L8) {
          v[g] = *reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride);
          if (CNT) cv[g] = *reinterpret_cast<const uint4*>(p.cnt + off + int64_t(g) * kChunkStride);
        }
      float d0 = 0.f, d1 = 0.f;
#pragma unroll
      for (int g = 0; g < kMaxRegGroups; ++g) {
        if (g < L8 && sp.ablate < 2) {
          uint32_t s[8];
          unpack8(v[g], s);
          if (CNT) {
            uint32_t k[8];
            unpack8(cv[g], k);
            d0 += wl[s[0]] * float(k[0]) + wl[s[2]] * float(k[2]) + wl[s[4]] * float(k[4]) +
                  wl[s[6]] * float(k[6]);
            d1 += wl[s[1]] * float(k[1]) + wl[s[3]] * float(k[3]) + wl[s[5]] * float(k[5]) +
                  wl[s[7]] * float(k[7]);
          } else {
            d0 += wl[s[0]] + wl[s[2]] + wl[s[4]] + wl[s[6]];
            d1 += wl[s[1]] + wl[s[3]] + wl[s[5]] + wl[s[7]];
          }
        }
      }
      float dot = d0 + d1;
      if (sp.ablate >= 2) {
        uint32_t s[8];
        unpack8(v[0], s);
        dot += float(s[0] + s[7]) * 1e-30f;  // keep the loads live
      }
      dot += __shfl_xor(dot, 1, kWave);
      dot += __shfl_xor(dot, 2, kWave);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
      if (res != 0.f && sp.ablate == 0) {
        const unsigned long long q = to_fix(res, clamped, sp.fix_lim);
#pragma unroll
        for (int g = 0; g < kMaxRegGroups; ++g) {
          if (g < L8) {
            uint32_t s[8];
            unpack8(v[g], s);
            if (CNT) {
              uint32_t k[8];
              unpack8(cv[g], k);
#pragma unroll
              for (int e = 0; e < 8; ++e) atomicAdd(&gl[s[e] * REP + rep], q * (unsigned long long)k[e]);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) atomicAdd(&gl[s[e] * REP + rep], q);
            }
          }
        }
      }
    } else {  // very long rows: stream the slots twice (never merged: count 1)
      float dot = 0.f;
      for (int32_t g = 0; g < L8; ++g) {
        uint32_t s[8];
        unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
        for (int k = 0; k < 8; ++k) dot += wl[s[k]];
      }
      dot += __shfl_xor(dot, 1, kWave);
      dot += __shfl_xor(dot, 2, kWave);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
      if (res != 0.f) {
        const unsigned long long q = to_fix(res, clamped, sp.fix_lim);
        for (int32_t g = 0; g < L8; ++g) {
          uint32_t s[8];
          unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
          for (int k = 0; k < 8; ++k) atomicAdd(&gl[s[k] * REP + rep], q);
        }
      }
    }
  }

  if (__any(clamped) && lane == 0) d.state[7] = 1.0;
  double* prow = d.part + int64_t(blockIdx.x) * d.pstride;
  part_scalars<STATS, SAMPLE>(d, acc, wsc, prow);   // includes the block barrier
  const int64_t hi = kNumNumeric + d.n_unique;      // pads are never flushed
  for (int64_t s = kNumNumeric + threadIdx.x; s < ns; s += kIterBlock)
    prow[s] = s < hi ? part_slot<REP>(gl, s) : 0.0;
}

// ---------------------------------------------------------------------------
// Hybrid dense-hot path (layout: hot_split.hip).  Per chunk a lane reads its
// row's 32 hot counts (16 B: 4-bit counts of hot ids 32t..32t+31) and the
// row-balanced cold groups.  Hot weights are read from LDS with b128 loads
// (broadcast across the 16 lanes of a quarter), the hot gradient accumulates
// in VGPRs (fp32 per lane, fp64 across waves); only cold entries use the LDS
// fixed-point gradient.  Chunks left
// in the plain layout (clen8c < 0) take the plain route.
// ---------------------------------------------------------------------------
constexpr int kHotRows = kWave / 16;  // 16-lane rows per wave (hot-gradient partials per wave)
constexpr int kMaxColdGroups = 8;   // cold 4-entry groups kept in VGPRs (32 cold entries per lane)
constexpr int kHotPerLane = kHot / kLanesPerRow;   // 32

// wq: this lane's 32 hot weights in LDS (quarter t, 16-B aligned, stride 36
// floats so the four quarters' b128 reads hit different banks)
constexpr int kHotLdsStride = kHotPerLane + 4;

// Hot weights as 4 signed base-128 digits of a 28-bit fixed-point value
// (w ~= S * 2^-27 * (d0 2^21 + d1 2^14 + d2 2^7 + d3), S = max |w_hot| of
// the pass): the forward dot of a lane's 32 hot counts is 32
// v_dot4_i32_iu8 (4 counts x 4 digits each, exact int32), not 96 VALU ops
// of extract / convert / fma.  Quantisation error <= S * 2^-28 per weight.
// LDS per lane quarter t (kHotLdsStride dwords): dword (d*4 + q)*2 + half
// packs digit d of the 4 hot ids held in the even (half 0) / odd (half 1)
// nibbles of the lane's count dword q; dwords 32..35 hold the 4 digit scales.
// (Counts 0..15 are valid signed bytes, so the signed v_dot4_i32_i8 serves.)
__device__ __forceinline__ void nib_split(uint32_t x, uint32_t& lo, uint32_t& hi) {
  lo = x & 0x0F0F0F0Fu;           // nibbles 0,2,4,6 -> bytes 0..3
  hi = (x >> 4) & 0x0F0F0F0Fu;    // nibbles 1,3,5,7 -> bytes 0..3
}

__device__ __forceinline__ float hot_dot(const uint4 hv, const uint32_t* wq) {
  const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w};
  int acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint4 a = reinterpret_cast<const uint4*>(wq)[2 * d];       // q 0,1
    const uint4 b = reinterpret_cast<const uint4*>(wq)[2 * d + 1];   // q 2,3
    const uint32_t dg[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t lo, hi;
      nib_split(hw[q], lo, hi);
      acc[d] = __builtin_amdgcn_sdot4(int(lo), int(dg[2 * q]), acc[d], false);
      acc[d] = __builtin_amdgcn_sdot4(int(hi), int(dg[2 * q + 1]), acc[d], false);
    }
  }
  const float4 sc = reinterpret_cast<const float4*>(wq)[8];
  return float(acc[0]) * sc.x + float(acc[1]) * sc.y + float(acc[2]) * sc.z + float(acc[3]) * sc.w;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// gh[j] accumulates hot ids (2j, 2j+1) of the lane's quarter: counts convert
// straight from bytes (v_cvt_f32_ubyteN) and pairs update with v_pk_fma_f32.
__device__ __forceinline__ void hot_grad(const uint4 hv, float res, f32x2 (&gh)[kHotPerLane / 2]) {
  const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w};
  const f32x2 r2 = {res, res};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t lo, hi;
    nib_split(hw[q], lo, hi);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x2 c = {float((lo >> (8 * i)) & 0xFFu), float((hi >> (8 * i)) & 0xFFu)};
      gh[4 * q + i] = __builtin_elementwise_fma(c, r2, gh[4 * q + i]);
    }
  }
}

// Build the digit table of the pass from the LDS weights (one wave; the
// caller synchronises).  Hot id h: quarter t = h / 32, count dword
// q = (h % 32) / 8, nibble k = h % 8 -> half = k & 1, byte i = k >> 1.
__device__ __forceinline__ void hot_digits(const DevPrepared& p, const float* wl, uint32_t* whl) {
  const int lane = lane_id();
  const float wa = wl[p.hot_slot[lane]], wb = wl[p.hot_slot[lane + kWave]];
  float S = fmaxf(fabsf(wa), fabsf(wb));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) S = fmaxf(S, __shfl_xor(S, off, kWave));
  const float inv = S > 0.f ? 134217728.0f / S : 0.f;   // 2^27 / S
  uint8_t* bytes = reinterpret_cast<uint8_t*>(whl);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int h = lane + u * kWave;
    int32_t W = int32_t(rintf((u ? wb : wa) * inv));
    int32_t dg[4];
#pragma unroll
    for (int d = 3; d > 0; --d) {   // balanced base-128 digits, least significant first
      const int32_t x = ((W + 64) & 127) - 64;
      dg[d] = x;
      W = (W - x) >> 7;
    }
    dg[0] = W;                       // |W| <= 2^27 -> |d0| <= 64
    const int t = h / 32, q = (h % 32) / 8, k = h % 8;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      bytes[(t * kHotLdsStride + (d * 4 + q) * 2 + (k & 1)) * 4 + (k >> 1)] = uint8_t(int8_t(dg[d]));
  }
  if (lane < kLanesPerRow) {
    float* sc = reinterpret_cast<float*>(whl + lane * kHotLdsStride + 32);
    const float s0 = S * (1.0f / 64.0f);   // S * 2^-27 * 2^21
    sc[0] = s0;
    sc[1] = s0 * (1.0f / 128.0f);
    sc[2] = s0 * (1.0f / 16384.0f);
    sc[3] = s0 * (1.0f / 2097152.0f);
  }
}

__device__ __forceinline__ float sgpr_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// wctr: the workgroup's LDS chunk counter, zeroed by hyb_lds_init.
template <bool STATS, bool SAMPLE, int REP>
__device__ __forceinline__ void hyb_pass(const DevSgd& d, const DevPrepared& p, const SgdParams& sp,
                                         const float* wl, unsigned long long* gl, const uint32_t* whl,
                                         float (*hsum)[kHot], double (*wsc)[kPartVals], double* prow,
                                         uint32_t* wctr, uint64_t* tst = nullptr) {
  const int64_t ns = d.ns;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);   // wave-uniform
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  const int rep = lane % REP;
  const int64_t n_kept = p.counters[0];
  const int64_t nch = sp.ablate % 10 == 7 ? 0 : (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;  // 7: fixed cost
  const uint16_t* slot = static_cast<const uint16_t*>(p.slot);
  const uint4* hdense = reinterpret_cast<const uint4*>(p.hot_dense);
  const int32_t* __restrict__ clen8c = p.clen8c;
  const int64_t* __restrict__ cbase = p.cbase;
  // the 4 numeric-feature weights are wave-uniform: SGPRs, not 4 VGPRs (the
  // chunk loop sits at the 128-VGPR limit of 1024-thread workgroups)
  const float w0 = sgpr_f(wl[0]), w1 = sgpr_f(wl[1]), w2 = sgpr_f(wl[2]), w3 = sgpr_f(wl[3]);
  const uint32_t* wq = whl + t * kHotLdsStride;
  f32x2 gh[kHotPerLane / 2];
#pragma unroll
  for (int i = 0; i < kHotPerLane / 2; ++i) gh[i] = f32x2{0.f, 0.f};
  RowAcc acc;
  bool clamped = false;

  // Dynamic chunk assignment inside the workgroup: workgroup b owns chunks
  // b, b + G, b + 2G, ... and its waves take the next one from an LDS
  // counter.  (A static round robin let the oldest waves, which the SIMD
  // arbiter favours, finish ~20 us before the youngest -- the tail then ran
  // at one wave per SIMD.)  The next chunk's index and metadata are fetched
  // one chunk ahead (scalar loads), so the grab costs no memory round trip.
  const int abl = sp.ablate;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t nj = nch > b ? (nch - b + G - 1) / G : 0;
  auto grab = [&]() -> int64_t {
    uint32_t j = 0;
    if (lane == 0) j = atomicAdd(wctr, 1u);
    return int64_t(__builtin_amdgcn_readfirstlane(__shfl(int(j), 0, kWave)));
  };
  int k = 0;   // chunks this wave took
  int64_t j = grab();
  int32_t L8n = 0;
  int64_t cbn = 0;
  if (j < nj) {
    L8n = clen8c[b + j * G];
    cbn = cbase[b + j * G];
  }
  while (j < nj) {
    const int64_t c = b + j * G;
    const int32_t L8c = L8n;
    const int64_t cb = cbn;
    ++k;
    j = grab();
    if (j < nj) {
      L8n = clen8c[b + j * G];
      cbn = cbase[b + j * G];
    }
    const int64_t pos = c * kRowsPerChunk + r;
    const int64_t off = cb * kChunkStride + lane * kGroup;
    const RowIn ri = row_in(p, pos);
    if (L8c >= 0) {
      const uint4 hv = hdense[c * kWave + lane];
      // cold stream: L8c groups of kColdGroup slots per lane (hot_split.hip)
      const uint16_t* sl = p.cslot + cb * kChunkStride + lane * kColdGroup;
      const bool reg = L8c <= kMaxColdGroups;
      uint2 v[kMaxColdGroups];
      if (reg) {
#pragma unroll
        for (int g = 0; g < kMaxColdGroups; ++g)
          if (g < L8c) v[g] = *reinterpret_cast<const uint2*>(sl + int64_t(g) * kColdStride);
      }
      if (abl == 6) {  // loads only: memory floor of the chunk stream
        uint32_t x = hv.x ^ hv.y ^ hv.z ^ hv.w ^ __float_as_uint(ri.y + ri.n0 + ri.n1 + ri.n2 + ri.n3);
        if (reg) {
#pragma unroll
          for (int g = 0; g < kMaxColdGroups; ++g)
            if (g < L8c) x ^= v[g].x ^ v[g].y;
        }
        acc.loss += float(x & 1u);
        continue;
      }
      // ablate 4: no hot dot (counts still loaded)
      float d0 = abl == 4 ? __uint_as_float(hv.x & 1u) : hot_dot(hv, wq), d1 = 0.f;
      if (reg) {
#pragma unroll
        for (int g = 0; g < kMaxColdGroups; ++g)
          if (g < L8c) {
            uint32_t s[4];
            unpack4(v[g], s);
            d0 += wl[s[0]] + wl[s[2]];
            d1 += wl[s[1]] + wl[s[3]];
          }
      } else {
        for (int32_t g = 0; g < L8c; ++g) {
          uint32_t s[4];
          unpack4(*reinterpret_cast<const uint2*>(sl + int64_t(g) * kColdStride), s);
          d0 += wl[s[0]] + wl[s[2]];
          d1 += wl[s[1]] + wl[s[3]];
        }
      }
      float dot = d0 + d1;
      dot += __shfl_xor(dot, 1, kWave);
      dot += __shfl_xor(dot, 2, kWave);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
      if (res != 0.f) {
        // opaque copy: re-extract the counts instead of keeping 32 converted
        // floats live across the residual (register pressure)
        uint4 hg = hv;
        asm volatile("" : "+v"(hg.x), "+v"(hg.y), "+v"(hg.z), "+v"(hg.w));
        if (abl != 1 && abl != 3) hot_grad(hg, res, gh);   // ablate 3: no hot grad
        if (abl == 1 || abl == 5) continue;                 // 1/5: no cold scatter
        const unsigned long long q = to_fix(res, clamped, sp.fix_lim);
        if (reg) {
#pragma unroll
          for (int g = 0; g < kMaxColdGroups; ++g)
            if (g < L8c) {
              uint32_t s[4];
              unpack4(v[g], s);
#pragma unroll
              for (int e = 0; e < 4; ++e) atomicAdd(&gl[s[e] * REP + rep], q);
            }
        } else {
          for (int32_t g = 0; g < L8c; ++g) {
            uint32_t s[4];
            unpack4(*reinterpret_cast<const uint2*>(sl + int64_t(g) * kColdStride), s);
#pragma unroll
            for (int e = 0; e < 4; ++e) atomicAdd(&gl[s[e] * REP + rep], q);
          }
        }
      }
    } else {  // plain layout: every entry (hot ones too) through the LDS gradient
      const int32_t L8 = p.clen8[c];
      const uint16_t* sl = slot + off;
      float dot = 0.f;
      for (int32_t g = 0; g < L8; ++g) {
        uint32_t s[8];
        unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
        for (int k = 0; k < 8; ++k) dot += wl[s[k]];
      }
      dot += __shfl_xor(dot, 1, kWave);
      dot += __shfl_xor(dot, 2, kWave);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
      if (res != 0.f) {
        const unsigned long long q = to_fix(res, clamped, sp.fix_lim);
        for (int32_t g = 0; g < L8; ++g) {
          uint32_t s[8];
          unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
          for (int k = 0; k < 8; ++k) atomicAdd(&gl[s[k] * REP + rep], q);
        }
      }
    }
  }

  if (tst) tst[3] = __builtin_amdgcn_s_memrealtime();
  if (d.tdbg && blockIdx.x == 0 && lane == 0) {   // per-wave end of the chunk loop (WG 0)
    uint64_t* we = d.tdbg + 4096 + int64_t(sp.iteration) * 32 + w * 2;
    we[0] = __builtin_amdgcn_s_memrealtime();
    we[1] = uint64_t(k);
  }
  if (__any(clamped) && lane == 0) d.state[7] = 1.0;
  // hot gradient: sum the 16 lanes of each quarter t (per wave), into LDS
  // per 16-lane row (DPP), the four row partials of each hot id go to LDS
  // and the slot loop adds the 4 x 16 of them
  float* hrow = hsum[w * kHotRows + lane / 16];
#pragma unroll
  for (int i = 0; i < kHotPerLane; ++i) {
    const float v = row_sum_mod4((i & 1) ? gh[i >> 1].y : gh[i >> 1].x);
    if ((lane & 15) < kLanesPerRow) hrow[kHotPerLane * (lane & 3) + i] = v;
  }
  if (tst) tst[4] = __builtin_amdgcn_s_memrealtime();
  part_scalars<STATS, SAMPLE>(d, acc, wsc, prow);   // includes the block barrier
  if (tst) tst[5] = __builtin_amdgcn_s_memrealtime();
  const int64_t hi = kNumNumeric + d.n_unique;      // pads are never flushed
  for (int64_t s = kNumNumeric + threadIdx.x; s < ns; s += kIterBlock) {
    double v = 0.0;
    if (s < hi) {
      v = part_slot<REP>(gl, s);
      const uint32_t h = p.hot_of[s];
      if (h != 0xFFu) {
        double hv = 0.0;
        for (int k = 0; k < kIterBlock / kWave * kHotRows; ++k) hv += double(hsum[k][h]);
        v += hv;
      }
    }
    prow[s] = v;
  }
}


// Weights -> LDS (fp32 compact weights, hot weights in hot order) and a
// zeroed fixed-point gradient; ends with a block barrier.
// Loads of data other workgroups wrote during the persistent kernel:
// device-scope (sc1) so they are not served from this CU's (non-coherent) L1.
template <typename T>
__device__ __forceinline__ T ld_coh(const T* ptr) {
  return __hip_atomic_load(ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Slots >= hi (pads) get weight 0 whatever wsrc holds there.
template <int REP>
__device__ __forceinline__ void hyb_lds_init(const DevPrepared& p, const float* wsrc, int64_t ns,
                                             int64_t hi, float* wl, unsigned long long* gl, uint32_t* whl,
                                             uint32_t* wctr) {
  if (threadIdx.x == 0) *wctr = 0u;
  for (int64_t s = threadIdx.x; s < ns; s += kIterBlock) wl[s] = s < hi ? ld_coh(wsrc + s) : 0.f;
  for (int64_t s = threadIdx.x; s < ns * REP; s += kIterBlock) gl[s] = 0ull;
  __syncthreads();
  if (threadIdx.x < kWave) hot_digits(p, wl, whl);
  __syncthreads();
}

template <bool STATS, bool SAMPLE, int REP>
__global__ __launch_bounds__(kIterBlock) void k_sgd_iter_hyb(DevSgd d, DevPrepared p, SgdParams sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double wsc[kIterBlock / kWave][kPartVals];
  __shared__ float hsum[kIterBlock / kWave * kHotRows][kHot];
  __shared__ __attribute__((aligned(16))) uint32_t whl[kLanesPerRow * kHotLdsStride];
  __shared__ int stop_flag;
  __shared__ uint32_t wctr;
  uint64_t* tst = nullptr;
  if (d.tdbg && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    tst = d.tdbg + (int64_t(sp.iteration) * 2 + (blockIdx.x == 0 ? 0 : 1)) * 8;
  if (tst) tst[0] = __builtin_amdgcn_s_memrealtime();
  if (sgd_stop(d, sp, &stop_flag)) return;
  if (tst) tst[1] = __builtin_amdgcn_s_memrealtime();
  float* wl = lds;
  unsigned long long* gl = reinterpret_cast<unsigned long long*>(lds + d.ns);
  hyb_lds_init<REP>(p, d.wc32, d.ns, kNumNumeric + d.n_unique, wl, gl, whl, &wctr);
  if (tst) tst[2] = __builtin_amdgcn_s_memrealtime();
  hyb_pass<STATS, SAMPLE, REP>(d, p, sp, wl, gl, whl, hsum, wsc, d.part + int64_t(blockIdx.x) * d.pstride, &wctr, tst);
  if (tst) tst[6] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------
// Persistent GD loop (single GPU, hybrid layout, iterations 2..N).
//
// One workgroup per CU for the whole loop, so the ~25 us of per-iteration
// launch / prologue / epilogue / update-kernel overhead of the multi-kernel
// path disappears.  Per iteration:
//   pass      gradient over the workgroup's chunks -> partial row (UC memory)
//   barrier A
//   update    workgroup b owns ~ns/G columns: fixed-order sum of the G
//             partial rows, SimpleUpdater, fp32 copy -> UC memory, norms
//   barrier B
//   converged?  every workgroup sums the G norm partials in the same order
//             (identical verdicts), MLlib test as k_sgd_update/sgd_stop.
// Cross-workgroup data lives in uncached (hipDeviceMallocUncached) memory,
// so the barriers need no L2 write-back / invalidate (a device-scope fence
// on MI355X writes back the XCD's whole L2 -- measured, see profiles/).
// The grid barrier is hierarchical: one arrival counter per XCD group
// (blockIdx % 8), the last arriver of a group bumps the global counter, the
// last group publishes the generation.  Spins are bounded: a stuck barrier
// raises bar->err and every workgroup leaves the loop.
// ---------------------------------------------------------------------------
__device__ bool grid_sync(GridBar* gb, uint32_t target, int* flag) {
  __builtin_amdgcn_s_waitcnt(0);   // this thread's UC stores have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t G = gridDim.x, x = blockIdx.x & 7u;
    const uint32_t nx = (G - x + 7u) / 8u;
    const uint32_t ng = G < 8u ? G : 8u;
    if (atomicAdd(&gb->cnt[x * 16], 1u) + 1u == target * nx)
      if (atomicAdd(&gb->gcnt, 1u) + 1u == target * ng)
        __hip_atomic_store(&gb->gen, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    uint32_t spins = 0;
    while (__hip_atomic_load(&gb->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(&gb->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 25)) {
        __hip_atomic_store(&gb->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *flag = ok;
  }
  __syncthreads();
  return *flag != 0;
}

template <int REP>
__global__ __launch_bounds__(kIterBlock) void k_sgd_gd_hyb(DevSgd d, DevPrepared p, SgdParams sp,
                                                           DevCoh coh, int it_first) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double wsc[kIterBlock / kWave][kPartVals];
  __shared__ float hsum[kIterBlock / kWave * kHotRows][kHot];
  __shared__ __attribute__((aligned(16))) uint32_t whl[kLanesPerRow * kHotLdsStride];
  __shared__ double red[kIterBlock / kWave][2];
  __shared__ int flag, conv_sh;
  __shared__ uint32_t wctr;
  const int64_t ns = d.ns, hi = kNumNumeric + d.n_unique;
  float* wl = lds;
  unsigned long long* gl = reinterpret_cast<unsigned long long*>(lds + ns);
  const int G = int(gridDim.x), b = int(blockIdx.x);
  const int lane = lane_id(), w = int(threadIdx.x) / kWave;
  const double m = d.state[5];
  double rest = d.state[4] - d.state[6];
  if (rest < 0.0) rest = 0.0;
  // update columns of this workgroup: index k in [0, hi] -> column k (< hi) or the loss (ns)
  const int64_t nk = hi + 1, cpw = (nk + G - 1) / G;
  const int64_t k0 = int64_t(b) * cpw, k1 = k0 + cpw < nk ? k0 + cpw : nk;
  double* prow = coh.part + int64_t(b) * d.pstride;
  uint32_t gen = 0;
  int it = it_first;
  uint64_t* tst = nullptr;
  auto stamp = [&](int k) {
    if (tst && b == 0 && threadIdx.x == 0) tst[k] = __builtin_amdgcn_s_memrealtime();
  };
  for (;; ++it) {
    sp.iteration = it;
    tst = coh.tdbg ? coh.tdbg + int64_t(it) * 8 : nullptr;
    stamp(0);
    hyb_lds_init<REP>(p, it == it_first ? d.wc32 : coh.w32, ns, hi, wl, gl, whl, &wctr);
    stamp(1);
    hyb_pass<false, false, REP>(d, p, sp, wl, gl, whl, hsum, wsc, prow, &wctr);
    stamp(2);
    if (!grid_sync(coh.bar, ++gen, &flag)) break;
    stamp(3);
    // ---- update of this workgroup's columns (one wave per column)
    const double alpha = sp.step_size / sqrt(double(it));
    double ds = 0.0, ws = 0.0;
    for (int64_t k = k0 + w; k < k1; k += kIterBlock / kWave) {
      const int64_t col = k < hi ? k : ns;
      // the G partials of this column, all loads in flight at once
      double a[kMaxPersistGrid / kWave];
#pragma unroll
      for (int q = 0; q < kMaxPersistGrid / kWave; ++q) {
        const int j = lane + q * kWave;
        a[q] = j < G ? ld_coh(coh.part + int64_t(j) * d.pstride + col) : 0.0;
      }
      double g = 0.0;
#pragma unroll
      for (int q = 0; q < kMaxPersistGrid / kWave; ++q) g += a[q];
      g = wave_sum(g);
      if (lane == 0) {
        if (col < hi) {
          const double step = alpha * (g / m);
          const double wn = d.wc64[col] - step;
          d.wc64[col] = wn;
          coh.w32[col] = float(wn);
          ds += step * step;
          ws += wn * wn;
        } else {
          d.loss_hist[it] = g / m;
        }
      }
    }
    if (lane == 0) {
      red[w][0] = ds;
      red[w][1] = ws;
    }
    __syncthreads();
    double* nrm = coh.norms + int64_t(it & 1) * 2 * G;
    if (threadIdx.x < 2) {
      double t = 0.0;
      for (int k = 0; k < kIterBlock / kWave; ++k) t += red[k][threadIdx.x];
      nrm[2 * b + threadIdx.x] = t;
    }
    stamp(4);
    if (!grid_sync(coh.bar, ++gen, &flag)) break;
    stamp(5);
    // ---- convergence (every workgroup, same fixed-order sums)
    if (threadIdx.x < kWave) {
      double dsum = 0.0, wsum = 0.0;
      for (int j = lane; j < G; j += kWave) {
        dsum += ld_coh(nrm + 2 * j);
        wsum += ld_coh(nrm + 2 * j + 1);
      }
      dsum = wave_sum(dsum);
      wsum = wave_sum(wsum);
      const double wnorm = sqrt(wsum + rest);
      const bool conv = sqrt(dsum) < sp.tol * (wnorm > 1.0 ? wnorm : 1.0);   // it >= 2: second update on
      if (threadIdx.x == 0) conv_sh = conv ? 1 : 0;
    }
    __syncthreads();
    stamp(6);
    const bool conv = conv_sh != 0;
    if (conv || it >= sp.num_iterations) {
      if (b == 0 && threadIdx.x == 0) {
        d.state[0] = 1.0;
        if (conv) d.state[1] = 1.0;
        d.state[2] = double(it);
        d.state[3] = double(it);
      }
      break;
    }
  }
  if (b == 0 && threadIdx.x == 0 &&
      __hip_atomic_load(&coh.bar->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
    d.state[7] = 2.0;   // barrier timeout: reported by the host
}

// Generic path: any slot width, weights read from global (L2), gradient by
// global fp64 atomics.  Used when the active set exceeds LDS.
template <typename SlotT, bool STATS, bool SAMPLE>
__global__ __launch_bounds__(kBlock) void k_sgd_iter_global(DevSgd d, DevPrepared p, SgdParams sp) {
  __shared__ double scratch[kBlock / kWave];
  __shared__ int stop_flag;
  if (sgd_stop(d, sp, &stop_flag)) return;
  const float* w = d.wc32;
  const int lane = lane_id();
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t wave = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t nwaves = int64_t(gridDim.x) * (kBlock / kWave);
  const SlotT* slot = static_cast<const SlotT*>(p.slot);
  const float w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
  RowAcc acc;
  for (int64_t c = wave; c < nch; c += nwaves) {
    const int32_t L8 = p.clen8[c];
    const SlotT* sl = slot + p.cbase[c] * kChunkStride + lane * kGroup;
    const int64_t pos = c * kRowsPerChunk + r;
    float dot = 0.f;
    for (int32_t g = 0; g < L8; ++g) {
      uint32_t s[8];
      SlotLoad<SlotT>::load(sl + int64_t(g) * kChunkStride, s);
#pragma unroll
      for (int k = 0; k < 8; ++k) dot += w[s[k]];
    }
    dot += __shfl_xor(dot, 1, kWave);
    dot += __shfl_xor(dot, 2, kWave);
    const float res = row_residual<STATS, SAMPLE>(dot, pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
    if (res != 0.f) {
      for (int32_t g = 0; g < L8; ++g) {
        uint32_t s[8];
        SlotLoad<SlotT>::load(sl + int64_t(g) * kChunkStride, s);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (s[k] >= kNumNumeric && s[k] < kNumNumeric + d.n_unique) atomicAdd(&d.g64[s[k]], double(res));
      }
    }
  }
  flush_scalars<STATS, SAMPLE>(d, acc, scratch, sp.iteration);
}

// LDS bytes of the fast path for a given replication factor.
static int64_t lds_bytes(int64_t ns, int rep) {
  return ns * int64_t(sizeof(float)) + ns * rep * int64_t(sizeof(unsigned long long));
}

// Replication factor for the LDS gradient (0 = does not fit -> global path).
// Replicas of a slot are interleaved (gl[s * REP + lane % REP]) so lanes
// hitting the same hot slot land in different banks.  TWTML_SGD_REP
// overrides the choice (1/2/4/8) for tuning.
static int rep_override() {
  static const int v = [] {
    const char* e = std::getenv("TWTML_SGD_REP");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

int sgd_lds_rep(int64_t ns) {
  const int o = rep_override();
  if ((o == 1 || o == 2 || o == 4 || o == 8) && lds_bytes(ns, o) <= 160 * 1024 - 2048) return o;
  // Measured on MI355X (1M-tweet batch, ~1.4K active slots): bank conflicts
  // on hot slots dominate, so more replicas beat occupancy -- REP 8 at one
  // 512-thread block per CU runs 13% faster than REP 2 at four.
  for (int rep : {8, 4, 2})
    if (lds_bytes(ns, rep) <= 100 * 1024) return rep;
  if (lds_bytes(ns, 1) <= 160 * 1024 - 2048) return 1;
  return 0;
}

bool sgd_hybrid_fits(int64_t ns) {
  const int rep = sgd_lds_rep(ns);
  const int64_t statics = int64_t(kIterBlock / kWave) * (kHot * int64_t(sizeof(float)) + int64_t(sizeof(double)));
  return ns <= kMaxHybridSlots && rep > 0 && lds_bytes(ns, rep) + statics <= 160 * 1024 - 1024;
}

template <bool STATS, bool SAMPLE>
static void launch_iter_t(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, bool u16,
                          int rep, int grid, hipStream_t s) {
  if (u16 && rep > 0 && p.hybrid) {
    const size_t lds = size_t(lds_bytes(d.ns, rep));
#define TWTML_HYB(R) \
  hipLaunchKernelGGL((k_sgd_iter_hyb<STATS, SAMPLE, R>), dim3(grid), dim3(kIterBlock), lds, s, d, p, sp)
    switch (rep) {
      case 8: TWTML_HYB(8); break;
      case 4: TWTML_HYB(4); break;
      case 2: TWTML_HYB(2); break;
      default: TWTML_HYB(1); break;
    }
#undef TWTML_HYB
  } else if (u16 && rep > 0) {
    const size_t lds = size_t(lds_bytes(d.ns, rep));
#define TWTML_ITER(R, C) \
  hipLaunchKernelGGL((k_sgd_iter_lds<STATS, SAMPLE, R, C>), dim3(grid), dim3(kIterBlock), lds, s, d, p, sp)
    const bool cnt = p.dedup != 0;
    switch (rep) {
      case 8: if (cnt) TWTML_ITER(8, true); else TWTML_ITER(8, false); break;
      case 4: if (cnt) TWTML_ITER(4, true); else TWTML_ITER(4, false); break;
      case 2: if (cnt) TWTML_ITER(2, true); else TWTML_ITER(2, false); break;
      default: if (cnt) TWTML_ITER(1, true); else TWTML_ITER(1, false); break;
    }
#undef TWTML_ITER
  } else if (u16) {
    hipLaunchKernelGGL((k_sgd_iter_global<uint16_t, STATS, SAMPLE>), dim3(grid * 2), dim3(kBlock), 0, s, d, p, sp);
  } else {
    hipLaunchKernelGGL((k_sgd_iter_global<uint32_t, STATS, SAMPLE>), dim3(grid * 2), dim3(kBlock), 0, s, d, p, sp);
  }
}

// Workgroups of the (non-stats, non-sampled) LDS iteration kernel that fit a
// CU at once: LDS *and* registers (a 1024-thread workgroup at 122-128 VGPRs
// is one per CU -- an LDS-only estimate launched 2-3 rounds of workgroups
// for mid-sized active sets, each round paying the full per-iteration
// overhead and adding partial rows).
static int iter_blocks_per_cu(int64_t ns, int rep, bool hybrid) {
  const size_t lds = size_t(lds_bytes(ns, rep));
  int n = 0;
  hipError_t e = hipSuccess;
#define TWTML_OCC(K) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, K, kIterBlock, lds)
  switch (rep) {
    case 8: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 8>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 8, false>)); break;
    case 4: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 4>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 4, false>)); break;
    case 2: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 2>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 2, false>)); break;
    default: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 1>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 1, false>)); break;
  }
#undef TWTML_OCC
  if (e != hipSuccess || n < 1) {
    (void)hipGetLastError();
    n = 1;
  }
  return n;
}

int sgd_iter_grid(int64_t ns, int64_t n_kept, int num_cu, bool hybrid) {
  const int rep = sgd_lds_rep(ns);
  int per_cu = 2;
  if (rep > 0) per_cu = std::min(4, iter_blocks_per_cu(ns, rep, hybrid));
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t waves_per_wg = kIterBlock / kWave;
  int64_t g = std::min<int64_t>(int64_t(num_cu) * per_cu, (nch + waves_per_wg - 1) / waves_per_wg);
  return int(g < 1 ? 1 : g);
}

void launch_sgd_iter(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, int64_t /*groups*/,
                     bool u16, int grid, hipStream_t s) {
  const int rep = u16 ? sgd_lds_rep(d.ns) : 0;
  const bool stats = sp.iteration == 1;
  const bool sample = sp.sample != 0;
  if (stats && sample) launch_iter_t<true, true>(d, p, sp, u16, rep, grid, s);
  else if (stats) launch_iter_t<true, false>(d, p, sp, u16, rep, grid, s);
  else if (sample) launch_iter_t<false, true>(d, p, sp, u16, rep, grid, s);
  else launch_iter_t<false, false>(d, p, sp, u16, rep, grid, s);
}

int sgd_partials(int64_t ns, bool u16, int grid) {
  return (u16 && sgd_lds_rep(ns) > 0) ? grid : 0;
}

// Persistent loop: the grid it needs (0 = not applicable: generic / plain
// layout, sampling, or a workgroup per CU does not fit).
int sgd_persistent_grid(const DevSgd& d, const DevPrepared& p, bool u16, bool sample, int num_cu) {
  if (!u16 || sample || !p.hybrid) return 0;
  const int rep = sgd_lds_rep(d.ns);
  if (rep <= 0) return 0;
  const size_t lds = size_t(lds_bytes(d.ns, rep));
  int per_cu = 0;
  hipError_t e = hipSuccess;
  switch (rep) {
    case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sgd_gd_hyb<8>, kIterBlock, lds); break;
    case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sgd_gd_hyb<4>, kIterBlock, lds); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sgd_gd_hyb<2>, kIterBlock, lds); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sgd_gd_hyb<1>, kIterBlock, lds); break;
  }
  if (e != hipSuccess || per_cu < 1 || num_cu > kMaxPersistGrid) return 0;
  return num_cu;   // one workgroup per CU (co-resident by construction, cooperative launch checks)
}

void launch_sgd_persistent(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, const DevCoh& coh,
                           int it_first, int grid, hipStream_t s) {
  const int rep = sgd_lds_rep(d.ns);
  const unsigned lds = unsigned(lds_bytes(d.ns, rep));
  SgdParams spc = sp;
  DevSgd dc = d;
  DevPrepared pc = p;
  DevCoh cc = coh;
  int itf = it_first;
  void* args[] = {&dc, &pc, &spc, &cc, &itf};
  const void* fn = nullptr;
  switch (rep) {
    case 8: fn = reinterpret_cast<const void*>(k_sgd_gd_hyb<8>); break;
    case 4: fn = reinterpret_cast<const void*>(k_sgd_gd_hyb<4>); break;
    case 2: fn = reinterpret_cast<const void*>(k_sgd_gd_hyb<2>); break;
    default: fn = reinterpret_cast<const void*>(k_sgd_gd_hyb<1>); break;
  }
  TWTML_HIP_CHECK(hipLaunchCooperativeKernel(fn, dim3(grid), dim3(kIterBlock), args, lds, s));
}

// ---------------------------------------------------------------------------
// Per-iteration protocol (no grid-wide barrier, no contended atomics):
//
//   k_sgd_iter_*  (iteration i)  prologue: converged after update i-1?  ->
//                 every workgroup decides from record i-1 (fixed-order sums,
//                 so all workgroups -- and all DP ranks -- agree); workgroup
//                 0 publishes state[0..1] and the host flag.  Then one
//                 partial gradient row per workgroup.
//   [k_sgd_reduce + RCCL all-reduce of g64 when DP]
//   k_sgd_update  (iteration i)  multi-workgroup: sums the partial rows of
//                 64 columns (world 1) or reads the all-reduced g64,
//                 SimpleUpdater on them, per-workgroup ||dw||^2, ||w||^2
//                 into record i.
//   k_sgd_finish  after the loop: convergence of the last update.
//
// MLlib semantics: the update of iteration i is applied, then
// ||w_i - w_{i-1}|| < tol * max(||w_i||, 1) (from the second update on) ends
// the loop, i.e. the weights after the converging update are kept.
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// SimpleUpdater (fp64 master weights), one wave per column: lane j sums the
// partial rows j, j + 64, ... (all loads in flight) and a DPP wave sum
// gives the column (fixed order); 16 columns per 1024-thread workgroup, so
// a ~1.4K-slot batch spreads over ~90 CUs instead of 23.
// nparts > 0: the column gradients are the sums of the partial rows (single
// GPU); nparts == 0: g64 holds them (all-reduced, or the generic path).
// ---------------------------------------------------------------------------
constexpr int kUpdCols = 1024 / kWave;   // columns (waves) per workgroup

__device__ __forceinline__ double part_col_wave(const DevSgd& d, int64_t col, int nparts) {
  const int lane = lane_id();
  const double* src = d.part + col;
  const int64_t ps = d.pstride;
  double a[kMaxPersistGrid / kWave];
#pragma unroll
  for (int q = 0; q < kMaxPersistGrid / kWave; ++q) {
    const int g = lane + q * kWave;
    a[q] = g < nparts ? src[int64_t(g) * ps] : 0.0;
  }
  double t = 0.0;
  for (int g0 = kMaxPersistGrid; g0 < nparts; g0 += kWave)   // grids beyond 512 (not launched today)
    if (g0 + lane < nparts) t += src[int64_t(g0 + lane) * ps];
#pragma unroll
  for (int q = 0; q < kMaxPersistGrid / kWave; ++q) t += a[q];
  return wave_sum(t);
}

__global__ __launch_bounds__(1024) void k_sgd_update(DevSgd d, SgdParams sp, int nparts) {
  __shared__ double wsc[kUpdCols][2];
  __shared__ double m_sh;
  if (d.state[0] != 0.0) return;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  const int it = sp.iteration;
  const int64_t ns = d.ns, hi = kNumNumeric + d.n_unique;
  const int64_t ncols = ns + kPartVals - kNumNumeric;
  // m: global kept rows, or the sampled row count of this iteration
  if (tid < kWave) {
    double m = d.state[5];
    if (sp.sample) {
      m = *sgd_red_m(d, it);
      if (nparts > 0) {
        double t = 0.0;
        for (int g = tid; g < nparts; g += kWave) t += d.part[int64_t(g) * d.pstride + ns + 1];
        m += wave_sum(t);
      }
    }
    if (tid == 0) m_sh = m;
  }
  __syncthreads();
  const double m = m_sh;
  const double alpha = sp.step_size / sqrt(double(it));
  double ds = 0.0, ws = 0.0;
  for (int64_t col = int64_t(blockIdx.x) * kUpdCols + w; col < ncols; col += int64_t(gridDim.x) * kUpdCols) {
    double g = col <= ns ? d.g64[col] : 0.0;   // wave-uniform load
    if (nparts > 0) g += part_col_wave(d, col, nparts);
    if (lane == 0) {
      if (col < hi) {
        if (m > 0.0) {
          const double step = alpha * (g / m);
          const double wn = d.wc64[col] - step;
          d.wc64[col] = wn;
          d.wc32[col] = float(wn);
          ds += step * step;
          ws += wn * wn;
        }
        d.g64[col] = 0.0;
      } else if (col == ns) {
        if (m > 0.0) d.loss_hist[it] = g / m;
        d.g64[ns] = 0.0;
      } else if (col >= ns + 2 && nparts > 0) {
        d.stats[col - ns - 2] += g;     // batch stats (iteration 1, single GPU)
      }
    }
  }
  if (lane == 0) {
    wsc[w][0] = ds;
    wsc[w][1] = ws;
  }
  __syncthreads();
  double* rec = sgd_rec(d, it);
  if (tid < 2) {
    double t = 0.0;
    for (int k = 0; k < kUpdCols; ++k) t += wsc[k][tid];
    rec[kRecHead + 2 * blockIdx.x + tid] = t;
  }
  if (blockIdx.x == 0 && tid == 0) {
    const double nupd = (it > 1 ? sgd_rec(d, it - 1)[0] : 0.0) + (m > 0.0 ? 1.0 : 0.0);
    rec[0] = nupd;
    rec[1] = m;
    rec[2] = double(gridDim.x);
    d.state[2] = nupd;
    d.state[3] = double(it);
    *sgd_red_m(d, it + 1) = 0.0;      // the next iteration's sampled count accumulates from 0
  }
}

void launch_sgd_update(const DevSgd& d, const SgdParams& sp, int nparts, hipStream_t s) {
  const int64_t tiles = (d.ns + kPartVals - kNumNumeric + kUpdCols - 1) / kUpdCols;
  const int grid = int(std::min<int64_t>(tiles, kMaxUpdGrid));
  hipLaunchKernelGGL(k_sgd_update, dim3(grid), dim3(1024), 0, s, d, sp, nparts);
}

// Cross-workgroup reduction of the partial rows (DP: before the all-reduce)
// into g64 (+ loss, sampled count, batch stats): one wave per column, fixed
// summation order.
__global__ __launch_bounds__(1024) void k_sgd_reduce(DevSgd d, SgdParams sp) {
  if (d.state[0] != 0.0) return;
  const int64_t ncols = d.ns + kPartVals - kNumNumeric;
  const int64_t col = int64_t(blockIdx.x) * kUpdCols + threadIdx.x / kWave;
  if (col >= ncols) return;   // wave-uniform
  const double v = part_col_wave(d, col, d.nparts);
  if (lane_id() == 0) {
    if (col <= d.ns) d.g64[col] = v;                     // slots, then the loss at [ns]
    else if (col == d.ns + 1) *sgd_red_m(d, sp.iteration) = v;   // sampled row count
    else d.stats[col - d.ns - 2] += v;                   // batch stats (iteration 1)
  }
}

void launch_sgd_reduce(const DevSgd& d, const SgdParams& sp, hipStream_t s) {
  if (d.nparts <= 0) return;
  const int grid = int((d.ns + kPartVals - kNumNumeric + kUpdCols - 1) / kUpdCols);
  hipLaunchKernelGGL(k_sgd_reduce, dim3(grid), dim3(1024), 0, s, d, sp);
}

// Convergence of the last update (the loop ended without a prologue seeing it).
__global__ void k_sgd_finish(DevSgd d, SgdParams sp) {
  if (threadIdx.x >= kWave || d.state[0] != 0.0) return;
  const int last = int(d.state[3]);
  const bool conv = last >= 1 && sgd_converged_wave(d, last, sp.tol);
  if (threadIdx.x == 0) {
    d.state[0] = 1.0;
    if (conv) d.state[1] = 1.0;
  }
}

void launch_sgd_finish(const DevSgd& d, const SgdParams& sp, hipStream_t s) {
  hipLaunchKernelGGL(k_sgd_finish, dim3(1), dim3(kWave), 0, s, d, sp);
}

// ---------------------------------------------------------------------------
// Gather / scatter between full-width fp64 weights and the compact space.
// ---------------------------------------------------------------------------
// Squared norms are reduced deterministically: each block writes its partial
// to d.nrm[blockIdx], one wave adds the partials in a fixed order (DP ranks
// hold identical weights, so their convergence verdicts must match bit for
// bit; float atomics would add in arrival order).
// mode 0: out = sum; 1: out = |w_rest|^2 (state[4] - state[6]) + sum; 2: out = state[4]
__global__ void k_norm_sum(const double* parts, int n, double* out, const double* state, int mode) {
  double acc = 0.0;
  for (int k = lane_id(); k < n; k += kWave) acc += parts[k];
  acc = wave_sum(acc);
  if (threadIdx.x == 0) {
    double base = 0.0;
    if (mode == 1) {             // rest of the previous batch + active part
      base = state[4] - state[6];
      if (base < 0.0) base = 0.0;
    }
    *out = mode == 2 ? state[4] : base + acc;
  }
}

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
    d.g64[s] = 0.0;
    acc += v * v;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) d.nrm[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void k_norm2(const double* v, int64_t n, double* parts) {
  __shared__ double scratch[kBlock / kWave];
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    acc += v[i] * v[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) parts[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void k_scatter_w(DevSgd d, const int32_t* uniq) {
  __shared__ double scratch[kBlock / kWave];
  double acc = 0.0;
  for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < kNumNumeric + d.n_unique;
       s += int64_t(gridDim.x) * kBlock) {
    const double v = d.wc64[s];
    if (s < kNumNumeric) d.w64[d.F + s] = v;
    else d.w64[uniq[s - kNumNumeric]] = v;
    acc += v * v;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) d.nrm[blockIdx.x] = acc;
}

static int gather_grid(const DevSgd& d) { return std::max(1, std::min(ceil_div(d.ns, kBlock), kNormParts)); }
static int scatter_grid(const DevSgd& d) {
  return std::max(1, std::min(ceil_div(kNumNumeric + d.n_unique, kBlock), kNormParts));
}

void launch_gather_w(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  const int grid = gather_grid(d);
  hipLaunchKernelGGL(k_gather_w, dim3(grid), dim3(kBlock), 0, s, d, p.uniq);
  hipLaunchKernelGGL(k_norm_sum, dim3(1), dim3(kWave), 0, s, d.nrm, grid, &d.state[6], d.state, 0);
}

void launch_norm2(const double* v, int64_t n, double* out, const DevSgd& d, hipStream_t s) {
  int grid = ceil_div(n, kBlock * 8);
  if (grid > kNormParts) grid = kNormParts;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_norm2, dim3(grid), dim3(kBlock), 0, s, v, n, d.nrm);
  hipLaunchKernelGGL(k_norm_sum, dim3(1), dim3(kWave), 0, s, d.nrm, grid, out, d.state, 0);
}

void launch_scatter_w(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  hipLaunchKernelGGL(k_scatter_w, dim3(scatter_grid(d)), dim3(kBlock), 0, s, d, p.uniq);
}

void launch_norm_next(const DevSgd& d, bool trained, hipStream_t s) {
  hipLaunchKernelGGL(k_norm_sum, dim3(1), dim3(kWave), 0, s, d.nrm, trained ? scatter_grid(d) : 0,
                     d.wnorm_next, d.state, trained ? 1 : 2);
}

__global__ void k_norm_carry(DevSgd d) {
  if (threadIdx.x == 0) d.state[4] = *d.wnorm_next;
}

void launch_norm_carry(const DevSgd& d, hipStream_t s) {
  hipLaunchKernelGGL(k_norm_carry, dim3(1), dim3(kWave), 0, s, d);
}

// Per-batch SGD state in one launch: state (m = global kept rows at [5]),
// batch stats, sampled counts, the loss slot g64[ns] and the loss history.
__global__ void k_batch_init(DevSgd d, double m_global, int n_loss) {
  const int i = threadIdx.x;
  if (i < 8) {
    d.state[i] = i == 5 ? m_global : 0.0;
    d.stats[i] = 0.0;
  }
  if (i < 4) d.red64[i] = 0.0;
  if (i == 0) d.g64[d.ns] = 0.0;
  for (int k = i; k < n_loss; k += blockDim.x) d.loss_hist[k] = 0.0;
}

void launch_batch_init(const DevSgd& d, double m_global, int n_loss, hipStream_t s) {
  hipLaunchKernelGGL(k_batch_init, dim3(1), dim3(256), 0, s, d, m_global, n_loss);
}

}  // namespace twtml
