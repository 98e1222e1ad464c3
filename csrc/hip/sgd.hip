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
#include <stdexcept>

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
// Far gradients (tiered layout) sum over all of a slot's entries in the
// batch (all ranks): a coarser 2^-16 scale and a clamp from the batch's
// entry count keep those int64 sums from overflowing (SgdParams::far_lim).
constexpr float kFarScale = 65536.0f;           // 2^16
constexpr double kFarInv = 1.0 / 65536.0;

// Iteration record i (k_sgd_update -> convergence test) and the sampled row
// count of iteration i (double-buffered by parity: iteration i+1's count is
// zeroed while iteration i's is still being read).
__device__ __forceinline__ double* sgd_rec(const DevSgd& d, int it) { return d.itrec + int64_t(it) * kRecStride; }
__device__ __forceinline__ double* sgd_red_m(const DevSgd& d, int it) { return d.red64 + 2 * (it & 1) + 1; }

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
    prow[tid < kNumNumeric ? int64_t(tid) : d.nl + (tid - kNumNumeric)] = t;
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

float sgd_far_limit(int64_t entries_total) {
  const double e = double(entries_total < 1 ? 1 : entries_total);
  return float(std::min(double(kFixClamp) * double(kFarScale), 4.611686018427388e18 / e) * 0.999);
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
// DP ranks only skip the pass on their own verdict (state[8] = iteration):
// k_sgd_reduce puts rank 0's into the gradient all-reduce and k_sgd_update
// acts on the agreed value.
__device__ bool sgd_stop(const DevSgd& d, const SgdParams& sp, int* flag) {
  if (threadIdx.x < kWave) {
    const bool done = d.state[0] != 0.0;
    bool stop = done;
    if (!done && sp.iteration > 1) {
      stop = sgd_converged_wave(d, sp.iteration - 1, sp.tol);
      if (stop && blockIdx.x == 0 && threadIdx.x == 0) {
        if (!sp.dp) {
          d.state[0] = 1.0;
          d.state[1] = 1.0;
        } else {
          // DP: this rank skips the pass (identical weights -> every rank
          // does); the agreed verdict in k_sgd_update ends the batch
          d.state[8] = double(sp.iteration);
        }
      }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && d.host_flags && sp.iteration > 1 && !sp.dp) {
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
  const int64_t ns = d.nl;        // multiple of 64 (== d.ns: the plain path is never tiered)
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
// TIERED: the chunk's far entries (p.fslot list, weights from global memory)
// join the row dots through the per-wave LDS row sums fdot, and every row's
// residual goes to d.rbuf for the far backward (k_far_grad).
template <bool STATS, bool SAMPLE, int REP, bool TIERED>
__device__ __forceinline__ void hyb_pass(const DevSgd& d, const DevPrepared& p, const SgdParams& sp,
                                         const float* wl, unsigned long long* gl, const uint32_t* whl,
                                         float (*hsum)[kHot], double (*wsc)[kPartVals], double* prow,
                                         uint32_t* wctr, float (*fdot)[kRowsPerChunk], uint64_t* tst = nullptr) {
  const int64_t ns = d.nl;
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
  int32_t L8n = 0, fcn = 0;
  int64_t cbn = 0;
  if (j < nj) {
    L8n = clen8c[b + j * G];
    cbn = cbase[b + j * G];
    if (TIERED) fcn = p.fcount[b + j * G];
  }
  while (j < nj) {
    const int64_t c = b + j * G;
    const int32_t L8c = L8n, fc = fcn;
    const int64_t cb = cbn;
    ++k;
    j = grab();
    if (j < nj) {
      L8n = clen8c[b + j * G];
      cbn = cbase[b + j * G];
      if (TIERED) fcn = p.fcount[b + j * G];
    }
    const int64_t pos = c * kRowsPerChunk + r;
    const int64_t off = cb * kChunkStride + lane * kGroup;
    const RowIn ri = row_in(p, pos);
    // far entries of the chunk: their row sums land in lane t == 0 of the row
    float far = 0.f;
    if (TIERED && fc > 0 && abl != 8) {   // wave-uniform (ablate 8: no far forward)
      float* fd = fdot[w];
      if (lane < kRowsPerChunk) fd[lane] = 0.f;
      wave_lds_sync();
      const uint32_t* fl = p.fslot + cb * kChunkStride;
      for (int32_t k0 = 0; k0 < fc; k0 += kWave)
        if (k0 + lane < fc) {
          const uint32_t e = fl[k0 + lane];
          atomicAdd(&fd[e >> 28], d.wc32[e & 0x0FFFFFFFu]);
        }
      wave_lds_sync();
      if (t == 0) far = fd[r];
    }
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
      float d0 = abl == 4 ? __uint_as_float(hv.x & 1u) : hot_dot(hv, wq), d1 = far;
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
      if (TIERED && t == 0) d.rbuf[pos] = res;
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
      float dot = far;
      for (int32_t g = 0; g < L8; ++g) {
        uint32_t s[8];
        unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
        for (int k = 0; k < 8; ++k) dot += wl[s[k]];
      }
      dot += __shfl_xor(dot, 1, kWave);
      dot += __shfl_xor(dot, 2, kWave);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, w0, w1, w2, w3, acc);
      if (TIERED && t == 0) d.rbuf[pos] = res;
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
  float* hrow = hsum[w];
#pragma unroll
  for (int i = 0; i < kHotPerLane; ++i) {
    float v = row_sum_mod4((i & 1) ? gh[i >> 1].y : gh[i >> 1].x);
    v += __shfl_xor(v, 16, kWave);   // the wave's four 16-lane rows
    v += __shfl_xor(v, 32, kWave);
    if (lane < kLanesPerRow) hrow[kHotPerLane * lane + i] = v;
  }
  if (tst) tst[4] = __builtin_amdgcn_s_memrealtime();
  part_scalars<STATS, SAMPLE>(d, acc, wsc, prow);   // includes the block barrier
  if (tst) tst[5] = __builtin_amdgcn_s_memrealtime();
  const int64_t hi = d.far_base;                    // pads (and far slots) are never flushed
  for (int64_t s = kNumNumeric + threadIdx.x; s < ns; s += kIterBlock) {
    double v = 0.0;
    if (s < hi) {
      v = part_slot<REP>(gl, s);
      const uint32_t h = p.hot_of[s];
      if (h != 0xFFu) {
        double hv = 0.0;
        for (int k = 0; k < kIterBlock / kWave; ++k) hv += double(hsum[k][h]);
        v += hv;
      }
    }
    prow[s] = v;
  }
}


// Weights -> LDS (fp32 compact weights, hot weights in hot order) and a
// zeroed fixed-point gradient; ends with a block barrier.

// Slots >= hi (pads) get weight 0 whatever wsrc holds there.
template <int REP>
__device__ __forceinline__ void hyb_lds_init(const DevPrepared& p, const float* wsrc, int64_t ns,
                                             int64_t hi, float* wl, unsigned long long* gl, uint32_t* whl,
                                             uint32_t* wctr) {
  if (threadIdx.x == 0) *wctr = 0u;
  for (int64_t s = threadIdx.x; s < ns; s += kIterBlock) wl[s] = s < hi ? wsrc[s] : 0.f;
  for (int64_t s = threadIdx.x; s < ns * REP; s += kIterBlock) gl[s] = 0ull;
  __syncthreads();
  if (threadIdx.x < kWave) hot_digits(p, wl, whl);
  __syncthreads();
}

template <bool STATS, bool SAMPLE, int REP, bool TIERED>
__global__ __launch_bounds__(kIterBlock) void k_sgd_iter_hyb(DevSgd d, DevPrepared p, SgdParams sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double wsc[kIterBlock / kWave][kPartVals];
  __shared__ float hsum[kIterBlock / kWave][kHot];
  __shared__ float fdot[TIERED ? kIterBlock / kWave : 1][kRowsPerChunk];
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
  unsigned long long* gl = reinterpret_cast<unsigned long long*>(lds + d.nl);
  hyb_lds_init<REP>(p, d.wc32, d.nl, d.far_base, wl, gl, whl, &wctr);
  if (tst) tst[2] = __builtin_amdgcn_s_memrealtime();
  hyb_pass<STATS, SAMPLE, REP, TIERED>(d, p, sp, wl, gl, whl, hsum, wsc, d.part + int64_t(blockIdx.x) * d.pstride,
                                       &wctr, fdot, tst);
  if (tst) tst[6] = __builtin_amdgcn_s_memrealtime();
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
  // static LDS of k_sgd_iter_hyb<.., TIERED>: wsc, hsum, fdot per wave + whl, flags
  const int64_t statics = int64_t(kIterBlock / kWave) *
                              (kPartVals * int64_t(sizeof(double)) + kHot * int64_t(sizeof(float)) +
                               kRowsPerChunk * int64_t(sizeof(float))) +
                          kLanesPerRow * kHotLdsStride * int64_t(sizeof(uint32_t)) + 64;
  return ns <= kMaxHybridSlots && rep > 0 && lds_bytes(ns, rep) + statics <= 160 * 1024 - 1024;
}

template <bool STATS, bool SAMPLE>
static void launch_iter_t(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, bool u16,
                          int rep, int grid, hipStream_t s) {
  if (u16 && rep > 0 && p.hybrid) {
    const size_t lds = size_t(lds_bytes(d.nl, rep));
#define TWTML_HYB(R, T) \
  hipLaunchKernelGGL((k_sgd_iter_hyb<STATS, SAMPLE, R, T>), dim3(grid), dim3(kIterBlock), lds, s, d, p, sp)
    const bool tiered = p.tiered != 0;
    switch (rep) {
      case 8: if (tiered) TWTML_HYB(8, true); else TWTML_HYB(8, false); break;
      case 4: if (tiered) TWTML_HYB(4, true); else TWTML_HYB(4, false); break;
      case 2: if (tiered) TWTML_HYB(2, true); else TWTML_HYB(2, false); break;
      default: if (tiered) TWTML_HYB(1, true); else TWTML_HYB(1, false); break;
    }
#undef TWTML_HYB
  } else if (u16 && rep > 0) {
    const size_t lds = size_t(lds_bytes(d.nl, rep));
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
  } else {
    throw std::logic_error("launch_sgd_iter: active set exceeds LDS (the tiered path handles it)");
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
    case 8: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 8, true>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 8, false>)); break;
    case 4: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 4, true>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 4, false>)); break;
    case 2: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 2, true>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 2, false>)); break;
    default: if (hybrid) TWTML_OCC((k_sgd_iter_hyb<false, false, 1, true>)); else TWTML_OCC((k_sgd_iter_lds<false, false, 1, false>)); break;
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
  const int rep = u16 ? sgd_lds_rep(d.nl) : 0;
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

// ---------------------------------------------------------------------------
// Per-iteration protocol (no grid-wide barrier, no contended atomics):
//
//   k_sgd_iter_*  (iteration i)  prologue: converged after update i-1?  ->
//                 every workgroup decides from record i-1 (fixed-order sums,
//                 so all workgroups -- and all DP ranks -- agree); workgroup
//                 0 publishes state[0..1] and the host flag.  Then one
//                 partial gradient row per workgroup.
//   [k_sgd_reduce + RCCL all-reduce of g64 when DP; the verdict on update
//    i-1 rides along in g64[nl + 1] -- rank 0's, so the all-reduced value is
//    exact and the same on every rank whatever the backend's summation
//    order -- and k_sgd_update i acts on it: no update, state[0..1] and the
//    host flag.  Each rank skips the gradient pass of iteration i on its own
//    verdict (state[8]; identical weights -> the same verdict everywhere)
//    and then contributes zeros, but only the agreed verdict ends the loop,
//    so ranks can never disagree on the iteration count (a mismatch would
//    pair unequal collectives).]
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
// SimpleUpdater (fp64 master weights).  The partial rows are summed per
// block of 64 columns: lane l owns column col0 + l, the 16 waves of the
// workgroup take partial rows w, w + 16, ... (each load one coalesced 512-B
// row segment, all of a wave's rows in flight), and wave 0 adds the 16 wave
// sums in a fixed order -- deterministic, like every reduction here.  (The
// previous one-wave-per-column form read each column with 64 scattered
// 8-B loads: 20 us per iteration at 12.5K slots x 256 partial rows.)
// nparts > 0: the column gradients are the sums of the partial rows (single
// GPU); nparts == 0: g64 holds them (all-reduced, or the generic path).
// ---------------------------------------------------------------------------
constexpr int kUpdWaves = 1024 / kWave;   // waves per workgroup (partial-row split)

// Sum of partial rows for columns [col0, col0 + 64): returns lane's column
// sum in wave 0 (other waves: 0).  Contains a block barrier.
__device__ __forceinline__ double part_block_sum(const DevSgd& d, int64_t col0, int64_t ncols, int nparts,
                                                 double (*red)[kWave]) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int64_t col = col0 + lane;
  double acc = 0.0;
  if (col < ncols) {
    const double* src = d.part + col;
    const int64_t ps = d.pstride;
#pragma unroll 8
    for (int g = w; g < nparts; g += kUpdWaves) acc += src[int64_t(g) * ps];
  }
  red[w][lane] = acc;
  __syncthreads();
  double t = 0.0;
  if (w == 0) {
#pragma unroll
    for (int k = 0; k < kUpdWaves; ++k) t += red[k][lane];
  }
  __syncthreads();   // red is reused by the next column block
  return t;
}

__global__ __launch_bounds__(1024) void k_sgd_update(DevSgd d, SgdParams sp, int nparts) {
  __shared__ double wsc[kUpdWaves][2];
  __shared__ double red[kUpdWaves][kWave];
  __shared__ double m_sh;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  const int it = sp.iteration;
  if (sp.dp && it > 1) {   // the agreed verdict on update it - 1 (checked before state[0]:
                           // block 0 sets it below while other blocks may still start)
    const bool stop = d.g64[d.nl + 1] > 0.5;
    if (blockIdx.x == 0 && tid == 0 && d.host_flags)
      __hip_atomic_store(&d.host_flags[it - 1], stop ? 1.0 : 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (stop) {
      const int64_t n_far = kNumNumeric + d.n_unique - d.far_base;   // this pass's far sums are dropped
      for (int64_t j = int64_t(blockIdx.x) * 1024 + tid; j < n_far; j += int64_t(gridDim.x) * 1024)
        d.gfix[j] = 0ull;
      if (blockIdx.x == 0 && tid == 0) {
        d.state[0] = 1.0;
        d.state[1] = 1.0;
      }
      return;
    }
  }
  if (d.state[0] != 0.0) return;
  const int64_t ns = d.nl, hi = d.far_base;   // partial-row columns; near text slots end at far_base
  const int64_t ncols = ns + kPartVals - kNumNumeric;
  // m: global kept rows, or the sampled row count of this iteration
  if (tid < kWave) {
    double m = d.state[5];
    if (sp.sample) {
      m = *sgd_red_m(d, it);
      if (nparts > 0) {
        double t = 0.0;
        for (int g = tid; g < nparts; g += kWave) t += d.part[int64_t(g) * d.pstride + ns + 1];   // ns = nl
        m += wave_sum(t);
      }
    }
    if (tid == 0) m_sh = m;
  }
  __syncthreads();
  const double m = m_sh;
  const double alpha = sp.step_size / sqrt(double(it));
  double ds = 0.0, ws = 0.0;
  for (int64_t col0 = int64_t(blockIdx.x) * kWave; col0 < ncols; col0 += int64_t(gridDim.x) * kWave) {
    const double gp = nparts > 0 ? part_block_sum(d, col0, ncols, nparts, red) : 0.0;
    const int64_t col = col0 + lane;
    if (w == 0 && col < ncols) {
      const double g = (col <= ns ? d.g64[col] : 0.0) + gp;
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
  // tiered: far slots [far_base, 4 + n_unique), one thread per slot, from
  // the fixed-point far gradient (k_far_grad / all-reduced), re-zeroed here
  const int64_t n_far = kNumNumeric + d.n_unique - d.far_base;
  if (n_far > 0) {
    const double inv_m = m > 0.0 ? 1.0 / m : 0.0;
    for (int64_t j = int64_t(blockIdx.x) * 1024 + tid; j < n_far; j += int64_t(gridDim.x) * 1024) {
      const double g = double((long long)d.gfix[j]) * kFarInv;
      d.gfix[j] = 0ull;
      if (m > 0.0) {
        const int64_t col = d.far_base + j;
        const double step = alpha * (g * inv_m);
        const double wn = d.wc64[col] - step;
        d.wc64[col] = wn;
        d.wc32[col] = float(wn);
        ds += step * step;
        ws += wn * wn;
      }
    }
  }
  ds = wave_sum(ds);   // fixed order within the wave, then across waves
  ws = wave_sum(ws);
  if (lane == 0) {
    wsc[w][0] = ds;
    wsc[w][1] = ws;
  }
  __syncthreads();
  double* rec = sgd_rec(d, it);
  if (tid < 2) {
    double t = 0.0;
    for (int k = 0; k < kUpdWaves; ++k) t += wsc[k][tid];
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
  const int64_t tiles = (d.nl + kPartVals - kNumNumeric + kWave - 1) / kWave;
  const int64_t far_tiles = (kNumNumeric + d.n_unique - d.far_base + 1023) / 1024;
  const int grid = int(std::max<int64_t>(1, std::min<int64_t>(std::max(tiles, far_tiles), kMaxUpdGrid)));
  hipLaunchKernelGGL(k_sgd_update, dim3(grid), dim3(1024), 0, s, d, sp, nparts);
}

// Cross-workgroup reduction of the partial rows (DP: before the all-reduce)
// into g64 (+ loss, sampled count, batch stats): 64 columns per workgroup,
// fixed summation order.
__global__ __launch_bounds__(1024) void k_sgd_reduce(DevSgd d, SgdParams sp) {
  __shared__ double red[kUpdWaves][kWave];
  if (d.state[0] != 0.0) return;
  // DP pass skipped on this rank's verdict: its partial rows are stale, it
  // contributes zeros
  const bool skipped = d.state[8] == double(sp.iteration);
  if (d.nparts > 0) {
    const int64_t ncols = d.nl + kPartVals - kNumNumeric;
    const int64_t col0 = int64_t(blockIdx.x) * kWave;
    const double v = skipped ? 0.0 : part_block_sum(d, col0, ncols, d.nparts, red);
    const int64_t col = col0 + lane_id();
    if (threadIdx.x < kWave && col < ncols) {
      if (col <= d.nl) d.g64[col] = v;                     // slots, then the loss at [nl]
      else if (col == d.nl + 1) *sgd_red_m(d, sp.iteration) = v;   // sampled row count
      else d.stats[col - d.nl - 2] += v;                   // batch stats (iteration 1)
    }
  }
  // DP: rank 0's verdict on update i-1 -> g64[nl + 1] (all-reduced with the gradient)
  if (sp.dp && blockIdx.x == 0 && threadIdx.x < kWave) {
    const bool conv = sp.iteration > 1 && sgd_converged_wave(d, sp.iteration - 1, sp.tol);
    if (threadIdx.x == 0) d.g64[d.nl + 1] = (conv && sp.rank0) ? 1.0 : 0.0;
  }
}

void launch_sgd_reduce(const DevSgd& d, const SgdParams& sp, hipStream_t s) {
  if (d.nparts <= 0 && !sp.dp) return;
  const int grid = d.nparts > 0 ? int((d.nl + kPartVals - kNumNumeric + kWave - 1) / kWave) : 1;
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
// Far backward (tiered layout): the CSC lists every far entry grouped by
// slot; lane e of the grid takes entry e, converts its row's residual to the
// 2^-16 fixed point (kFarScale), and a segmented inclusive scan over
// the wave (segments = runs of equal slot) leaves each run's sum in its last
// lane, which adds it to gfix[slot - far_base] with one 64-bit integer
// atomic.  Integer sums are exact, so the result does not depend on the
// order of entries inside a slot or on which wave adds first: no per-entry
// float atomics, deterministic across runs and DP ranks.
// ---------------------------------------------------------------------------
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v) {
  return uint32_t(__builtin_amdgcn_update_dpp(int(old), int(v), CTRL, ROWS, 0xf, false));
}
// One Hillis-Steele step of a segmented 64-bit sum: lanes without a DPP
// source (or outside ROWS) see slot ~0 and add nothing.
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_scan_step(long long& q, uint32_t sl) {
  const uint32_t lo = dpp_u32<CTRL, ROWS>(0u, uint32_t(uint64_t(q)));
  const uint32_t hi = dpp_u32<CTRL, ROWS>(0u, uint32_t(uint64_t(q) >> 32));
  const uint32_t su = dpp_u32<CTRL, ROWS>(0xFFFFFFFFu, sl);
  if (su == sl) q += (long long)((uint64_t(hi) << 32) | lo);
}

__global__ __launch_bounds__(256) void k_far_grad(DevSgd d, SgdParams sp) {
  if (d.state[0] != 0.0 || d.state[8] == double(sp.iteration)) return;   // done / DP pass skipped
  const int64_t n = *d.far_n;
  const int lane = lane_id();
  bool clamped = false;
  const int64_t stride = int64_t(gridDim.x) * 256;
  for (int64_t e0 = int64_t(blockIdx.x) * 256 + (threadIdx.x & ~(kWave - 1)); e0 < n; e0 += stride) {
    const int64_t e = e0 + lane;
    const bool valid = e < n;
    uint32_t sl = valid ? d.fcsc_slot[e] : 0xFFFFFFFFu;
    long long q = 0;
    if (valid) {
      float v = d.rbuf[d.fcsc_pos[e]] * kFarScale;
      if (fabsf(v) > sp.far_lim) {
        clamped = true;
        v = v > 0.f ? sp.far_lim : -sp.far_lim;
      }
      q = __float2ll_rn(v);
    }
    // segmented inclusive scan on the VALU (DPP row shifts, then the row
    // broadcasts across the four 16-lane rows) instead of 18 LDS permutes:
    // the CSC is slot-sorted, so a lane k places back is in this lane's
    // segment iff it holds the same slot
    seg_scan_step<0x111, 0xf>(q, sl);   // row_shr:1
    seg_scan_step<0x112, 0xf>(q, sl);   // row_shr:2
    seg_scan_step<0x114, 0xf>(q, sl);   // row_shr:4
    seg_scan_step<0x118, 0xf>(q, sl);   // row_shr:8
    seg_scan_step<0x142, 0xa>(q, sl);   // row_bcast:15 -> rows 1, 3
    seg_scan_step<0x143, 0xc>(q, sl);   // row_bcast:31 -> rows 2, 3
    const uint32_t sn = uint32_t(__shfl_down(int(sl), 1, kWave));
    const bool tail = valid && (lane == kWave - 1 || e + 1 >= n || sn != sl);
    if (tail && q != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(&d.gfix[sl - d.far_base]), (unsigned long long)q);
  }
  if (__any(clamped) && lane == 0) d.state[7] = 1.0;
}

void launch_far_grad(const DevSgd& d, const SgdParams& sp, int num_cu, hipStream_t s) {
  hipLaunchKernelGGL(k_far_grad, dim3(std::max(1, num_cu * 4)), dim3(256), 0, s, d, sp);
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
    else if (s < kNumNumeric + d.n_unique) v = d.w64[d.slot_fid ? d.slot_fid[s] : uniq[s - kNumNumeric]];
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
    else d.w64[d.slot_fid ? d.slot_fid[s] : uniq[s - kNumNumeric]] = v;
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
  if (i < kStateLen) d.state[i] = i == 5 ? m_global : 0.0;
  if (i < 8) d.stats[i] = 0.0;
  if (i < 4) d.red64[i] = 0.0;
  if (i == 0) d.g64[d.nl] = 0.0;
  for (int k = i; k < n_loss; k += blockDim.x) d.loss_hist[k] = 0.0;
}

void launch_batch_init(const DevSgd& d, double m_global, int n_loss, hipStream_t s) {
  hipLaunchKernelGGL(k_batch_init, dim3(1), dim3(256), 0, s, d, m_global, n_loss);
}

}  // namespace twtml
