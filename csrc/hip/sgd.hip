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
// Exact, partition-independent arithmetic.  Per iteration i three kinds of
// fixed point are chosen from values every workgroup and every DP rank holds
// bit for bit (sgd_scales):
//   * weights: w_fix = rint(w32 * 2^K) with K from max |w_text| and the
//     longest row, so a row's whole text dot fits int32 (< 2^30 + 2^13);
//     a row's text dot is the int32 sum of count * w_fix -- hot counts
//     against base-128 weight digits (v_dot4_i32_i8), cold slots from LDS,
//     far slots from global memory -- so it does not depend on which of
//     those paths (layout, hot set, LDS tier) an entry took;
//   * gradients: q = rint(r * 2^S) with S from a rigorous bound B >= |r|
//     (max row bigram count * max |w| + sum max |n_k| |w_k| + max |y|), so
//     |q| <= 2^22 and 32 rows x count 15 of it fit an int32 hot accumulator;
//     cold entries add q into int64 LDS slots (ds_add_u64), far entries go
//     through the slot-sorted CSC (k_far_grad), the numeric features and the
//     loss are int64 sums at their own scales (2^N_k, 2^L);
//   * every cross-lane / workgroup / rank sum is an int64 sum.
// Integer sums are independent of the order rows are added in, so the
// gradient of a batch is the same whether one workgroup or 256, one GPU or
// eight DP ranks (any sharding) computed it: DP is bit-identical to one GPU.
//
// k_sgd_iter_hyb (the hot kernel): a 1024-thread workgroup stages the int32
// weights in LDS, streams its SELL-16x4 chunks (4 lanes per row, the row's
// slots kept in VGPRs between the forward gather and the backward scatter)
// and writes one int64 partial row (plain stores, no contended atomics).  At
// iteration 1 the same pass yields the prequential predictions and batch
// statistics (K4 + K7 fused: output op #1 uses the weights before training).
// k_sgd_update: fp64 master update + norms + max |w| + convergence record;
// every later kernel of the batch early-exits once the flag is set.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace twtml {

// Workgroup epilogue: every workgroup writes one int64 partial row (plain
// stores) that k_sgd_update / k_sgd_reduce sum (exact in any order):
//   cols 0..3 numeric gradients (2^N_k), 4..far_base-1 text slots (2^S),
//   far_base..nl-1 zero, nl loss (2^L), nl+1 sampled row count.
constexpr int kPartVals = 6;

// 256-thread update / reduce workgroups: they run beside the prep stream's
// kernels, and a 1024-thread workgroup needs 16 free wave slots on one CU --
// with prep workgroups resident, the r5 per-workgroup stamps showed the
// 433 update workgroups dispatched over ~52 us for ~5 us of work each.
constexpr int kUpdThreads = 256;
constexpr int kUpdWaves = kUpdThreads / kWave;   // waves per workgroup (partial-row split)
constexpr int kUpdFarSlots = kUpdThreads;        // far slots per far update workgroup (one per thread)

// Per-workgroup start / end stamps of the GD kernels (TWTML_ITER_TIMING only).
__device__ __forceinline__ void kdbg_stamp(uint64_t* base, int it, int kind, int end) {
  if (!base || threadIdx.x != 0 || blockIdx.x >= unsigned(kKdbgWgs)) return;
  base[((int64_t(it) * kKdbgKinds + kind) * kKdbgWgs + blockIdx.x) * 2 + end] = __builtin_amdgcn_s_memrealtime();
}

// Iteration record i and its per-update-workgroup partials.
__device__ __forceinline__ double* sgd_rec(const DevSgd& d, int it) { return d.itrec + int64_t(it) * kRecStride; }

__device__ __forceinline__ void unpack4(const uint2 v, uint32_t (&s)[4]) {
  s[0] = v.x & 0xFFFF; s[1] = v.x >> 16; s[2] = v.y & 0xFFFF; s[3] = v.y >> 16;
}

__device__ __forceinline__ void unpack8(const uint4 v, uint32_t (&s)[8]) {
  s[0] = v.x & 0xFFFF; s[1] = v.x >> 16; s[2] = v.y & 0xFFFF; s[3] = v.y >> 16;
  s[4] = v.z & 0xFFFF; s[5] = v.z >> 16; s[6] = v.w & 0xFFFF; s[7] = v.w >> 16;
}

// ---------------------------------------------------------------------------
// 64-bit lane exchanges.  DPP moves on the two halves stay on the VALU;
// shuffles go through ds_bpermute (used only in epilogues).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t shfl_xor_i64(int64_t v, int m) {
  const int lo = __shfl_xor(int(uint32_t(uint64_t(v))), m, kWave);
  const int hi = __shfl_xor(int(uint32_t(uint64_t(v) >> 32)), m, kWave);
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

template <int CTRL>
__device__ __forceinline__ int64_t dpp_i64(int64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, int(uint32_t(uint64_t(v))), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, int(uint32_t(uint64_t(v) >> 32)), CTRL, 0xf, 0xf, false);
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

// every lane: the sum over the 4 lanes j, j+4, j+8, j+12 of its 16-lane row
__device__ __forceinline__ int64_t row_sum_mod4_i64(int64_t v) {
  v += dpp_i64<0x124>(v);   // row_ror:4
  v += dpp_i64<0x128>(v);   // row_ror:8
  return v;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += shfl_xor_i64(v, off);
  return v;
}

// ---------------------------------------------------------------------------
// Per-iteration fixed-point scales.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int floor_log2(double x) {   // x > 0, finite
  int e;
  (void)frexp(x, &e);
  return e - 1;
}
__device__ __forceinline__ int ceil_log2(double x) {    // x >= 1
  const int e = floor_log2(x);
  return ldexp(1.0, e) < x ? e + 1 : e;
}

struct IterScale {
  float wscale, wunscale;   // 2^K, 2^-K
  float qscale;             // 2^S
  float lhalf;              // 2^(L/2)
  float nscale[kNumNumeric];    // 2^N_k
  int K, S, L, N[kNumNumeric];
  double B;
  int bad;
};

// Deterministic in (max |w_text|, numeric weights, batch bounds, m): every
// workgroup, every iteration kernel and every DP rank derives the same.
__device__ IterScale sgd_scales(const double* bd, double maxw, const float* wn) {
  IterScale s{};
  double B = bd[0] * maxw + bd[1];
#pragma unroll
  for (int k = 0; k < kNumNumeric; ++k) B += bd[2 + k] * fabs(double(wn[k]));
  B = B * (1.0 + 1.0 / 1024.0) + 1.0;   // fp32 rounding of the dot, rint of the weights
  s.B = B;
  // diverged: the residual bound (or the weights) left any usable range
  s.bad = !(B < 1e30) || !(maxw < 1e30) || !(B == B);
  if (s.bad) {
    s.wscale = s.wunscale = s.qscale = s.lhalf = 1.f;
    for (int k = 0; k < kNumNumeric; ++k) s.nscale[k] = 1.f;
    return s;
  }
  // maxw 2^K < 2^25 (4 base-128 digits) and rowmax maxw 2^K < 2^30: a row's
  // fixed-point dot, rint errors included (<= rowmax / 2), fits int32
  int K = 0;
  if (maxw > 0.0) {
    K = 24 - floor_log2(maxw);
    const double T = bd[0] * maxw;
    if (T > 0.0) K = min(K, 29 - floor_log2(T));
  }
  K = K < -120 ? -120 : (K > 120 ? 120 : K);
  const int eb = floor_log2(B) + 1;                     // B < 2^eb
  // Per row |q|, |r n_k| 2^N_k and r^2 2^L stay <= 2^22: kHotFlush rows of
  // them (x count 15 for q) fit the kernels' int32 accumulators, and m rows
  // (m < 2^31) the int64 sums.
  s.K = K;
  s.S = 22 - eb;                                        // |q| <= B 2^S + 1/2 <= 2^22
  s.L = 2 * (11 - eb);                                  // (r 2^(L/2))^2 <= 2^22
  s.wscale = ldexpf(1.f, K);
  s.wunscale = ldexpf(1.f, -K);
  s.qscale = ldexpf(1.f, s.S);
  s.lhalf = ldexpf(1.f, 11 - eb);
#pragma unroll
  for (int k = 0; k < kNumNumeric; ++k) {
    const double nm = bd[2 + k];
    int n = nm > 0.0 ? 22 - eb - (floor_log2(nm) + 1) : 0;   // B max|n_k| 2^N < 2^22
    n = n < -120 ? -120 : (n > 120 ? 120 : n);
    s.N[k] = n;
    s.nscale[k] = ldexpf(1.f, n);
  }
  return s;
}

__device__ __forceinline__ float sgpr_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ double sgpr_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(u))));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(u >> 32))));
  return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}

// What a lane of the iteration kernels keeps of the scales: wave-uniform
// factors in SGPRs, its numeric feature's weight and scale.
struct LaneScale {
  float wscale, wunscale, qscale, lhalf;
  float nsc_t;   // 2^N_t of this lane's numeric feature
  float wn_t;
};

__device__ __forceinline__ LaneScale lane_scale(const IterScale& sc, const DevSgd& d, int t) {
  LaneScale l;
  l.wscale = sgpr_f(sc.wscale);
  l.wunscale = sgpr_f(sc.wunscale);
  l.qscale = sgpr_f(sc.qscale);
  l.lhalf = sgpr_f(sc.lhalf);
  l.nsc_t = sc.nscale[t];
  l.wn_t = d.wc32[t];
  return l;
}


// ---------------------------------------------------------------------------
// Convergence after update `it`, evaluated by one wave (lane-parallel loads,
// fixed-order DPP reduction): identical in every caller.  Also returns the
// max |w_text| after that update (the next iteration's weight scale).
// ---------------------------------------------------------------------------
// Near column tiles and far slot ranges of every update launch of the batch:
// a function of the layout only (the same on every DP rank).  ONE helper for
// the host launch (launch_sgd_update) and the device convergence check, which
// reads that many partials per record without reading the record's own count
// (rec[2]) first (the two must not drift).
struct UpdSplit {
  int nt, nf;
};
__host__ __device__ __forceinline__ UpdSplit upd_split(const DevSgd& d) {
  const int64_t tiles = (d.nl + kPartVals - kNumNumeric + kWave - 1) / kWave;
  const int64_t n_far = kNumNumeric + d.n_unique - d.far_base;
  const int64_t nt = tiles < 1 ? 1 : (tiles < kMaxUpdGrid / 2 ? tiles : kMaxUpdGrid / 2);
  int64_t nf = 0;
  if (n_far > 0) {
    nf = (n_far + kUpdFarSlots - 1) / kUpdFarSlots;
    if (nf > kMaxUpdGrid - nt) nf = kMaxUpdGrid - nt;
    if (nf < 1) nf = 1;
  }
  return UpdSplit{int(nt), int(nf)};
}
__device__ __forceinline__ int upd_grid(const DevSgd& d) {
  const UpdSplit u = upd_split(d);
  return u.nt + u.nf;
}

// The update writes its per-workgroup partials (sum step^2, sum w^2, max |w|)
// as three arrays of kMaxUpdGrid (rec_part): one wave reads them 512 B per
// load instruction.
__device__ __forceinline__ int rec_part(int c, int k) { return kRecHead + c * kMaxUpdGrid + k; }

// Every load is issued before the first add: kConvU partials per lane and
// array in flight, the record head and the norm state too (a loop that
// waited on each step's loads made the iteration prologue ~14 dependent L2
// round trips, 5.9 us per iteration kernel: profiles/r6/ablate_iter.txt).
// The per-lane sums add the partials in increasing k, as before.
constexpr int kConvU = 8;

__device__ bool sgd_converged_wave(const DevSgd& d, int it, double tol, double* maxw_out = nullptr) {
  const double* rec = sgd_rec(d, it);
  const int nw = upd_grid(d);   // (rec[2] holds the same; reading it first cost a dependent round trip)
  const double r0 = rec[0], r1 = rec[1], st4 = d.state[4], st6 = d.state[6];
  double ds = 0.0, ws = 0.0, mx = 0.0;
  for (int k0 = lane_id(); k0 < nw; k0 += kWave * kConvU) {
    double a[kConvU], b[kConvU], c[kConvU];
#pragma unroll
    for (int u = 0; u < kConvU; ++u) {
      const int k = k0 + u * kWave;
      const bool ok = k < nw;
      a[u] = ok ? rec[rec_part(0, k)] : 0.0;
      b[u] = ok ? rec[rec_part(1, k)] : 0.0;
      c[u] = ok ? rec[rec_part(2, k)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kConvU; ++u) {
      if (k0 + u * kWave < nw) {
        ds += a[u];
        ws += b[u];
        mx = fmax(mx, c[u]);
      }
    }
  }
  ds = wave_sum(ds);
  ws = wave_sum(ws);
  mx = wave_max(mx);
  if (maxw_out) *maxw_out = mx;
  if (!(r1 > 0.0) || r0 < 2.0) return false;   // no update this iteration / first update
  double rest = st4 - st6;
  if (rest < 0.0) rest = 0.0;
  const double wnorm = sqrt(ws + rest);
  return sqrt(ds) < tol * (wnorm > 1.0 ? wnorm : 1.0);
}

// Iteration-kernel prologue (every thread calls it; `flag` / `sc` are
// workgroup-shared): true when the batch is finished (the caller returns).
// Wave 0 checks convergence after update i-1, derives iteration i's scales
// (workgroup 0 records them for the far backward / reduce / update kernels)
// and publishes the verdict on update i-1 to the host (zero-copy pinned
// memory, initialised to -1 by the host) which polls it to stop enqueueing.
// A diverged model (scales invalid) stops like a converged one, with
// state[7] set instead of state[1].  DP ranks only skip the pass on their
// own verdict (state[8] = iteration): k_sgd_reduce puts rank 0's into the
// gradient all-reduce and k_sgd_update acts on the agreed value.
__device__ bool sgd_prologue(const DevSgd& d, const SgdParams& sp, int* flag, IterScale* sc) {
  if (threadIdx.x < kWave) {
    const int it = sp.iteration;
    // every load up front and independent of the others (one memory round
    // trip instead of four dependent ones: ~3.8 us of each iteration's
    // prologue in the per-workgroup timeline, r5)
    const double st0 = d.state[0];
    double maxw = d.state[9];
    const float wn[kNumNumeric] = {d.wc32[0], d.wc32[1], d.wc32[2], d.wc32[3]};
    double bd[kBoundsLen];
#pragma unroll
    for (int k = 0; k < kBoundsLen; ++k) bd[k] = d.bounds[k];
    const bool conv = it > 1 && sgd_converged_wave(d, it - 1, sp.tol, &maxw);
    const bool done = st0 != 0.0;
    bool stop = done;
    if (!done) {
      const IterScale s = sgd_scales(bd, maxw, wn);
      stop = conv || s.bad;
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        double* rec = sgd_rec(d, it);
        rec[kRecK] = s.K;
        rec[kRecS] = s.S;
        rec[kRecL] = s.L;
        for (int k = 0; k < kNumNumeric; ++k) rec[kRecN + k] = s.N[k];
        rec[kRecB] = s.B;
        rec[kRecBad] = s.bad ? 1.0 : 0.0;
        if (s.bad) d.state[7] = 1.0;
        if (stop) {
          if (!sp.dp) {
            d.state[0] = 1.0;
            if (conv && !s.bad) d.state[1] = 1.0;
          } else {
            d.state[8] = double(it);   // DP: skip this pass; the agreed verdict ends the batch
          }
        }
      }
      if (threadIdx.x == 0) *sc = s;
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

// ---------------------------------------------------------------------------
// Row epilogue shared by the iteration kernels.
// ---------------------------------------------------------------------------
// Per-lane accumulators.  Lane t of a row owns numeric feature t; lane 0 the
// loss, sampled count and batch statistics.  qn / ql hold at most kHotFlush
// rows (int32, <= 2^22 per row) before the kernel folds them into int64.
struct RowAcc {
  int32_t qn = 0;     // sum rint(r n_t 2^N_t)
  int32_t ql = 0;     // sum rint((r 2^(L/2))^2) (t == 0)
  int32_t msum = 0;   // rows in the sampled gradient (t == 0, SAMPLE)
};

struct RowIn {
  float nt, y;   // this lane's numeric feature, the label
};

__device__ __forceinline__ RowIn row_in(const DevPrepared& p, int64_t pos, int t) {
  return RowIn{p.num[int64_t(t) * p.cap_rows16 + pos], p.y[pos]};
}

// sum of a row's 4 lane values (every lane of the row gets the same bits)
__device__ __forceinline__ int32_t row_total(int32_t v) {
  v += __shfl_xor(v, 1, kWave);
  v += __shfl_xor(v, 2, kWave);
  return v;
}

// Residual of the row at sorted position pos from its fixed-point text dot
// (already summed over the row's 4 lanes); STATS (iteration 1): the row's
// rounded prediction to pbuf (k_batch_stats sums the moments exactly) and
// the plot's pred / real; accumulates numeric-feature gradients, loss and
// the sampled count.  Returns r (0 for rows outside the batch / the sample).
template <bool STATS, bool SAMPLE>
__device__ __forceinline__ float row_residual(int32_t dot_fix, const RowIn& ri, int64_t pos, int t,
                                              const DevSgd& d, const DevPrepared& p, const SgdParams& sp,
                                              int64_t n_kept, const LaneScale& sc, RowAcc& acc) {
  const bool valid = pos < n_kept;
  // numeric part: (n0 w0 + n1 w1) + (n2 w2 + n3 w3), the same bits on the row's 4 lanes
  float vn = ri.nt * sc.wn_t;
  vn += __shfl_xor(vn, 1, kWave);
  vn += __shfl_xor(vn, 2, kWave);
  const float dot = float(dot_fix) * sc.wunscale + vn;
  bool in = valid;
  if (SAMPLE && valid)
    in = sample_uniform(uint64_t(42 + sp.iteration), uint64_t(sp.row_offset + p.perm[pos])) < sp.fraction;
  const float r = in ? dot - ri.y : 0.f;
  if (t == 0) {
    if (STATS && valid) {
      // round half away of an fp32 value is an fp32 value (|dot| >= 2^23 is
      // already an integer), so the float holds the prediction exactly
      const float pr = float(round_half_away(double(dot)));
      d.pbuf[pos] = pr;
      if (sp.want_pred) {
        d.pred_out[p.perm[pos]] = pr;
        d.real_out[p.perm[pos]] = ri.y;
      }
    }
    if (SAMPLE && in) ++acc.msum;
    const float u = r * sc.lhalf;
    acc.ql += __float2int_rn(u * u);
  }
  acc.qn += __float2int_rn((r * ri.nt) * sc.nsc_t);
  return r;
}


template <bool STATS>
__device__ __forceinline__ void part_scalars(const DevSgd& d, int64_t qn, int64_t ql, const RowAcc& acc,
                                             const unsigned long long* wg_tot, int64_t (*wsc)[kPartVals],
                                             int64_t* prow) {
  const int w = threadIdx.x / kWave, lane = lane_id();
  // numeric: lanes with t == k hold feature k -> sum per quad column, then the 4 rows
  qn = row_sum_mod4_i64(qn);
  qn += shfl_xor_i64(qn, 16);
  qn += shfl_xor_i64(qn, 32);
  ql = wave_sum_i64(ql);
  const int ms = wave_sum(acc.msum);
  if (lane < kNumNumeric) wsc[w][lane] = qn;
  if (lane == 0) {
    wsc[w][4] = ql;
    wsc[w][5] = ms;
  }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < kPartVals) {
    const int nw = int(blockDim.x) / kWave;
    int64_t v = (wg_tot && tid < 5) ? (long long)wg_tot[tid] : 0;
    for (int k = 0; k < nw; ++k) v += wsc[k][tid];
    const int64_t col = tid < kNumNumeric ? int64_t(tid) : d.nl + (tid - kNumNumeric);
    prow[col] = v;
  }
}

template <int REP>
__device__ __forceinline__ int64_t part_slot(const unsigned long long* gl, int64_t s) {
  long long v = 0;
#pragma unroll
  for (int k = 0; k < REP; ++k) v += (long long)gl[s * REP + k];
  return v;
}

__device__ __forceinline__ int32_t w_to_fix(float w, float wscale) {
  return __float2int_rn(w * wscale);
}

// ---------------------------------------------------------------------------
// Plain path (u16 slots, no hot split): LDS int32 weights + REP replicated
// int64 gradients.  CNT: entries carry HashingTF term counts (p.cnt, merged
// duplicates, chunk lengths p.clen8d); otherwise every entry counts once.
// ---------------------------------------------------------------------------
constexpr int kIterBlock = 1024;

template <bool STATS, bool SAMPLE, int REP, bool CNT>
__global__ __launch_bounds__(kIterBlock) void k_sgd_iter_lds(DevSgd d, DevPrepared p, SgdParams sp) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds[];
  __shared__ int64_t wsc[kIterBlock / kWave][kPartVals];
  __shared__ int stop_flag;
  __shared__ IterScale scs;
  if (sgd_prologue(d, sp, &stop_flag, &scs)) return;   // converged / finished: the rest of the batch is a no-op
  const int lane = lane_id();
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  const LaneScale sc = lane_scale(scs, d, t);
  const int64_t ns = d.nl;        // multiple of 64 (== d.ns: the plain path is never tiered)
  int32_t* wl = lds;
  unsigned long long* gl = reinterpret_cast<unsigned long long*>(lds + ns);
  const int64_t hi_slot = kNumNumeric + d.n_unique;
  for (int64_t s = threadIdx.x; s < ns; s += kIterBlock)
    wl[s] = (s >= kNumNumeric && s < hi_slot) ? w_to_fix(d.wc32[s], sc.wscale) : 0;
  for (int64_t s = threadIdx.x; s < ns * REP; s += kIterBlock) gl[s] = 0ull;
  __syncthreads();
  const int rep = lane % REP;
  const int64_t n_kept = p.counters[0];
  const int64_t nch = (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;
  const int64_t wave = int64_t(blockIdx.x) * (kIterBlock / kWave) +
                       __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);   // wave-uniform
  const int64_t nwaves = int64_t(gridDim.x) * (kIterBlock / kWave);
  const uint16_t* slot = static_cast<const uint16_t*>(p.slot);
  RowAcc acc;
  int64_t qn64 = 0, ql64 = 0;   // acc.qn / acc.ql folded every chunk

  // chunk metadata for 64 chunks at a time in lanes
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
    const RowIn ri = row_in(p, pos, t);
    qn64 += acc.qn;   // the previous chunk's row
    ql64 += acc.ql;
    acc.qn = acc.ql = 0;
    if (L8 <= kMaxRegGroups) {
      uint4 v[kMaxRegGroups];
      uint4 cv[CNT ? kMaxRegGroups : 1];
#pragma unroll
      for (int g = 0; g < kMaxRegGroups; ++g)
        if (g < L8) {
          v[g] = *reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride);
          if (CNT) cv[g] = *reinterpret_cast<const uint4*>(p.cnt + off + int64_t(g) * kChunkStride);
        }
      int32_t d0 = 0, d1 = 0;   // partial sums of the row's int32 dot (sgd_scales)
#pragma unroll
      for (int g = 0; g < kMaxRegGroups; ++g) {
        if (g < L8) {
          uint32_t s[8];
          unpack8(v[g], s);
          if (CNT) {
            uint32_t kk[8];
            unpack8(cv[g], kk);
            d0 += wl[s[0]] * int32_t(kk[0]) + wl[s[2]] * int32_t(kk[2]) + wl[s[4]] * int32_t(kk[4]) +
                  wl[s[6]] * int32_t(kk[6]);
            d1 += wl[s[1]] * int32_t(kk[1]) + wl[s[3]] * int32_t(kk[3]) + wl[s[5]] * int32_t(kk[5]) +
                  wl[s[7]] * int32_t(kk[7]);
          } else {
            d0 += wl[s[0]] + wl[s[2]] + wl[s[4]] + wl[s[6]];
            d1 += wl[s[1]] + wl[s[3]] + wl[s[5]] + wl[s[7]];
          }
        }
      }
      const int32_t dot = row_total(d0 + d1);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, sc, acc);
      if (res != 0.f && sp.ablate == 0) {
        const unsigned long long q = (unsigned long long)(long long)__float2int_rn(res * sc.qscale);
#pragma unroll
        for (int g = 0; g < kMaxRegGroups; ++g) {
          if (g < L8) {
            uint32_t s[8];
            unpack8(v[g], s);
            if (CNT) {
              uint32_t kk[8];
              unpack8(cv[g], kk);
#pragma unroll
              for (int e = 0; e < 8; ++e) atomicAdd(&gl[s[e] * REP + rep], q * (unsigned long long)kk[e]);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) atomicAdd(&gl[s[e] * REP + rep], q);
            }
          }
        }
      }
    } else {  // very long rows: stream the slots twice (never merged: count 1)
      int32_t dot = 0;
      for (int32_t g = 0; g < L8; ++g) {
        uint32_t s[8];
        unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
        for (int e = 0; e < 8; ++e) dot += wl[s[e]];
      }
      dot = row_total(dot);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, sc, acc);
      if (res != 0.f) {
        const unsigned long long q = (unsigned long long)(long long)__float2int_rn(res * sc.qscale);
        for (int32_t g = 0; g < L8; ++g) {
          uint32_t s[8];
          unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
          for (int e = 0; e < 8; ++e) atomicAdd(&gl[s[e] * REP + rep], q);
        }
      }
    }
  }

  int64_t* prow = d.part + int64_t(blockIdx.x) * d.pstride;
  part_scalars<STATS>(d, qn64 + acc.qn, ql64 + acc.ql, acc, nullptr, wsc, prow);   // includes the block barrier
  for (int64_t s = kNumNumeric + threadIdx.x; s < ns; s += kIterBlock)
    prow[s] = s < hi_slot ? part_slot<REP>(gl, s) : 0;   // pads are never flushed
}

// ---------------------------------------------------------------------------
// Hybrid dense-hot path (layout: hot_split.hip).  Per chunk a lane reads its
// row's 32 hot counts (16 B: 4-bit counts of hot ids 32t..32t+31) and the
// row-balanced cold groups.  Hot weights are read from LDS as base-128
// digit planes (b128 loads, broadcast across the 16 lanes of a quarter), the
// hot gradient accumulates as int32 count * q per lane (flushed to an int64
// LDS row every kHotFlush chunks); cold entries use the LDS int64 gradient.
// Chunks left in the plain layout (clen8c < 0) take the plain route.
// ---------------------------------------------------------------------------
constexpr int kMaxColdGroups = 8;   // cold 4-entry groups kept in VGPRs (32 cold entries per lane)
constexpr int kHotPerLane = kHot / kLanesPerRow;   // 32
// rows a lane adds into its int32 hot accumulators between flushes:
// kHotFlush * 15 * 2^22 < 2^31
constexpr int kHotFlush = 32;

// wq: this lane's 32 hot weight digits in LDS (quarter t, 16-B aligned,
// stride 36 dwords so the four quarters' b128 reads hit different banks)
constexpr int kHotLdsStride = kHotPerLane + 4;

// Hot weights w_fix (|w_fix| < 2^25) as 4 signed base-128 digits
// (w_fix = d0 2^21 + d1 2^14 + d2 2^7 + d3): the forward dot of a lane's 32
// hot counts is 32 v_dot4_i32_i8 (4 counts x 4 digits each, exact int32).
// LDS per lane quarter t (kHotLdsStride dwords): dword (d*4 + q)*2 + half
// packs digit d of the 4 hot ids held in the even (half 0) / odd (half 1)
// nibbles of the lane's count dword q.
__device__ __forceinline__ void nib_split(uint32_t x, uint32_t& lo, uint32_t& hi) {
  lo = x & 0x0F0F0F0Fu;           // nibbles 0,2,4,6 -> bytes 0..3
  hi = (x >> 4) & 0x0F0F0F0Fu;    // nibbles 1,3,5,7 -> bytes 0..3
}

__device__ __forceinline__ int32_t hot_dot(const uint4 hv, const uint32_t* wq) {
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
  // the lane's exact hot dot, a partial sum of the row's int32 dot (sgd_scales)
  return (((acc[0] << 7) + acc[1]) << 14) + (acc[2] << 7) + acc[3];
}

// gh[i] += count of hot id 32t + i times q (v_bfe + v_mad_i32_i24)
__device__ __forceinline__ void hot_grad(const uint4 hv, int32_t q, int32_t (&gh)[kHotPerLane]) {
  const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t c = int32_t((hw[qq] >> (4 * k)) & 15u);
      // in place (tied operand): the accumulators keep their registers
      // across the loop instead of being renamed and copied back
      asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(gh[8 * qq + k]) : "v"(c), "v"(q));
    }
  }
}

// int32 hot / numeric / loss accumulators -> the workgroup's int64 row
// hsum[0, kHot + 5): per quad column over the 16-lane row (DPP), then lanes
// 0..3 of each row add (4 rows per address; once per kHotFlush chunks).
__device__ __forceinline__ void hot_flush(int32_t (&gh)[kHotPerLane], RowAcc& acc, unsigned long long* hsum) {
  const int lane = lane_id();
  const bool head = (lane & 15) < kLanesPerRow;
#pragma unroll
  for (int i = 0; i < kHotPerLane; ++i) {
    const int64_t v = row_sum_mod4_i64(int64_t(gh[i]));
    if (head && v != 0) atomicAdd(&hsum[kHotPerLane * (lane & 3) + i], (unsigned long long)v);
    asm volatile("v_mov_b32 %0, 0" : "+v"(gh[i]));   // zeroed in place (no second register set)
  }
  const int64_t qn = row_sum_mod4_i64(int64_t(acc.qn));
  const int64_t ql = row_sum_mod4_i64(int64_t(acc.ql));
  if (head && qn != 0) atomicAdd(&hsum[kHot + (lane & 3)], (unsigned long long)qn);
  if ((lane & 15) == 0 && ql != 0) atomicAdd(&hsum[kHot + kNumNumeric], (unsigned long long)ql);
  acc.qn = 0;
  acc.ql = 0;
}

// Build the digit table of the pass from the LDS int32 weights (one wave; the
// caller synchronises).  Hot id h: quarter t = h / 32, count dword
// q = (h % 32) / 8, nibble k = h % 8 -> half = k & 1, byte i = k >> 1.
__device__ __forceinline__ void hot_digits(const DevPrepared& p, const int32_t* wl, uint32_t* whl) {
  const int lane = lane_id();
  uint8_t* bytes = reinterpret_cast<uint8_t*>(whl);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int h = lane + u * kWave;
    int32_t W = wl[p.hot_slot[h]];
    int32_t dg[4];
#pragma unroll
    for (int d = 3; d > 0; --d) {   // balanced base-128 digits, least significant first
      const int32_t x = ((W + 64) & 127) - 64;
      dg[d] = x;
      W = (W - x) >> 7;
    }
    dg[0] = W;                       // |W| <= 2^25 -> |d0| <= 16
    const int t = h / 32, q = (h % 32) / 8, k = h % 8;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      bytes[(t * kHotLdsStride + (d * 4 + q) * 2 + (k & 1)) * 4 + (k >> 1)] = uint8_t(int8_t(dg[d]));
  }
}

// wctr: the workgroup's LDS chunk counter, zeroed by hyb_lds_init.
// TIERED: the chunk's far entries (p.fslot list, weights from global memory)
// join the row dots through the per-wave LDS row sums fdot (int32), and every
// row's residual goes to d.rbuf for the far backward (k_far_grad).
template <bool STATS, bool SAMPLE, int REP, bool TIERED>
__device__ __forceinline__ void hyb_pass(const DevSgd& d, const DevPrepared& p, const SgdParams& sp,
                                         const LaneScale& sc, const int32_t* wl, unsigned long long* gl,
                                         const uint32_t* whl, unsigned long long* hsum,
                                         int64_t (*wsc)[kPartVals], int64_t* prow, uint32_t* wctr,
                                         int32_t (*fdot)[kRowsPerChunk], uint64_t* tst = nullptr) {
  const int64_t ns = d.nl;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);   // wave-uniform
  const int r = lane / kLanesPerRow, t = lane % kLanesPerRow;
  const int rep = lane % REP;
  const int64_t n_kept = p.counters[0];
  const int64_t nch = sp.ablate == 7 ? 0 : (n_kept + kRowsPerChunk - 1) / kRowsPerChunk;  // 7: fixed cost
  const uint16_t* slot = static_cast<const uint16_t*>(p.slot);
  const uint4* hdense = reinterpret_cast<const uint4*>(p.hot_dense);
  const int32_t* __restrict__ clen8c = p.clen8c;
  const int64_t* __restrict__ cbase = p.cbase;
  const uint32_t* wq = whl + t * kHotLdsStride;
  int32_t gh[kHotPerLane];
#pragma unroll
  for (int i = 0; i < kHotPerLane; ++i) gh[i] = 0;
  RowAcc acc;

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
  int k = 0;          // chunks this wave took
  int64_t j = grab();
  int32_t L8n = 0, fcn = 0;
  int64_t cbn = 0;
  if (j < nj) {
    L8n = clen8c[b + j * G];
    cbn = cbase[b + j * G];
    if (TIERED) fcn = p.fcount[b + j * G];
  }
  // epochs of at most kHotFlush chunks: each lane adds <= kHotFlush rows
  // into its int32 accumulators before they are folded into the int64 row
  while (j < nj) {
  for (int e = 0; e < kHotFlush && j < nj; ++e) {
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
    const RowIn ri = row_in(p, pos, t);
    // The chunk's hot block and cold slots are loaded first: their latency
    // then overlaps the far forward's two dependent round trips below.
    uint4 hv = make_uint4(0, 0, 0, 0);
    uint2 v[kMaxColdGroups];
    // cold stream: L8c groups of kColdGroup slots per lane (hot_split.hip)
    const uint16_t* csl = p.cslot + cb * kChunkStride + lane * kColdGroup;
    const bool reg = L8c >= 0 && L8c <= kMaxColdGroups;
    if (L8c >= 0) {
      hv = hdense[c * kWave + lane];
      if (reg) {
#pragma unroll
        for (int g = 0; g < kMaxColdGroups; ++g)
          if (g < L8c) v[g] = *reinterpret_cast<const uint2*>(csl + int64_t(g) * kColdStride);
      }
    }
    // far entries of the chunk: their row sums land in lane t == 0 of the row;
    // up to 4 list entries per lane in flight, then their weight gathers
    int32_t far = 0;
    if (TIERED && fc > 0 && abl != 8) {   // wave-uniform (ablate 8: no far forward)
      int32_t* fd = fdot[w];
      if (lane < kRowsPerChunk) fd[lane] = 0;
      wave_lds_sync();
      const uint32_t* fl = p.fslot + cb * kChunkStride;
      constexpr int kFarU = 4;
      for (int32_t k0 = 0; k0 < fc; k0 += kFarU * kWave) {
        uint32_t e[kFarU];
        float fw[kFarU];
#pragma unroll
        for (int u = 0; u < kFarU; ++u) e[u] = k0 + u * kWave + lane < fc ? fl[k0 + u * kWave + lane] : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < kFarU; ++u) fw[u] = e[u] != 0xFFFFFFFFu ? d.wc32[e[u] & 0x0FFFFFFFu] : 0.f;
#pragma unroll
        for (int u = 0; u < kFarU; ++u)
          if (e[u] != 0xFFFFFFFFu) atomicAdd(&fd[e[u] >> 28], w_to_fix(fw[u], sc.wscale));   // ds_add_u32: exact
      }
      wave_lds_sync();
      if (t == 0) far = fd[r];
    }
    if (L8c >= 0) {
      const uint16_t* sl = csl;
      // timing-only ablations (results meaningless): 12 no hot dot, 13 no
      // cold forward, 14 no hot gradient, 11 no cold backward atomics
      int32_t d0 = abl == 12 ? int32_t(hv.x) : hot_dot(hv, wq), d1 = far;   // partial sums of the row's int32 dot
      if (reg && abl == 13) {
#pragma unroll
        for (int g = 0; g < kMaxColdGroups; ++g)
          if (g < L8c) d0 += int32_t(v[g].x ^ v[g].y);
      } else if (reg) {
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
      const int32_t dot = row_total(d0 + d1);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, sc, acc);
      if (TIERED && t == 0) d.rbuf[pos] = res;
      const int32_t q = __float2int_rn(res * sc.qscale);
      // unconditional (q = 0 adds nothing): the accumulators then need no
      // second register set for a skipped update
      if (abl != 14) hot_grad(hv, q, gh);
      if (res != 0.f && abl != 11) {
        const unsigned long long qq = (unsigned long long)(long long)q;
        if (reg) {
#pragma unroll
          for (int g = 0; g < kMaxColdGroups; ++g)
            if (g < L8c) {
              uint32_t s[4];
              unpack4(v[g], s);
#pragma unroll
              for (int e = 0; e < 4; ++e) atomicAdd(&gl[s[e] * REP + rep], qq);
            }
        } else {
          for (int32_t g = 0; g < L8c; ++g) {
            uint32_t s[4];
            unpack4(*reinterpret_cast<const uint2*>(sl + int64_t(g) * kColdStride), s);
#pragma unroll
            for (int e = 0; e < 4; ++e) atomicAdd(&gl[s[e] * REP + rep], qq);
          }
        }
      }
    } else {  // plain layout: every entry (hot ones too) through the LDS gradient
      const int32_t L8 = p.clen8[c];
      const uint16_t* sl = slot + off;
      int32_t dot = far;
      for (int32_t g = 0; g < L8; ++g) {
        uint32_t s[8];
        unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
        for (int e = 0; e < 8; ++e) dot += wl[s[e]];
      }
      dot = row_total(dot);
      const float res = row_residual<STATS, SAMPLE>(dot, ri, pos, t, d, p, sp, n_kept, sc, acc);
      if (TIERED && t == 0) d.rbuf[pos] = res;
      if (res != 0.f) {
        const unsigned long long q = (unsigned long long)(long long)__float2int_rn(res * sc.qscale);
        for (int32_t g = 0; g < L8; ++g) {
          uint32_t s[8];
          unpack8(*reinterpret_cast<const uint4*>(sl + int64_t(g) * kChunkStride), s);
#pragma unroll
          for (int e = 0; e < 8; ++e) atomicAdd(&gl[s[e] * REP + rep], q);
        }
      }
    }
  }
  hot_flush(gh, acc, hsum);
  }

  if (tst) tst[3] = __builtin_amdgcn_s_memrealtime();
  if (d.tdbg && blockIdx.x == 0 && lane == 0) {   // per-wave end of the chunk loop (WG 0)
    uint64_t* we = d.tdbg + 4096 + int64_t(sp.iteration) * 32 + w * 2;
    we[0] = __builtin_amdgcn_s_memrealtime();
    we[1] = uint64_t(k);
  }
  if (tst) tst[4] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();   // every wave's hsum adds
  part_scalars<STATS>(d, 0, 0, acc, hsum + kHot, wsc, prow);   // includes the block barrier
  if (tst) tst[5] = __builtin_amdgcn_s_memrealtime();
  const int64_t hi = d.far_base;            // pads (and far slots) are never flushed
  // kFlushU slots per thread per step: their hot_of loads are all in flight
  // before the first LDS read (one L2 round trip per step, not per slot)
  constexpr int kFlushU = 4;
  for (int64_t s0 = kNumNumeric + threadIdx.x; s0 < ns; s0 += int64_t(kIterBlock) * kFlushU) {
    uint32_t h[kFlushU];
#pragma unroll
    for (int u = 0; u < kFlushU; ++u) {
      const int64_t s = s0 + int64_t(u) * kIterBlock;
      h[u] = s < hi ? uint32_t(p.hot_of[s]) : 0xFFu;
    }
#pragma unroll
    for (int u = 0; u < kFlushU; ++u) {
      const int64_t s = s0 + int64_t(u) * kIterBlock;
      if (s >= ns) break;
      int64_t v = 0;
      if (s < hi) {
        v = part_slot<REP>(gl, s);
        if (h[u] != 0xFFu) v += (long long)hsum[h[u]];
      }
      prow[s] = v;
    }
  }
}

// Weights -> LDS (int32 fixed point; slots >= hi, the pads, get 0), a
// zeroed int64 gradient and hot row, the hot digit table; ends with a block
// barrier.
template <int REP>
__device__ __forceinline__ void hyb_lds_init(const DevPrepared& p, const float* wsrc, int64_t ns, int64_t hi,
                                             float wscale, int32_t* wl, unsigned long long* gl,
                                             uint32_t* whl, unsigned long long* hsum, uint32_t* wctr) {
  if (threadIdx.x == 0) *wctr = 0u;
  // 16-byte LDS stores (ns is a multiple of 64; wl and gl are 16-B aligned):
  // 4 weights and 2 gradient words per store instead of one; kInitU float4
  // loads per thread in flight before the first store (the tiered near tier
  // is ~3.3 float4 per thread: one L2 round trip instead of four)
  constexpr int kInitU = 4;
  for (int64_t q0 = threadIdx.x; q0 < ns / 4; q0 += int64_t(kIterBlock) * kInitU) {
    float4 wv[kInitU];
#pragma unroll
    for (int u = 0; u < kInitU; ++u) {
      const int64_t s4 = q0 + int64_t(u) * kIterBlock;
      wv[u] = s4 < ns / 4 ? *reinterpret_cast<const float4*>(wsrc + 4 * s4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kInitU; ++u) {
      const int64_t s4 = q0 + int64_t(u) * kIterBlock;
      if (s4 >= ns / 4) break;
      const int64_t s = 4 * s4;
      const float wf[4] = {wv[u].x, wv[u].y, wv[u].z, wv[u].w};
      int32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (s + k >= kNumNumeric && s + k < hi) ? w_to_fix(wf[k], wscale) : 0;
      reinterpret_cast<int4*>(wl)[s4] = make_int4(o[0], o[1], o[2], o[3]);
    }
  }
  for (int64_t s2 = threadIdx.x; s2 < ns * REP / 2; s2 += kIterBlock)
    reinterpret_cast<uint4*>(gl)[s2] = make_uint4(0u, 0u, 0u, 0u);
  for (int s = threadIdx.x; s < kHot + 8; s += kIterBlock) hsum[s] = 0ull;
  __syncthreads();
  if (threadIdx.x < kWave) hot_digits(p, wl, whl);
  __syncthreads();
}

template <bool STATS, bool SAMPLE, int REP, bool TIERED>
__global__ __launch_bounds__(kIterBlock) void k_sgd_iter_hyb(DevSgd d, DevPrepared p, SgdParams sp) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds[];
  __shared__ int64_t wsc[kIterBlock / kWave][kPartVals];
  __shared__ unsigned long long hsum[kHot + 8];
  __shared__ int32_t fdot[TIERED ? kIterBlock / kWave : 1][kRowsPerChunk];
  __shared__ __attribute__((aligned(16))) uint32_t whl[kLanesPerRow * kHotLdsStride];
  __shared__ int stop_flag;
  __shared__ uint32_t wctr;
  __shared__ IterScale scs;
  uint64_t* tst = nullptr;
  if (d.tdbg && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    tst = d.tdbg + (int64_t(sp.iteration) * 2 + (blockIdx.x == 0 ? 0 : 1)) * 8;
  if (tst) tst[0] = __builtin_amdgcn_s_memrealtime();
  kdbg_stamp(d.kdbg, sp.iteration, 0, 0);
  if (sgd_prologue(d, sp, &stop_flag, &scs)) return;
  const LaneScale sc = lane_scale(scs, d, lane_id() % kLanesPerRow);
  if (tst) tst[1] = __builtin_amdgcn_s_memrealtime();
  int32_t* wl = lds;
  unsigned long long* gl = reinterpret_cast<unsigned long long*>(lds + d.nl);
  hyb_lds_init<REP>(p, d.wc32, d.nl, d.far_base, sc.wscale, wl, gl, whl, hsum, &wctr);
  if (tst) tst[2] = __builtin_amdgcn_s_memrealtime();
  hyb_pass<STATS, SAMPLE, REP, TIERED>(d, p, sp, sc, wl, gl, whl, hsum, wsc,
                                       d.part + int64_t(blockIdx.x) * d.pstride, &wctr, fdot, tst);
  if (tst) tst[6] = __builtin_amdgcn_s_memrealtime();
  if (d.kdbg) {
    __syncthreads();
    kdbg_stamp(d.kdbg, sp.iteration, 0, 1);
  }
}

// LDS bytes of the fast path for a given replication factor.
static int64_t lds_bytes(int64_t ns, int rep) {
  return ns * int64_t(sizeof(int32_t)) + ns * rep * int64_t(sizeof(unsigned long long));
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
  // static LDS of k_sgd_iter_hyb<.., TIERED>: wsc, fdot per wave + hot row, whl, scales, flags
  const int64_t statics = int64_t(kIterBlock / kWave) *
                              (kPartVals * int64_t(sizeof(int64_t)) + kRowsPerChunk * int64_t(sizeof(int32_t))) +
                          (kHot + 8) * int64_t(sizeof(int64_t)) +
                          kLanesPerRow * kHotLdsStride * int64_t(sizeof(uint32_t)) + int64_t(sizeof(IterScale)) + 64;
  return ns <= kMaxHybridSlots && rep > 0 && lds_bytes(ns, rep) + statics <= 160 * 1024 - 1024;
}

template <bool STATS, bool SAMPLE>
static void launch_iter_t(const DevSgd& d, const DevPrepared& p, const SgdParams& sp, bool u16,
                          int rep, int grid, hipStream_t s) {
  if (u16 && rep > 0 && p.hybrid) {
    const size_t lds = size_t(lds_bytes(d.nl, rep));
#define TWTML_HYB(R, T) \
  TWTML_LAUNCH((k_sgd_iter_hyb<STATS, SAMPLE, R, T>), dim3(grid), dim3(kIterBlock), lds, s, d, p, sp)
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
  TWTML_LAUNCH((k_sgd_iter_lds<STATS, SAMPLE, R, C>), dim3(grid), dim3(kIterBlock), lds, s, d, p, sp)
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
//                 so all workgroups -- and all DP ranks -- agree) and derives
//                 iteration i's fixed-point scales; workgroup 0 records them
//                 and publishes state[0..1] and the host flag.  Then one int64
//                 partial row per workgroup.
//   k_far_grad    (tiered) far slots' int64 sums into gacc[far_off ..].
//   [DP: k_sgd_reduce sums the partial rows into gacc[0, nl + 2), adds rank
//    0's verdict on update i-1 and this rank's ready word to the tail, and
//    ONE int64 all-reduce covers the whole packed buffer (near columns, loss,
//    sampled m, verdict, ready words, far slots): integer sums, so the
//    result is exact and the same on every rank whatever the backend's
//    summation order.  k_sgd_update i acts on the agreed verdict.  Each rank
//    skips the gradient pass of iteration i on its own verdict (state[8];
//    identical weights -> the same verdict everywhere) and then contributes
//    zeros, but only the agreed verdict ends the loop, so ranks can never
//    disagree on the iteration count (a mismatch would pair unequal
//    collectives).]
//   k_sgd_update  (iteration i)  multi-workgroup: sums the partial rows of
//                 64 columns (world 1) or reads the all-reduced gacc, and
//                 (tiered) updates the far slots in fixed slot ranges,
//                 SimpleUpdater on them, per-workgroup ||dw||^2, ||w||^2,
//                 max |w_text| into record i.
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
// sums -- int64 (exact) for the fixed-point columns, fp64 in a fixed order
// for the batch-stat columns.
// nparts > 0: the column sums come from the partial rows (single GPU);
// nparts == 0: gacc holds them (all-reduced).
// ---------------------------------------------------------------------------

// Sum of partial rows for columns [col0, col0 + 64): returns lane's column
// sum in wave 0 (other waves: 0); columns >= dcol0 are fp64 (bits returned).
// Contains a block barrier.
__device__ __forceinline__ int64_t part_block_sum(const DevSgd& d, int64_t col0, int64_t ncols, int64_t dcol0,
                                                  int nparts, int64_t (*red)[kWave]) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int64_t col = col0 + lane;
  const bool dbl = col >= dcol0;
  int64_t acc = 0;
  double accd = 0.0;
  if (col < ncols) {
    const int64_t* src = d.part + col;
    const int64_t ps = d.pstride;
    if (!dbl) {
#pragma unroll 16
      for (int g = w; g < nparts; g += kUpdWaves) acc += src[int64_t(g) * ps];
    } else {
      for (int g = w; g < nparts; g += kUpdWaves) accd += __builtin_bit_cast(double, src[int64_t(g) * ps]);
      acc = __builtin_bit_cast(int64_t, accd);
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  int64_t t = 0;
  if (w == 0) {
    if (!dbl) {
#pragma unroll
      for (int k = 0; k < kUpdWaves; ++k) t += red[k][lane];
    } else {
      double td = 0.0;
      for (int k = 0; k < kUpdWaves; ++k) td += __builtin_bit_cast(double, red[k][lane]);
      t = __builtin_bit_cast(int64_t, td);
    }
  }
  __syncthreads();   // red is reused by the next column block
  return t;
}

// Host flag of update it-1 (zero-copy): stop bit, DP "every rank's next
// batch is locally prepared" bit, and the largest ready active-set size.
__device__ __forceinline__ double flag_word(bool stop, bool all_ready, int64_t max_u) {
  return double(stop ? 1 : 0) + 2.0 * double(all_ready ? 1 : 0) + 4.0 * double(max_u);
}

// One Hillis-Steele step of a segmented 64-bit sum: lanes without a DPP
// source (or outside ROWS) see slot ~0 and add nothing.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v) {
  return uint32_t(__builtin_amdgcn_update_dpp(int(old), int(v), CTRL, ROWS, 0xf, false));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_scan_step(long long& q, uint32_t sl) {
  const uint32_t lo = dpp_u32<CTRL, ROWS>(0u, uint32_t(uint64_t(q)));
  const uint32_t hi = dpp_u32<CTRL, ROWS>(0u, uint32_t(uint64_t(q) >> 32));
  const uint32_t su = dpp_u32<CTRL, ROWS>(0xFFFFFFFFu, sl);
  if (su == sl) q += (long long)((uint64_t(hi) << 32) | lo);
}

// Segmented inclusive sum over the wave of far CSC entries e (slot-sorted):
// q = rint(residual of the entry's row * 2^S); the last lane of each run of
// equal slots returns true with the run's sum in q.  DPP row shifts, then the
// row broadcasts across the four 16-lane rows: the CSC is slot-sorted, so a
// lane k places back is in this lane's run iff it holds the same slot.
__device__ __forceinline__ bool far_seg_scan(int64_t e, int64_t n, uint32_t sl, long long& q) {
  const int lane = lane_id();
  const bool valid = e < n;
  seg_scan_step<0x111, 0xf>(q, sl);   // row_shr:1
  seg_scan_step<0x112, 0xf>(q, sl);   // row_shr:2
  seg_scan_step<0x114, 0xf>(q, sl);   // row_shr:4
  seg_scan_step<0x118, 0xf>(q, sl);   // row_shr:8
  seg_scan_step<0x142, 0xa>(q, sl);   // row_bcast:15 -> rows 1, 3
  seg_scan_step<0x143, 0xc>(q, sl);   // row_bcast:31 -> rows 2, 3
  const uint32_t sn = uint32_t(__shfl_down(int(sl), 1, kWave));
  return valid && (lane == kWave - 1 || e + 1 >= n || sn != sl);
}


// Update workgroups.  Blocks [0, nt) own 64-column tiles of the near (LDS)
// slots, grid-stride over nt; blocks [nt, nt + nf) own far slot range k =
// [n_far k / nf, n_far (k + 1) / nf) of the tiered layout, read from the far
// gradient sums (k_far_grad; DP: the all-reduced packed buffer).  The near
// tiles and the far ranges run side by side instead of every block doing a
// tile and then a grid-stride share of the far slots (under prep overlap
// the kernel tables show no measurable change: r3 27-32 us, r4 30-35 us;
// 21 us alone, profiles/r4/pmc_summary.md).  Measured and reverted: far blocks summing their
// range's CSC segments themselves (no k_far_grad) -- the far entries are
// skewed over slot ranges, and the slowest block made the update ~100 us.
// The grouping is a function of the layout only, so the fp64 norm partials
// (and the convergence verdicts) are the same bits on one GPU and in DP.
__global__ __launch_bounds__(kUpdThreads) void k_sgd_update(DevSgd d, SgdParams sp, int nparts, int nt, int nf) {
  __shared__ double wsc[kUpdWaves][3];
  __shared__ int64_t red[kUpdWaves][kWave];
  __shared__ double m_sh;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  const int it = sp.iteration;
  kdbg_stamp(d.kdbg, it, 2, 0);
  const int64_t ns = d.nl, hi = d.far_base;   // partial-row columns; near text slots end at far_base
  int64_t* tail = d.gacc + ns;
  const int64_t n_far = kNumNumeric + d.n_unique - d.far_base;
  int64_t* gfar = d.gacc + d.far_off;
  if (sp.dp) {
    // the agreed verdict on update it - 1 (checked before state[0]: block 0
    // sets it below while other blocks may still start), and the ready words
    const bool stop = it > 1 && tail[kTailVerdict] != 0;
    if (blockIdx.x == 0 && tid == 0 && d.host_flags) {
      bool all = true;
      int64_t mx = 0;
      for (int r = 0; r < d.world; ++r) {
        const int64_t v = tail[kTailReady + r];
        all = all && v > 0;
        mx = v - 1 > mx ? v - 1 : mx;
      }
      __hip_atomic_store(&d.host_flags[it - 1], flag_word(stop, all, mx), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (stop) {
      for (int64_t j = int64_t(blockIdx.x) * kUpdThreads + tid; j < n_far; j += int64_t(gridDim.x) * kUpdThreads)
        gfar[j] = 0;   // this pass's far sums are dropped
      if (blockIdx.x == 0 && tid == 0) {
        d.state[0] = 1.0;
        if (d.state[7] == 0.0) d.state[1] = 1.0;
      }
      return;
    }
  }
  const int64_t ncols = ns + kPartVals - kNumNumeric;
  // Single GPU: the first column tile's partial-row loads and its master
  // weights are issued before the batch-state / record loads are waited on
  // (they do not depend on them), so the kernel's dependent chain is one
  // memory round trip shorter; a block that then finds the batch finished
  // drops them.
  const int64_t col_first = int64_t(blockIdx.x) * kWave;
  if (sp.ablate == 10) nparts = 0;   // timing only: the update without its partial-row reads
  const bool pre = nparts > 0 && int(blockIdx.x) < nt;
  double wn_first = 0.0;
  if (pre && w == 0 && col_first + lane < hi) wn_first = d.wc64[col_first + lane];
  const int64_t gp_first = pre ? part_block_sum(d, col_first, ncols, ncols, nparts, red) : 0;
  if (d.state[0] != 0.0) return;
  const double* rec_it = sgd_rec(d, it);
  const int sS = int(rec_it[kRecS]), sL = int(rec_it[kRecL]);
  // m: global kept rows, or the sampled row count of this iteration
  if (tid < kWave) {
    double m = d.state[5];
    if (sp.sample) {
      int64_t t = 0;
      if (nparts > 0) {
        for (int g = tid; g < nparts; g += kWave) t += d.part[int64_t(g) * d.pstride + ns + 1];
        t = wave_sum_i64(t);
      } else {
        t = tail[kTailM];
      }
      m = double(t);
    }
    if (tid == 0) m_sh = m;
  }
  __syncthreads();
  const double m = m_sh;
  const double alpha = sp.step_size / sqrt(double(it));
  const double gsc = ldexp(1.0, -sS);
  double ds = 0.0, ws = 0.0, mx = 0.0;
  if (int(blockIdx.x) < nt) {
    for (int64_t col0 = col_first; col0 < ncols; col0 += int64_t(nt) * kWave) {
      const bool first = pre && col0 == col_first;
      const int64_t gp = first ? gp_first : (nparts > 0 ? part_block_sum(d, col0, ncols, ncols, nparts, red) : 0);
      const int64_t col = col0 + lane;
      if (w == 0 && col < ncols) {
        const int64_t gi = (nparts > 0 ? gp : (col <= ns + 1 ? d.gacc[col] : 0));
        if (col < hi) {
          double wn = first ? wn_first : d.wc64[col];
          if (m > 0.0) {
            const double g = double(gi) * (col < kNumNumeric ? ldexp(1.0, -int(rec_it[kRecN + col])) : gsc);
            const double step = alpha * (g / m);
            wn -= step;
            d.wc64[col] = wn;
            d.wc32[col] = float(wn);
            ds += step * step;
            ws += wn * wn;
          }
          if (col >= kNumNumeric) mx = fmax(mx, fabs(double(float(wn))));   // the next iteration's weight scale
        } else if (col == ns) {
          if (m > 0.0) d.loss_hist[it] = 0.5 * double(gi) * ldexp(1.0, -sL) / m;
        }
      }
    }
  } else if (n_far > 0) {
    // tiered: far slots [far_base + jlo, far_base + jhi) from the far
    // gradient sums (k_far_grad; DP: all-reduced), re-zeroed here
    const int64_t k = int64_t(blockIdx.x) - nt;
    const int64_t jlo = n_far * k / nf, jhi = n_far * (k + 1) / nf;
    for (int64_t j = jlo + tid; j < jhi; j += kUpdThreads) {
      const double g = double(gfar[j]) * gsc;
      gfar[j] = 0;
      const int64_t col = d.far_base + j;
      double wn = d.wc64[col];
      if (m > 0.0) {
        // the near columns' formula bit for bit: which tier a slot lands in
        // depends on sampled counts (row placement), its update must not
        const double step = alpha * (g / m);
        wn -= step;
        d.wc64[col] = wn;
        d.wc32[col] = float(wn);
        ds += step * step;
        ws += wn * wn;
      }
      mx = fmax(mx, fabs(double(float(wn))));
    }
  }
  ds = wave_sum(ds);   // fixed order within the wave, then across waves
  ws = wave_sum(ws);
  mx = wave_max(mx);
  if (lane == 0) {
    wsc[w][0] = ds;
    wsc[w][1] = ws;
    wsc[w][2] = mx;
  }
  __syncthreads();
  double* rec = sgd_rec(d, it);   // (= rec_it)
  if (tid < 3) {
    double t = 0.0;
    for (int k = 0; k < kUpdWaves; ++k) t = tid < 2 ? t + wsc[k][tid] : fmax(t, wsc[k][tid]);
    rec[rec_part(tid, int(blockIdx.x))] = t;
  }
  if (blockIdx.x == 0 && tid == 0) {
    const double nupd = (it > 1 ? sgd_rec(d, it - 1)[0] : 0.0) + (m > 0.0 ? 1.0 : 0.0);
    rec[0] = nupd;
    rec[1] = m;
    rec[2] = double(gridDim.x);
    d.state[2] = nupd;
    d.state[3] = double(it);
  }
  if (d.kdbg) {
    __syncthreads();
    kdbg_stamp(d.kdbg, it, 2, 1);
  }
}

void launch_sgd_update(const DevSgd& d, const SgdParams& sp, int nparts, hipStream_t s) {
  const UpdSplit u = upd_split(d);
  TWTML_LAUNCH(k_sgd_update, dim3(u.nt + u.nf), dim3(kUpdThreads), 0, s, d, sp, nparts, u.nt, u.nf);
}

// DP: cross-workgroup reduction of the partial rows into the packed buffer
// gacc[0, nl + 2) (slots, loss, sampled count), rank 0's verdict on update
// i-1 and this rank's ready word into the tail -- all of it int64, ahead of
// the one all-reduce per iteration.
__global__ __launch_bounds__(kUpdThreads) void k_sgd_reduce(DevSgd d, SgdParams sp) {
  __shared__ int64_t red[kUpdWaves][kWave];
  if (d.state[0] != 0.0) return;
  // pass skipped on this rank's verdict: its partial rows are stale, it contributes zeros
  const bool skipped = d.state[8] == double(sp.iteration);
  const int64_t nl = d.nl;
  if (d.nparts > 0) {
    const int64_t ncols = nl + kPartVals - kNumNumeric;
    const int64_t col0 = int64_t(blockIdx.x) * kWave;
    const int64_t v = skipped ? 0 : part_block_sum(d, col0, ncols, ncols, d.nparts, red);
    const int64_t col = col0 + lane_id();
    if (threadIdx.x < kWave && col < ncols) d.gacc[col] = v;   // slots, loss, sampled count
  }
  if (blockIdx.x == 0 && threadIdx.x < kWave) {
    // rank 0's verdict on update i-1 (converged, or this iteration's scales invalid)
    const bool conv = sp.iteration > 1 && sgd_converged_wave(d, sp.iteration - 1, sp.tol);
    const bool bad = sgd_rec(d, sp.iteration)[kRecBad] != 0.0;
    int64_t* tail = d.gacc + nl;
    if (threadIdx.x == 0) tail[kTailVerdict] = ((conv || bad) && sp.rank0) ? 1 : 0;
    for (int r = threadIdx.x; r < d.tail_len - kTailReady; r += kWave)
      tail[kTailReady + r] = (r == d.rank && d.ready_word)
                                 ? int64_t(__hip_atomic_load(const_cast<int64_t*>(d.ready_word), __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_SYSTEM))
                                 : 0;
  }
}

void launch_sgd_reduce(const DevSgd& d, const SgdParams& sp, hipStream_t s) {
  const int grid = d.nparts > 0 ? int((d.nl + kPartVals - kNumNumeric + kWave - 1) / kWave) : 1;
  TWTML_LAUNCH(k_sgd_reduce, dim3(grid), dim3(kUpdThreads), 0, s, d, sp);
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

// RCCL-footprint stand-in (DP cost model, README): at the all-reduce point of
// every GD iteration, wgs workgroups move the packed gradient buffer's bytes
// (read n, write n int64) -- the CU share a ring all-reduce kernel holds on
// each rank beside the next batch's prep.  Its workgroup stamps give the
// dispatch ramp it meets there (TWTML_ITER_TIMING).
__global__ __launch_bounds__(256) void k_rccl_standin(const int64_t* src, int64_t* dst, int64_t n,
                                                      uint64_t* kdbg, int it) {
  kdbg_stamp(kdbg, it, 3, 0);
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) dst[i] = src[i];
  __syncthreads();
  kdbg_stamp(kdbg, it, 3, 1);
}

void launch_rccl_standin(const int64_t* src, int64_t* dst, int64_t n, int wgs, uint64_t* kdbg, int it,
                         hipStream_t s) {
  if (n <= 0 || wgs <= 0) return;
  TWTML_LAUNCH(k_rccl_standin, dim3(wgs), dim3(256), 0, s, src, dst, n, kdbg, it);
}

void launch_sgd_finish(const DevSgd& d, const SgdParams& sp, hipStream_t s) {
  TWTML_LAUNCH(k_sgd_finish, dim3(1), dim3(kWave), 0, s, d, sp);
}


// ---------------------------------------------------------------------------
// Far backward (tiered layout): the CSC lists every far entry grouped by
// slot; lane e of the grid takes entry e, converts its row's residual to
// the iteration's 2^S fixed point (the same q as the LDS tier), and a
// segmented inclusive scan over the wave (segments = runs of equal slot)
// leaves each run's sum in its last lane, which adds it to the packed
// buffer's far part with one 64-bit integer atomic.  Integer sums are exact,
// so the result does not depend on the order of entries inside a slot or on
// which wave adds first: deterministic across runs and DP ranks.
// ---------------------------------------------------------------------------
template <int kU>
__global__ __launch_bounds__(256) void k_far_grad(DevSgd d, SgdParams sp) {
  kdbg_stamp(d.kdbg, sp.iteration, 1, 0);
  if (d.state[0] != 0.0 || d.state[8] == double(sp.iteration)) return;   // done / DP pass skipped
  const int64_t n = *d.far_n;
  const int lane = lane_id();
  const float qscale = ldexpf(1.f, int(sgd_rec(d, sp.iteration)[kRecS]));
  unsigned long long* gfar = reinterpret_cast<unsigned long long*>(d.gacc + d.far_off);
  // kU 64-entry tiles per wave step: every tile's (slot, row) loads, then
  // every residual gather, are in flight before the scans (1 / kU of the
  // dependent round trips of one tile per step)
  const int64_t stride = int64_t(gridDim.x) * 256 * kU;
  for (int64_t e0 = (int64_t(blockIdx.x) * 256 + (threadIdx.x & ~(kWave - 1))) * kU; e0 < n; e0 += stride) {
    uint32_t sl[kU], ps[kU];
    float rv[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t e = e0 + u * kWave + lane;
      const uint2 v = e < n ? d.fcsc[e] : make_uint2(0u, 0xFFFFFFFFu);
      ps[u] = v.x;
      sl[u] = v.y;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) rv[u] = e0 + u * kWave + lane < n ? d.rbuf[ps[u]] : 0.f;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      long long q = (long long)__float2int_rn(rv[u] * qscale);
      if (far_seg_scan(e0 + u * kWave + lane, n, sl[u], q) && q != 0 && sp.ablate != 9)   // 9: no atomics (timing)
        atomicAdd(&gfar[sl[u] - d.far_base], (unsigned long long)q);
    }
  }
  if (d.kdbg) {
    __syncthreads();
    kdbg_stamp(d.kdbg, sp.iteration, 1, 1);
  }
}

void launch_far_grad(const DevSgd& d, const SgdParams& sp, int num_cu, hipStream_t s) {
  static const int ku = [] {
    // tiles per wave step: 4 (r5 A/B on the wide bench: 2 -> 231.9, 4 ->
    // 233.1, 8 -> 233.2 M tweets/s; 8 costs VGPRs for no further gain)
    const char* e = std::getenv("TWTML_FAR_U");
    const int v = e ? std::atoi(e) : 4;
    return v == 2 || v == 8 ? v : 4;
  }();
  const dim3 g(std::max(1, num_cu * 4));
  if (ku == 8) TWTML_LAUNCH(k_far_grad<8>, g, dim3(256), 0, s, d, sp);
  else if (ku == 4) TWTML_LAUNCH(k_far_grad<4>, g, dim3(256), 0, s, d, sp);
  else TWTML_LAUNCH(k_far_grad<2>, g, dim3(256), 0, s, d, sp);
}

// ---------------------------------------------------------------------------
// Gather / scatter between full-width fp64 weights and the compact space.
// ---------------------------------------------------------------------------
// Squared norms are reduced deterministically: each block writes its partial
// to d.nrm[blockIdx], one wave adds the partials in a fixed order (DP ranks
// hold identical weights, so their convergence verdicts must match bit for
// bit; float atomics would add in arrival order).
// mode 0: out = sum (+ mx_out = max of the max partials); 1: out = |w_rest|^2
// (state[4] - state[6]) + sum; 2: out = state[4]
__global__ void k_norm_sum(const double* parts, int n, double* out, const double* state, int mode, double* mx_out) {
  double acc = 0.0, mx = 0.0;
  for (int k = lane_id(); k < n; k += kWave) {
    acc += parts[k];
    if (mx_out) mx = fmax(mx, parts[kNormParts + k]);
  }
  acc = wave_sum(acc);
  mx = wave_max(mx);
  if (threadIdx.x == 0) {
    double base = 0.0;
    if (mode == 1) {             // rest of the previous batch + active part
      base = state[4] - state[6];
      if (base < 0.0) base = 0.0;
    }
    *out = mode == 2 ? state[4] : base + acc;
    if (mx_out) *mx_out = mx;
  }
}

__global__ __launch_bounds__(kBlock) void k_gather_w(DevSgd d, const int32_t* uniq) {
  __shared__ double scratch[kBlock / kWave];
  __shared__ double mscratch[kBlock / kWave];
  double acc = 0.0, mx = 0.0;
  const int64_t text_end = kNumNumeric + d.n_unique;
  for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < d.ns;
       s += int64_t(gridDim.x) * kBlock) {
    double v = 0.0;
    if (s < kNumNumeric) v = d.w64[d.F + s];
    else if (s < text_end) v = d.w64[d.slot_fid ? d.slot_fid[s] : uniq[s - kNumNumeric]];
    d.wc64[s] = v;
    d.wc32[s] = float(v);
    acc += v * v;
    if (s >= kNumNumeric && s < text_end) mx = fmax(mx, fabs(double(float(v))));
    if (s >= d.far_base && s < text_end) d.gacc[d.far_off + s - d.far_base] = 0;   // far sums start at 0
  }
  // packed near columns + tail start at 0 (single GPU never writes them; DP rewrites them)
  for (int64_t s = int64_t(blockIdx.x) * kBlock + threadIdx.x; s < d.nl + d.tail_len;
       s += int64_t(gridDim.x) * kBlock)
    d.gacc[s] = 0;
  acc = block_sum(acc, scratch);
  mx = wave_max(mx);
  if (lane_id() == 0) mscratch[threadIdx.x / kWave] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m2 = 0.0;
    for (int k = 0; k < kBlock / kWave; ++k) m2 = fmax(m2, mscratch[k]);
    d.nrm[blockIdx.x] = acc;
    d.nrm[kNormParts + blockIdx.x] = m2;
  }
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
    const int64_t id = s < kNumNumeric ? d.F + s : int64_t(d.slot_fid ? d.slot_fid[s] : uniq[s - kNumNumeric]);
    d.w64[id] = v;
    d.touched[id] = 1;   // the snapshot reads only written weights
    acc += v * v;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) d.nrm[blockIdx.x] = acc;
}

static int gather_grid(const DevSgd& d) {
  return std::max(1, std::min(ceil_div(std::max<int64_t>(d.ns, d.nl + d.tail_len), kBlock), kNormParts));
}
static int scatter_grid(const DevSgd& d) {
  return std::max(1, std::min(ceil_div(kNumNumeric + d.n_unique, kBlock), kNormParts));
}

void launch_gather_w(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  const int grid = gather_grid(d);
  TWTML_LAUNCH(k_gather_w, dim3(grid), dim3(kBlock), 0, s, d, p.uniq);
  TWTML_LAUNCH(k_norm_sum, dim3(1), dim3(kWave), 0, s, d.nrm, grid, &d.state[6], d.state, 0, &d.state[9]);
}

void launch_norm2(const double* v, int64_t n, double* out, const DevSgd& d, hipStream_t s) {
  int grid = ceil_div(n, kBlock * 8);
  if (grid > kNormParts) grid = kNormParts;
  if (grid < 1) grid = 1;
  TWTML_LAUNCH(k_norm2, dim3(grid), dim3(kBlock), 0, s, v, n, d.nrm);
  TWTML_LAUNCH(k_norm_sum, dim3(1), dim3(kWave), 0, s, d.nrm, grid, out, d.state, 0, (double*)nullptr);
}

void launch_scatter_w(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  TWTML_LAUNCH(k_scatter_w, dim3(scatter_grid(d)), dim3(kBlock), 0, s, d, p.uniq);
}

void launch_norm_next(const DevSgd& d, bool trained, hipStream_t s) {
  TWTML_LAUNCH(k_norm_sum, dim3(1), dim3(kWave), 0, s, d.nrm, trained ? scatter_grid(d) : 0,
                     d.wnorm_next, d.state, trained ? 1 : 2, (double*)nullptr);
}

__global__ void k_norm_carry(DevSgd d) {
  if (threadIdx.x == 0) d.state[4] = *d.wnorm_next;
}

void launch_norm_carry(const DevSgd& d, hipStream_t s) {
  TWTML_LAUNCH(k_norm_carry, dim3(1), dim3(kWave), 0, s, d);
}

// Per-batch SGD state in one launch: state (m = global kept rows at [5]),
// batch stats and the loss history.
__global__ void k_batch_init(DevSgd d, double m_global, int n_loss) {
  const int i = threadIdx.x;
  if (i < kStateLen) d.state[i] = i == 5 ? m_global : 0.0;
  if (i < 8) d.stats[i] = 0.0;
  if (i < kStatI) d.stat_i[i] = 0;
  for (int k = i; k < n_loss; k += blockDim.x) d.loss_hist[k] = 0.0;
}

void launch_batch_init(const DevSgd& d, double m_global, int n_loss, hipStream_t s) {
  TWTML_LAUNCH(k_batch_init, dim3(1), dim3(256), 0, s, d, m_global, n_loss);
}

// ---------------------------------------------------------------------------
// Batch bounds of the scale choice: max bigram count of a kept row, max |y|,
// max |n_k| (non-negative doubles order like their bit patterns: u64 max).
// ---------------------------------------------------------------------------
constexpr int32_t kNnzCountMask = (1 << 30) - 1;   // featurize.hip: nnz bits 0..29 = bigram count

// |x| of an fp32 as its bit pattern; NaN -> 0 (fmax ignored NaN inputs too).
__device__ __forceinline__ uint32_t abs_bits(uint32_t x) {
  const uint32_t a = x & 0x7FFFFFFFu;
  return a > 0x7F800000u ? 0u : a;
}

// Maxima of non-negative values are taken on their bit patterns (u32 for the
// fp32 inputs, exact), reduced per workgroup in LDS, and published with ONE
// atomic per value per workgroup: a wave-level atomicMax from every wave
// (12K same-address L2 atomics on a 1M-row batch) serialised this kernel at
// 146 us for 24 MB of input.
constexpr int kBoundsThreads = 1024;   // 16 waves per workgroup, 256 workgroups: 4 waves per SIMD in flight

__global__ __launch_bounds__(kBoundsThreads) void k_batch_bounds(DevPrepared p, double* out) {
  constexpr int kB = 2 + kNumNumeric;
  __shared__ uint32_t red[kBoundsThreads / kWave][kB];
  const int64_t n_kept = p.counters[0];
  const int64_t cap = p.cap_rows16;
  uint32_t b[kB] = {0, 0, 0, 0, 0, 0};
  const uint32_t* yb = reinterpret_cast<const uint32_t*>(p.y);
  const uint32_t* nb = reinterpret_cast<const uint32_t*>(p.num);
  // 4 rows per thread per step: six 16-B loads in flight (a row per step left
  // one wave per SIMD waiting on 6 dependent-latency loads: 64 us for 24 MB)
  const int64_t gid = int64_t(blockIdx.x) * kBoundsThreads + threadIdx.x, gstride = int64_t(gridDim.x) * kBoundsThreads;
  const int64_t n4 = n_kept >> 2;
  for (int64_t i4 = gid; i4 < n4; i4 += gstride) {
    const int4 z = reinterpret_cast<const int4*>(p.nnz)[i4];
    const uint4 yv = reinterpret_cast<const uint4*>(yb)[i4];
    uint4 nv[kNumNumeric];
#pragma unroll
    for (int k = 0; k < kNumNumeric; ++k) nv[k] = reinterpret_cast<const uint4*>(nb + int64_t(k) * cap)[i4];
    b[0] = max(b[0], max(max(uint32_t(z.x & kNnzCountMask), uint32_t(z.y & kNnzCountMask)),
                         max(uint32_t(z.z & kNnzCountMask), uint32_t(z.w & kNnzCountMask))));
    b[1] = max(b[1], max(max(abs_bits(yv.x), abs_bits(yv.y)), max(abs_bits(yv.z), abs_bits(yv.w))));
#pragma unroll
    for (int k = 0; k < kNumNumeric; ++k)
      b[2 + k] = max(b[2 + k], max(max(abs_bits(nv[k].x), abs_bits(nv[k].y)), max(abs_bits(nv[k].z), abs_bits(nv[k].w))));
  }
  for (int64_t i = 4 * n4 + gid; i < n_kept; i += gstride) {   // the last n_kept % 4 rows
    b[0] = max(b[0], uint32_t(p.nnz[i] & kNnzCountMask));
    b[1] = max(b[1], abs_bits(yb[i]));
#pragma unroll
    for (int k = 0; k < kNumNumeric; ++k) b[2 + k] = max(b[2 + k], abs_bits(nb[int64_t(k) * cap + i]));
  }
  const int w = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < kB; ++k) {
    const uint32_t v = wave_max(b[k]);
    if (lane_id() == 0) red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < kB) {
    const int k = threadIdx.x;
    uint32_t v = 0;
    for (int j = 0; j < kBoundsThreads / kWave; ++j) v = max(v, red[j][k]);
    const double dv = k == 0 ? double(v) : double(__builtin_bit_cast(float, v));
    if (dv > 0.0)
      atomicMax(reinterpret_cast<unsigned long long*>(&out[k]), __builtin_bit_cast(unsigned long long, dv));
  }
}

void launch_batch_bounds(const DevPrepared& p, double* out, hipStream_t s, bool zeroed) {
  // zeroed: k_prep_init cleared them earlier in this prep
  if (!zeroed) TWTML_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(double) * kBoundsLen, s));
  const int grid = int(std::max<int64_t>(1, std::min<int64_t>((p.cap_rows + kBoundsThreads - 1) / kBoundsThreads, 256)));
  TWTML_LAUNCH(k_batch_bounds, dim3(grid), dim3(kBoundsThreads), 0, s, p, out);
}

// ---------------------------------------------------------------------------
// Exact batch statistics (K7; LinearRegression.scala:59-65: count, stdev of
// the labels and of the rounded predictions, MSE).  Every kept row's label y
// (a retweet count) and rounded prediction p (pbuf, written by iteration 1)
// are integers, so with |y|, |p| < 2^31 the six moments are int64 sums --
// n, sum y, sum p exactly, y^2 / p^2 / (y - p)^2 (< 2^64) in two 32-bit limbs
// each -- which no summation order changes: one GPU, any DP sharding and any
// all-reduce order (ncclInt64) give the same bits.  Rows outside that range
// (predictions beyond 2^31 retweets: a model close to divergence) are
// counted and summed in fp64 ("spill"; DP order then matters for them only).
// Block partials -> stat_part, one wave adds them in block order
// (k_batch_stats_fin): deterministic, no atomics.
//   stat_i: [0] n  [1] sum y  [2] sum p  [3,4] sum y^2 hi/lo  [5,6] sum p^2
//           hi/lo  [7,8] sum (y-p)^2 hi/lo  [9] spill rows
//   stats (fp64, spill rows): [0] n [1] sum y [2] sum y^2 [3] sum p [4] sum p^2 [5] sum (y-p)^2
// ---------------------------------------------------------------------------
constexpr int kStatThreads = 256;   // (1024 threads: 14 -> 25 us under prep overlap, waiting for 16 free wave slots per CU)

__global__ __launch_bounds__(kStatThreads) void k_batch_stats(DevSgd d, const float* y, const int64_t* counters) {
  __shared__ int64_t wi[kStatThreads / kWave][kStatI];
  __shared__ double wf[kStatThreads / kWave][6];
  // no prequential pass on this batch (diverged at iteration 1; DP: skipped)
  const bool none = d.state[0] != 0.0 || d.state[8] == 1.0;
  const int64_t n_kept = none ? 0 : counters[0];
  int64_t a[kStatI];
  double f[6];
#pragma unroll
  for (int k = 0; k < kStatI; ++k) a[k] = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) f[k] = 0.0;
  constexpr float kLim = 2147483648.0f;   // 2^31
  for (int64_t pos = int64_t(blockIdx.x) * kStatThreads + threadIdx.x; pos < n_kept;
       pos += int64_t(gridDim.x) * kStatThreads) {
    const float yv = y[pos], pv = d.pbuf[pos];
    if (fabsf(yv) < kLim && fabsf(pv) < kLim) {   // NaN fails the test: spill
      const int64_t Y = int64_t(yv), P = int64_t(pv);
      const uint64_t ay = uint64_t(Y < 0 ? -Y : Y), ap = uint64_t(P < 0 ? -P : P);
      const int64_t E = Y - P;
      const uint64_t ae = uint64_t(E < 0 ? -E : E);   // < 2^32
      const uint64_t y2 = ay * ay, p2 = ap * ap, e2 = ae * ae;
      a[0] += 1; a[1] += Y; a[2] += P;
      a[3] += int64_t(y2 >> 32); a[4] += int64_t(y2 & 0xFFFFFFFFull);
      a[5] += int64_t(p2 >> 32); a[6] += int64_t(p2 & 0xFFFFFFFFull);
      a[7] += int64_t(e2 >> 32); a[8] += int64_t(e2 & 0xFFFFFFFFull);
    } else {
      const double yd = double(yv), pd = double(pv), e = yd - pd;
      a[9] += 1;
      f[0] += 1.0; f[1] += yd; f[2] += yd * yd; f[3] += pd; f[4] += pd * pd; f[5] += e * e;
    }
  }
  const int w = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < kStatI; ++k) {
    const int64_t v = wave_sum_i64(a[k]);
    if (lane_id() == 0) wi[w][k] = v;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double v = wave_sum(f[k]);
    if (lane_id() == 0) wf[w][k] = v;
  }
  __syncthreads();
  int64_t* out = d.stat_part + int64_t(blockIdx.x) * 16;
  if (threadIdx.x < kStatI) {
    int64_t v = 0;
    for (int k = 0; k < kStatThreads / kWave; ++k) v += wi[k][threadIdx.x];
    out[threadIdx.x] = v;
  } else if (threadIdx.x < kStatI + 6) {
    double v = 0.0;
    for (int k = 0; k < kStatThreads / kWave; ++k) v += wf[k][threadIdx.x - kStatI];
    out[threadIdx.x] = __builtin_bit_cast(int64_t, v);
  }
}

// Block partials -> totals: lane l of wave w holds block w * 64 + l's
// partials (all loads in flight at once; a single lane walking the blocks
// was 256 dependent loads, ~70 us on the compute stream), a fixed butterfly
// per wave, then the 4 wave sums in order: deterministic for the fp64
// spill columns, exact for the int64 ones.
__global__ __launch_bounds__(kStatBlocks) void k_batch_stats_fin(DevSgd d, int nblocks) {
  __shared__ int64_t ws[kStatBlocks / kWave][kStatI + 6];
  const int b = threadIdx.x, lane = lane_id(), w = threadIdx.x / kWave;
  int64_t v[kStatI + 6];
#pragma unroll
  for (int k = 0; k < kStatI + 6; ++k) v[k] = b < nblocks ? d.stat_part[int64_t(b) * 16 + k] : 0;
#pragma unroll
  for (int k = 0; k < kStatI; ++k) {
    const int64_t t = wave_sum_i64(v[k]);
    if (lane == 0) ws[w][k] = t;
  }
#pragma unroll
  for (int k = kStatI; k < kStatI + 6; ++k) {
    const double t = wave_sum(b < nblocks ? __builtin_bit_cast(double, v[k]) : 0.0);
    if (lane == 0) ws[w][k] = __builtin_bit_cast(int64_t, t);
  }
  __syncthreads();
  const int k = threadIdx.x;
  if (k < kStatI) {
    int64_t t = 0;
    for (int j = 0; j < kStatBlocks / kWave; ++j) t += ws[j][k];
    d.stat_i[k] = t;
  } else if (k < kStatI + 6) {
    double t = 0.0;
    for (int j = 0; j < kStatBlocks / kWave; ++j) t += __builtin_bit_cast(double, ws[j][k]);
    d.stats[k - kStatI] = t;
  }
}

// The batch's results for the host -- model statistics (fp64 spill sums and
// the exact int64 moments), batch state, loss history -- written straight
// into mapped host memory by one launch (four small D2H copies were four
// blit kernels on the compute stream, ~14 us each under prep overlap).
__global__ __launch_bounds__(256) void k_batch_out(DevSgd d, double* out, int64_t* stat, int n_loss) {
  const int t = threadIdx.x;
  if (t < 8) out[t] = d.stats[t];
  else if (t < 16) out[t] = d.state[t - 8];
  else if (t < 16 + kStatI) stat[t - 16] = d.stat_i[t - 16];
  for (int i = t; i < n_loss; i += 256) out[16 + i] = d.loss_hist[i];
}

void launch_batch_out(const DevSgd& d, double* out, int64_t* stat, int n_loss, hipStream_t s) {
  TWTML_LAUNCH(k_batch_out, dim3(1), dim3(256), 0, s, d, out, stat, n_loss);
}

void launch_batch_stats(const DevSgd& d, const DevPrepared& p, hipStream_t s) {
  TWTML_LAUNCH(k_batch_stats, dim3(kStatBlocks), dim3(kStatThreads), 0, s, d, p.y, p.counters);
  TWTML_LAUNCH(k_batch_stats_fin, dim3(1), dim3(kStatBlocks), 0, s, d, kStatBlocks);
}

// ---------------------------------------------------------------------------
// Plot sample (output op #1's real / pred collect, LinearRegression.scala:77):
// P evenly spaced kept rows, out[2i] = pred, out[2i + 1] = real, so only P
// pairs cross PCIe when the Lightning plot is on.
// ---------------------------------------------------------------------------
__global__ void k_plot_sample(const float* pred, const float* real, int64_t n, int64_t P, float* out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < P; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = P > 1 ? (i * (n - 1)) / (P - 1) : 0;
    out[2 * i] = pred[r];
    out[2 * i + 1] = real[r];
  }
}

void launch_plot_sample(const float* pred, const float* real, int64_t n, int64_t P, float* out, hipStream_t s) {
  if (P <= 0 || n <= 0) return;
  const int grid = int(std::min<int64_t>(64, (P + 255) / 256));
  TWTML_LAUNCH(k_plot_sample, dim3(grid), dim3(256), 0, s, pred, real, n, P, out);
}

}  // namespace twtml
