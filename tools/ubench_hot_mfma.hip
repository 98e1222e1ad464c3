// Micro-benchmark: the hot tile of the LR gradient kernel (sgd.hip hyb_pass)
// on the VALU path it uses (v_dot4 over 4-bit counts x base-128 weight
// digits, pk_fma backward) against a matrix-core variant (forward as two
// v_mfma_i32_16x16x64_i8 per 16-row chunk: A = the chunk's 16 x 128 counts,
// B = 128 x 16 digit table with 4 used columns; backward stays VALU -- a
// GEMV has no N dimension to give the MFMA).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_hot_mfma tools/ubench_hot_mfma.hip
//   /tmp/ubench_hot_mfma [rows]
//
// Both kernels read the same bytes per chunk (16 B of counts per lane + the
// row labels), compute the row dots exactly in int32 per digit, the
// residuals, and accumulate the 128 hot gradients; results are checked
// against each other and against a host reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kWave = 64, kHot = 128, kRows = 16;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void nib_split(uint32_t x, uint32_t& lo, uint32_t& hi) {
  lo = x & 0x0F0F0F0Fu;
  hi = (x >> 4) & 0x0F0F0F0Fu;
}

// ---- VALU path (layout of hot_split.hip: lane 4r + t holds row r's ids
// 32t..32t+31; nibble k of dword q = id 32t + 8q + k) -------------------------
__global__ __launch_bounds__(256) void k_valu(const uint4* hot, const float* y, int64_t nch,
                                              const uint32_t* wtab, float* res_out, float* grad) {
  __shared__ __attribute__((aligned(16))) uint32_t wl[4 * 36];
  for (int i = threadIdx.x; i < 4 * 36; i += 256) wl[i] = wtab[i];
  __syncthreads();
  const int lane = threadIdx.x % kWave, r = lane / 4, t = lane % 4;
  const uint32_t* wq = wl + t * 36;
  f32x2 gh[16];
  for (int i = 0; i < 16; ++i) gh[i] = f32x2{0.f, 0.f};
  const int64_t wave = (int64_t(blockIdx.x) * 256 + threadIdx.x) / kWave, wave0 = wave;
  const int64_t nw = int64_t(gridDim.x) * 256 / kWave;
  for (int64_t c = wave; c < nch; c += nw) {
    const uint4 hv = hot[c * kWave + lane];
    const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w};
    int acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint4 a = reinterpret_cast<const uint4*>(wq)[2 * d], b = reinterpret_cast<const uint4*>(wq)[2 * d + 1];
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
    float dot = float(acc[0]) * sc.x + float(acc[1]) * sc.y + float(acc[2]) * sc.z + float(acc[3]) * sc.w;
    dot += __shfl_xor(dot, 1, kWave);
    dot += __shfl_xor(dot, 2, kWave);
    const float res = dot - y[c * kRows + r];
    if (t == 0) res_out[c * kRows + r] = res;
    const f32x2 r2 = {res, res};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t lo, hi;
      nib_split(hw[q], lo, hi);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 cc = {float((lo >> (8 * i)) & 0xFFu), float((hi >> (8 * i)) & 0xFFu)};
        gh[4 * q + i] = __builtin_elementwise_fma(cc, r2, gh[4 * q + i]);
      }
    }
  }
  // gh[4q + i].x: id 32t + 8q + 2i, .y: id 32t + 8q + 2i + 1 -> sum over the 16 rows
  for (int i = 0; i < 32; ++i) {
    float v = (i & 1) ? gh[i >> 1].y : gh[i >> 1].x;
    v += __shfl_xor(v, 4, kWave);
    v += __shfl_xor(v, 8, kWave);
    v += __shfl_xor(v, 16, kWave);
    v += __shfl_xor(v, 32, kWave);
    const int q = (i >> 1) / 4, ii = (i >> 1) % 4;
    const int id = 32 * t + 8 * q + 2 * ii + (i & 1);
    if (r == 0) grad[wave0 * kHot + id] = v;   // per-wave partial row (no atomics)
  }
}

// ---- MFMA path (lane 16g + r holds row r's ids 16g + j in dwords 0-1 and
// 64 + 16g + j in dwords 2-3; within a dword, id j (of 8) sits in nibble
// 2j (j < 4) or 2(j - 4) + 1, so nib_split yields bytes in k order) ----------
__global__ __launch_bounds__(256) void k_mfma(const uint4* hot, const float* y, int64_t nch,
                                              const v4i* bfrag, const float* dscale, float* res_out,
                                              float* grad) {
  const int lane = threadIdx.x % kWave, r = lane & 15, g = lane >> 4;
  const v4i b0 = bfrag[lane], b1 = bfrag[kWave + lane];
  const float scl = (lane & 15) < 4 ? dscale[lane & 15] : 0.f;
  f32x2 gh[16];
  for (int i = 0; i < 16; ++i) gh[i] = f32x2{0.f, 0.f};
  const int64_t wave = (int64_t(blockIdx.x) * 256 + threadIdx.x) / kWave, wave0 = wave;
  const int64_t nw = int64_t(gridDim.x) * 256 / kWave;
  for (int64_t c = wave; c < nch; c += nw) {
    const uint4 hv = hot[c * kWave + lane];
    uint32_t l0, h0, l1, h1, l2, h2, l3, h3;
    nib_split(hv.x, l0, h0);
    nib_split(hv.y, l1, h1);
    nib_split(hv.z, l2, h2);
    nib_split(hv.w, l3, h3);
    const v4i a0 = {int(l0), int(h0), int(l1), int(h1)}, a1 = {int(l2), int(h2), int(l3), int(h3)};
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, acc, 0, 0, 0);
    // acc[k] = D[row 4g + k][col lane & 15]; digits are columns 0..3
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = float(acc[k]) * scl;
      v[k] += __shfl_xor(v[k], 1, kWave);
      v[k] += __shfl_xor(v[k], 2, kWave);
    }
    // row r's dot sits in lane 16 (r >> 2), register r & 3
    const int src = 16 * (r >> 2);
    float d0 = __shfl(v[0], src, kWave), d1 = __shfl(v[1], src, kWave);
    float d2 = __shfl(v[2], src, kWave), d3 = __shfl(v[3], src, kWave);
    const int k = r & 3;
    const float dot = k == 0 ? d0 : k == 1 ? d1 : k == 2 ? d2 : d3;
    const float res = dot - y[c * kRows + r];
    if (g == 0) res_out[c * kRows + r] = res;
    const f32x2 r2 = {res, res};
    const uint32_t lh[8] = {l0, h0, l1, h1, l2, h2, l3, h3};
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x2 cc = {float((lh[q] >> (16 * i)) & 0xFFu), float((lh[q] >> (16 * i + 8)) & 0xFFu)};
        gh[2 * q + i] = __builtin_elementwise_fma(cc, r2, gh[2 * q + i]);
      }
  }
  // gh[2q + i]: byte pair (2i, 2i+1) of fragment dword q -> k = 4q + 2i (+1)
  for (int e = 0; e < 32; ++e) {
    float v = (e & 1) ? gh[e >> 1].y : gh[e >> 1].x;
    v += __shfl_xor(v, 1, kWave);
    v += __shfl_xor(v, 2, kWave);
    v += __shfl_xor(v, 4, kWave);
    v += __shfl_xor(v, 8, kWave);
    const int q = (e >> 1) >> 1, i = (e >> 1) & 1;
    const int kk = 4 * q + 2 * i + (e & 1);          // byte index 0..31 of the two fragments
    const int id = kk < 16 ? 16 * g + kk : 64 + 16 * g + (kk - 16);
    if (r == 0) grad[wave0 * kHot + id] = v;
  }
}

int main(int argc, char** argv) {
  const int64_t R = argc > 1 ? std::atoll(argv[1]) : (1 << 20);
  const int64_t C = R / kRows;
  std::mt19937 rng(7);
  // counts: ~120 hot entries per row over 128 ids, Zipf-like (toy profile)
  std::vector<uint8_t> cnt(size_t(R) * kHot);
  std::vector<double> zipf(kHot);
  for (int h = 0; h < kHot; ++h) zipf[h] = 1.0 / (h + 3);
  std::discrete_distribution<int> pick(zipf.begin(), zipf.end());
  for (int64_t r = 0; r < R; ++r)
    for (int e = 0; e < 120; ++e) {
      uint8_t& c = cnt[size_t(r) * kHot + pick(rng)];
      if (c < 15) ++c;
    }
  std::vector<float> w(kHot);
  std::vector<float> y{};
  y.resize(size_t(R));
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : w) x = nd(rng) * 0.05f;
  for (auto& x : y) x = 100.f + 10.f * nd(rng);
  // balanced base-128 digits of a 28-bit fixed point (as sgd.hip hot_digits)
  float S = 0.f;
  for (float x : w) S = std::fmax(S, std::fabs(x));
  int8_t dig[kHot][4];
  for (int h = 0; h < kHot; ++h) {
    int32_t W = int32_t(std::rint(w[h] * (134217728.0f / S)));
    for (int d = 3; d > 0; --d) {
      const int32_t x = ((W + 64) & 127) - 64;
      dig[h][d] = int8_t(x);
      W = (W - x) >> 7;
    }
    dig[h][0] = int8_t(W);
  }
  const float s0 = S / 64.f, scale[4] = {s0, s0 / 128.f, s0 / 16384.f, s0 / 2097152.f};
  // VALU layout + digit table (4 quarters x 36 dwords)
  std::vector<uint32_t> hv(size_t(C) * kWave * 4, 0u), wtab(4 * 36, 0u);
  for (int64_t c = 0; c < C; ++c)
    for (int r = 0; r < kRows; ++r)
      for (int h = 0; h < kHot; ++h) {
        const int t = h / 32, q = (h % 32) / 8, k = h % 8;
        hv[(size_t(c) * kWave + 4 * r + t) * 4 + q] |= uint32_t(cnt[size_t(c * kRows + r) * kHot + h]) << (4 * k);
      }
  {
    uint8_t* bytes = reinterpret_cast<uint8_t*>(wtab.data());
    for (int h = 0; h < kHot; ++h) {
      const int t = h / 32, q = (h % 32) / 8, k = h % 8;
      for (int d = 0; d < 4; ++d) bytes[(t * 36 + (d * 4 + q) * 2 + (k & 1)) * 4 + (k >> 1)] = uint8_t(dig[h][d]);
    }
    for (int t = 0; t < 4; ++t) std::memcpy(&wtab[t * 36 + 32], scale, sizeof(scale));
  }
  // MFMA layout + B fragments
  std::vector<uint32_t> hm(size_t(C) * kWave * 4, 0u);
  auto nib_of = [](int j) { return j < 4 ? 2 * j : 2 * (j - 4) + 1; };
  for (int64_t c = 0; c < C; ++c)
    for (int r = 0; r < kRows; ++r)
      for (int g = 0; g < 4; ++g)
        for (int half = 0; half < 2; ++half)
          for (int j = 0; j < 16; ++j) {
            const int id = half * 64 + 16 * g + j;
            const int dw = half * 2 + j / 8;
            hm[(size_t(c) * kWave + 16 * g + r) * 4 + dw] |=
                uint32_t(cnt[size_t(c * kRows + r) * kHot + id]) << (4 * nib_of(j % 8));
          }
  std::vector<int8_t> bf(2 * kWave * 16, 0);
  for (int m = 0; m < 2; ++m)
    for (int l = 0; l < kWave; ++l)
      for (int j = 0; j < 16; ++j) {
        const int col = l & 15, k = 16 * (l >> 4) + j;
        bf[(m * kWave + l) * 16 + j] = col < 4 ? dig[m * 64 + k][col] : 0;
      }
  // host reference of the residuals / gradients
  std::vector<double> ref_res(static_cast<size_t>(R)), ref_g(kHot, 0.0);
  for (int64_t r = 0; r < R; ++r) {
    double dot = 0;
    for (int h = 0; h < kHot; ++h) {
      const double wq = dig[h][0] * double(scale[0]) + dig[h][1] * double(scale[1]) + dig[h][2] * double(scale[2]) +
                        dig[h][3] * double(scale[3]);
      dot += cnt[size_t(r) * kHot + h] * wq;
    }
    ref_res[size_t(r)] = dot - y[size_t(r)];
    for (int h = 0; h < kHot; ++h) ref_g[h] += cnt[size_t(r) * kHot + h] * ref_res[size_t(r)];
  }

  uint4 *d_hv, *d_hm;
  float *d_y, *d_res, *d_g, *d_sc;
  uint32_t* d_wt;
  v4i* d_bf;
  CK(hipMalloc(&d_hv, hv.size() * 4));
  CK(hipMalloc(&d_hm, hm.size() * 4));
  CK(hipMalloc(&d_y, y.size() * 4));
  CK(hipMalloc(&d_res, y.size() * 4));
  const int grid0 = 256 * 8;
  CK(hipMalloc(&d_g, size_t(grid0) * 4 * kHot * 4));
  CK(hipMalloc(&d_wt, wtab.size() * 4));
  CK(hipMalloc(&d_bf, bf.size()));
  CK(hipMalloc(&d_sc, 16));
  CK(hipMemcpy(d_hv, hv.data(), hv.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_hm, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_y, y.data(), y.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_wt, wtab.data(), wtab.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_bf, bf.data(), bf.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sc, scale, 16, hipMemcpyHostToDevice));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int grid = std::min(grid0, prop.multiProcessorCount * 8);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[2] = {"valu (v_dot4 fwd, pk_fma bwd)", "mfma (i8 16x16x64 fwd, pk_fma bwd)"};
  for (int which = 0; which < 2; ++which) {
    float best = 1e30f;
    for (int rep = 0; rep < 12; ++rep) {
      CK(hipEventRecord(e0));
      if (which == 0)
        hipLaunchKernelGGL(k_valu, dim3(grid), dim3(256), 0, 0, d_hv, d_y, C, d_wt, d_res, d_g);
      else
        hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, d_hm, d_y, C, d_bf, d_sc, d_res, d_g);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 2) best = std::fmin(best, ms);
    }
    std::vector<float> res(y.size()), part(size_t(grid) * 4 * kHot);
    std::vector<double> gr(kHot, 0.0);
    CK(hipMemcpy(res.data(), d_res, res.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(part.data(), d_g, part.size() * 4, hipMemcpyDeviceToHost));
    for (size_t wv = 0; wv < size_t(grid) * 4; ++wv)
      for (int h = 0; h < kHot; ++h) gr[h] += part[wv * kHot + h];
    double er = 0, eg = 0, gs = 0;
    for (int64_t r = 0; r < R; ++r) er = std::fmax(er, std::fabs(res[size_t(r)] - ref_res[size_t(r)]) / (std::fabs(ref_res[size_t(r)]) + 1.0));
    for (int h = 0; h < kHot; ++h) {
      eg = std::fmax(eg, std::fabs(gr[h] - ref_g[h]));
      gs = std::fmax(gs, std::fabs(ref_g[h]));
    }
    std::printf("%-40s rows %lld  best %.1f us  (%.1f us / 1M rows)  max rel err residual %.2e gradient %.2e\n",
                names[which], (long long)R, best * 1e3, best * 1e3 * 1048576.0 / double(R), er, eg / gs);
  }
  return 0;
}
