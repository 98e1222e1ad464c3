// Standalone check of the DPP / permlane wave reductions in csrc/hip/common.h.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "../../csrc/hip/common.h"
using namespace twtml;
__global__ void k(const float* in, float* out_sum, float* out_mod4) {
  const float v = in[threadIdx.x];
  out_sum[threadIdx.x] = wave_sum_f32(v);
  out_mod4[threadIdx.x] = row_sum_mod4(v);
}
int main() {
  float h[64], s[64], m[64];
  for (int i = 0; i < 64; ++i) h[i] = float(1 << (i % 16)) + 0.001f * i;
  float *d, *ds, *dm;
  hipMalloc(&d, 256); hipMalloc(&ds, 256); hipMalloc(&dm, 256);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, ds, dm);
  hipMemcpy(s, ds, 256, hipMemcpyDeviceToHost);
  hipMemcpy(m, dm, 256, hipMemcpyDeviceToHost);
  double tot = 0; for (int i = 0; i < 64; ++i) tot += h[i];
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    double e = 0; for (int j = (i / 16) * 16 + i % 4; j < (i / 16) * 16 + 16; j += 4) e += h[j];
    if (std::fabs(s[i] - tot) > 1e-2 * std::fabs(tot)) { if (bad < 4) printf("sum lane %d got %g want %g\n", i, s[i], tot); ++bad; }
    if (std::fabs(m[i] - e) > 1e-2 * std::fabs(e)) { if (bad < 8) printf("mod4 lane %d got %g want %g\n", i, m[i], e); ++bad; }
  }
  printf("dpp_check: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);
  return bad ? 1 : 0;
}
