// Probe of the DPP reduction helpers (common.h) against a scalar reference on one wave.
#include <cstdio>
#include "../../sheeprl_prey_amd/ops/csrc/common.h"
using namespace srl;
__global__ void k(float* o, const float* x) {
  const float v = x[threadIdx.x];
  o[threadIdx.x] = row16_sum(v);
  o[64 + threadIdx.x] = row16_scan(v);
  o[128 + threadIdx.x] = row16_max(v);
  o[192 + threadIdx.x] = seg32_sum(v);
  o[256 + threadIdx.x] = seg32_scan(v);
  o[320 + threadIdx.x] = seg32_max(v);
  o[384 + threadIdx.x] = wave_sum_dpp(v);
}
int main() {
  float hx[64], ho[448];
  for (int i = 0; i < 64; ++i) hx[i] = (float)((i * 7) % 13) + 0.25f * i;
  float *dx, *dout;
  hipMalloc(&dx, sizeof hx);
  hipMalloc(&dout, sizeof ho);
  hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, dx);
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    float rs = 0, rsc = 0, rm = -1e30f, s32 = 0, sc32 = 0, m32 = -1e30f, ws = 0;
    for (int j = (i / 16) * 16; j < (i / 16) * 16 + 16; ++j) { rs += hx[j]; rm = hx[j] > rm ? hx[j] : rm; if (j <= i) rsc += hx[j]; }
    for (int j = (i / 32) * 32; j < (i / 32) * 32 + 32; ++j) { s32 += hx[j]; m32 = hx[j] > m32 ? hx[j] : m32; if (j <= i) sc32 += hx[j]; }
    for (int j = 0; j < 64; ++j) ws += hx[j];
    const float ref[7] = {rs, rsc, rm, s32, sc32, m32, ws};
    for (int f = 0; f < 7; ++f) {
      const float got = ho[64 * f + i];
      if (fabsf(got - ref[f]) > 1e-3f * (1.f + fabsf(ref[f]))) {
        if (bad < 20) printf("fn %d lane %d got %f want %f\n", f, i, got, ref[f]);
        ++bad;
      }
    }
  }
  printf("dpp probe: %d mismatches\n", bad);
  return bad != 0;
}
