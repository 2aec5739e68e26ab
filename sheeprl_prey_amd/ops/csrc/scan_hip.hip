#include "hip/hip_runtime.h"
// Reverse-time scans, one lane per column (the time loops of the reference run in Python):
//  * lambda-returns  (dreamer_v3/utils.py:44-55):  R_t = r_t + c_t*(1-lam)*v_t + c_t*lam*R_{t+1}, R_H = v_{H-1}
//    plus its adjoint (a forward scan) for the continuous-action dynamics-backprop path;
//  * GAE             (utils/utils.py:35-72).
#include "common.h"

namespace srl {

__global__ void __launch_bounds__(256) lambda_fwd_kernel(const float* __restrict__ r, const float* __restrict__ v,
                                                         const float* __restrict__ c, float* __restrict__ out, int H,
                                                         int M, float lam) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float nxt = v[(int64_t)(H - 1) * M + m];
  for (int t = H - 1; t >= 0; --t) {
    int64_t o = (int64_t)t * M + m;
    float ct = c[o];
    nxt = r[o] + ct * (1.f - lam) * v[o] + ct * lam * nxt;
    out[o] = nxt;
  }
}

__global__ void __launch_bounds__(256) lambda_bwd_kernel(const float* __restrict__ v, const float* __restrict__ c,
                                                         const float* __restrict__ ret, const float* __restrict__ g,
                                                         float* __restrict__ dr, float* __restrict__ dv,
                                                         float* __restrict__ dc, int H, int M, float lam) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float a = 0.f;
  for (int t = 0; t < H; ++t) {
    int64_t o = (int64_t)t * M + m;
    float prev_c = t > 0 ? c[o - M] : 0.f;
    a = g[o] + lam * prev_c * a;
    float ct = c[o];
    float rnext = (t + 1 < H) ? ret[o + M] : v[(int64_t)(H - 1) * M + m];
    dr[o] = a;
    dv[o] = a * ct * (1.f - lam);
    dc[o] = a * ((1.f - lam) * v[o] + lam * rnext);
  }
  // bootstrap R_H = v_{H-1}
  int64_t last = (int64_t)(H - 1) * M + m;
  dv[last] += lam * c[last] * a;
}

__global__ void __launch_bounds__(256) gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ done, const float* __restrict__ next_value,
                                                  float* __restrict__ ret, float* __restrict__ adv, int T, int N,
                                                  float gamma, float lam) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float last = 0.f;
  float nv = next_value[n];
  float nnt = 1.f - done[(int64_t)(T - 1) * N + n];
  for (int t = T - 1; t >= 0; --t) {
    int64_t o = (int64_t)t * N + n;
    if (t < T - 1) {
      nnt = 1.f - done[o];
      nv = val[o + N];
    }
    float delta = rew[o] + nv * nnt * gamma - val[o];
    last = delta + nnt * last * gamma * lam;
    adv[o] = last;
    ret[o] = last + val[o];
  }
}

}  // namespace srl

using namespace srl;

void launch_lambda_fwd(const float* r, const float* v, const float* c, float* out, int H, int M, float lam, hipStream_t st) {
  hipLaunchKernelGGL(lambda_fwd_kernel, dim3(cdiv(M, 256)), dim3(256), 0, st, r, v, c, out, H, M, lam);
}
void launch_lambda_bwd(const float* v, const float* c, const float* ret, const float* g, float* dr, float* dv, float* dc,
                       int H, int M, float lam, hipStream_t st) {
  hipLaunchKernelGGL(lambda_bwd_kernel, dim3(cdiv(M, 256)), dim3(256), 0, st, v, c, ret, g, dr, dv, dc, H, M, lam);
}
void launch_gae(const float* rew, const float* val, const float* done, const float* next_value, float* ret, float* adv, int T,
                int N, float gamma, float lam, hipStream_t st) {
  hipLaunchKernelGGL(gae_kernel, dim3(cdiv(N, 256)), dim3(256), 0, st, rew, val, done, next_value, ret, adv, T, N, gamma, lam);
}
