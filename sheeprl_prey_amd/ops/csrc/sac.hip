// Tanh-squashed Gaussian policy head (SAC / DroQ / SAC-AE actors), fp32.
//
// Reference semantics: sac/agent.py:100-138 (log_std clamped to [lo, hi]) and
// sac_ae/agent.py:227-320 (log_std = lo + (hi-lo)/2 * (tanh(raw)+1)):
//   std = exp(ls); x = mean + std*eps; y = tanh x; a = y*scale + bias
//   logp = sum_i [ -eps_i^2/2 - ls_i - log(2pi)/2 - log(scale_i*(1-y_i^2) + 1e-6) ]
// One row (one action vector of A <= 64 dims) per lane segment of W = next_pow2(A) lanes, so a wave64
// processes 64/W rows and the sum over A is a segmented xor-shuffle; the backward recomputes x, y
// from (mean, raw log_std, eps) instead of storing them.
#include "common.h"

namespace srl {

#define HALF_LOG_2PI 0.91893853320467274f

__device__ __forceinline__ float sq_logstd(float raw, int mode, float lo, float hi, float* dls_draw) {
  if (mode == 0) {
    *dls_draw = (raw >= lo && raw <= hi) ? 1.f : 0.f;
    return fminf(fmaxf(raw, lo), hi);
  }
  float t = tanhf(raw);
  *dls_draw = 0.5f * (hi - lo) * (1.f - t * t);
  return lo + 0.5f * (hi - lo) * (t + 1.f);
}

__global__ void __launch_bounds__(256) squashed_gaussian_fwd_kernel(
    const float* __restrict__ mean, const float* __restrict__ raw, const float* __restrict__ eps,
    const float* __restrict__ scale, const float* __restrict__ bias, float* __restrict__ action,
    float* __restrict__ logp, int R, int A, int W, int mode, float lo, float hi) {
  const int lane = threadIdx.x & 63;
  const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int r = gwave * (64 / W) + lane / W;
  const int k = lane % W;
  const bool valid = r < R && k < A;
  float lp = 0.f;
  if (valid) {
    const int64_t off = (int64_t)r * A + k;
    float d;
    const float ls = sq_logstd(raw[off], mode, lo, hi, &d);
    const float e = eps[off];
    const float x = mean[off] + __expf(ls) * e;
    const float y = tanhf(x);
    const float s = scale[k];
    action[off] = y * s + bias[k];
    lp = -0.5f * e * e - ls - HALF_LOG_2PI - __logf(s * (1.f - y * y) + 1e-6f);
  }
  lp = seg_sum(lp, W);
  if (valid && k == 0) logp[r] = lp;
}

// ga: dL/daction [R,A] or null; glp: dL/dlogp [R] or null
__global__ void __launch_bounds__(256) squashed_gaussian_bwd_kernel(
    const float* __restrict__ mean, const float* __restrict__ raw, const float* __restrict__ eps,
    const float* __restrict__ scale, const float* __restrict__ ga, const float* __restrict__ glp,
    float* __restrict__ dmean, float* __restrict__ draw, int R, int A, int W, int mode, float lo, float hi) {
  const int lane = threadIdx.x & 63;
  const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int r = gwave * (64 / W) + lane / W;
  const int k = lane % W;
  if (r >= R || k >= A) return;
  const int64_t off = (int64_t)r * A + k;
  float d;
  const float ls = sq_logstd(raw[off], mode, lo, hi, &d);
  const float e = eps[off];
  const float std = __expf(ls);
  const float y = tanhf(mean[off] + std * e);
  const float s = scale[k];
  const float one_m_y2 = 1.f - y * y;
  const float gl = glp ? glp[r] : 0.f;
  // d/dy of -log(s(1-y^2)+1e-6) = 2 s y / (s(1-y^2)+1e-6)
  float dy = (ga ? ga[off] * s : 0.f) + gl * (2.f * s * y / (s * one_m_y2 + 1e-6f));
  const float dx = dy * one_m_y2;
  dmean[off] = dx;
  draw[off] = (dx * std * e - gl) * d;
}

}  // namespace srl

using namespace srl;

static inline int seg_width(int A) {
  int W = 1;
  while (W < A) W <<= 1;
  return W;
}

void launch_squashed_gaussian_fwd(const float* mean, const float* raw, const float* eps, const float* scale,
                                  const float* bias, float* action, float* logp, int R, int A, int mode, float lo,
                                  float hi, hipStream_t st) {
  const int W = seg_width(A);
  const int rows_per_block = 4 * (64 / W);
  const int blocks = (R + rows_per_block - 1) / rows_per_block;
  if (blocks == 0) return;
  squashed_gaussian_fwd_kernel<<<blocks, 256, 0, st>>>(mean, raw, eps, scale, bias, action, logp, R, A, W, mode, lo, hi);
}

void launch_squashed_gaussian_bwd(const float* mean, const float* raw, const float* eps, const float* scale,
                                  const float* ga, const float* glp, float* dmean, float* draw, int R, int A, int mode,
                                  float lo, float hi, hipStream_t st) {
  const int W = seg_width(A);
  const int rows_per_block = 4 * (64 / W);
  const int blocks = (R + rows_per_block - 1) / rows_per_block;
  if (blocks == 0) return;
  squashed_gaussian_bwd_kernel<<<blocks, 256, 0, st>>>(mean, raw, eps, scale, ga, glp, dmean, draw, R, A, W, mode, lo,
                                                       hi);
}
