// DreamerV3 world-model loss assembly (reference dreamer_v3/loss.py:11-110 and dreamer_v3.py:179-196):
//
//   c[r]   = scale * BCEWithLogits(l[r], 1 - done[r])          continue loss per (t, b)
//   total  = mean_r (kl_reg * kl_loss[r] + obs[r] + rew[r] + c[r])
//   means  = (mean kl, mean kl_loss, mean rew, mean obs, mean c)   (logged metrics)
//
// The per-row terms come from the fused KL / two-hot / observation kernels; what is left - the
// continue BCE, the weighted sum, the mean and five metric means - was ~10 small ATen launches
// forward and ~12 backward.  Here it is one single-workgroup launch each way: the forward reduces
// the six sums in a fixed order (deterministic), the backward writes the four per-row gradients.
#include "common.h"

namespace srl {
namespace wmloss {

constexpr int NTH = 1024;

__device__ __forceinline__ float bce_logits(float l, float y) {
  // max(l, 0) - l y + log(1 + exp(-|l|)): torch's stable form
  return fmaxf(l, 0.f) - l * y + log1pf(__expf(-fabsf(l)));
}

__global__ __launch_bounds__(NTH) void fwd_kernel(const float* __restrict__ kl_loss, const float* __restrict__ obs,
                                                  const float* __restrict__ rew, const float* __restrict__ logit,
                                                  const float* __restrict__ done, const float* __restrict__ kl, int R,
                                                  float kl_reg, float scale, float* __restrict__ total,
                                                  float* __restrict__ means) {
  __shared__ float red[NTH / 64];
  float s_tot = 0.f, s_kl = 0.f, s_kll = 0.f, s_rew = 0.f, s_obs = 0.f, s_c = 0.f;
  for (int r = threadIdx.x; r < R; r += NTH) {
    const float c = logit ? scale * bce_logits(logit[r], 1.f - done[r]) : 0.f;
    const float kll = kl_loss[r], o = obs[r], w = rew[r];
    s_tot += kl_reg * kll + o + w + c;
    s_kl += kl[r];
    s_kll += kll;
    s_rew += w;
    s_obs += o;
    s_c += c;
  }
  const float inv = 1.f / (float)R;
  const float v0 = block_sum<NTH / 64>(s_tot, red), v1 = block_sum<NTH / 64>(s_kl, red);
  const float v2 = block_sum<NTH / 64>(s_kll, red), v3 = block_sum<NTH / 64>(s_rew, red);
  const float v4 = block_sum<NTH / 64>(s_obs, red), v5 = block_sum<NTH / 64>(s_c, red);
  if (threadIdx.x == 0) {
    total[0] = v0 * inv;
    means[0] = v1 * inv;
    means[1] = v2 * inv;
    means[2] = v3 * inv;
    means[3] = v4 * inv;
    means[4] = v5 * inv;
  }
}

// d total / d (kl_loss, obs, rew, logit); g: the upstream gradient of total (device scalar)
__global__ __launch_bounds__(256) void bwd_kernel(const float* __restrict__ logit, const float* __restrict__ done,
                                                  const float* __restrict__ g, int R, float kl_reg, float scale,
                                                  float* __restrict__ d_kll, float* __restrict__ d_obs,
                                                  float* __restrict__ d_rew, float* __restrict__ d_logit) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const float gr = g[0] / (float)R;
  d_kll[r] = gr * kl_reg;
  d_obs[r] = gr;
  d_rew[r] = gr;
  if (d_logit) {
    const float l = logit[r];
    d_logit[r] = gr * scale * (1.f / (1.f + __expf(-l)) - (1.f - done[r]));
  }
}

}  // namespace wmloss
}  // namespace srl

void launch_wm_loss_fwd(const float* kl_loss, const float* obs, const float* rew, const float* logit, const float* done,
                        const float* kl, int R, float kl_reg, float scale, float* total, float* means, hipStream_t st) {
  hipLaunchKernelGGL(srl::wmloss::fwd_kernel, dim3(1), dim3(srl::wmloss::NTH), 0, st, kl_loss, obs, rew, logit, done, kl, R,
                     kl_reg, scale, total, means);
}

void launch_wm_loss_bwd(const float* logit, const float* done, const float* g, int R, float kl_reg, float scale, float* d_kll,
                        float* d_obs, float* d_rew, float* d_logit, hipStream_t st) {
  hipLaunchKernelGGL(srl::wmloss::bwd_kernel, dim3((R + 255) / 256), dim3(256), 0, st, logit, done, g, R, kl_reg, scale,
                     d_kll, d_obs, d_rew, d_logit);
}
