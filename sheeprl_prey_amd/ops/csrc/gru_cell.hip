// Plain GRU cell activations (torch.nn.GRU semantics; DreamerV1 / P2E-DV1 recurrent model, reference
// dreamer_v1/agent.py:45-59):
//   r = sigmoid(gi_r + gh_r),  z = sigmoid(gi_z + gh_z),  n = tanh(gi_n + r * gh_n),  h' = (1 - z) n + z h
// with gi = x W_ih^T + b_ih and gh = h W_hh^T + b_hh computed by library GEMMs (autograd owns them).
// fwd: one pass writing h' and the (r, z, n) needed by the backward; bwd: one pass producing
// d gi, d gh and the direct d h term.  One thread per (row, unit), float loads of the three gate
// slices.
#include "common.h"

namespace srl {
namespace grucell {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(256) void gru_cell_fwd_kernel(const float* __restrict__ gi, const float* __restrict__ gh,
                                                           const float* __restrict__ h, float* __restrict__ hn,
                                                           float* __restrict__ rzn, int B, int H) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * H) return;
  const int b = i / H, u = i - b * H;
  const float* a = gi + (size_t)b * 3 * H;
  const float* c = gh + (size_t)b * 3 * H;
  const float r = sigm(a[u] + c[u]);
  const float z = sigm(a[H + u] + c[H + u]);
  const float n = tanhf(a[2 * H + u] + r * c[2 * H + u]);
  hn[i] = (1.f - z) * n + z * h[i];
  float* s = rzn + (size_t)b * 3 * H;
  s[u] = r;
  s[H + u] = z;
  s[2 * H + u] = n;
}

__global__ __launch_bounds__(256) void gru_cell_bwd_kernel(const float* __restrict__ gh, const float* __restrict__ h,
                                                           const float* __restrict__ rzn, const float* __restrict__ dhn,
                                                           float* __restrict__ dgi, float* __restrict__ dgh,
                                                           float* __restrict__ dh, int B, int H) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * H) return;
  const int b = i / H, u = i - b * H;
  const size_t o = (size_t)b * 3 * H;
  const float r = rzn[o + u], z = rzn[o + H + u], n = rzn[o + 2 * H + u];
  const float g = dhn[i];
  const float dn = g * (1.f - z);
  const float dz = g * (h[i] - n);
  dh[i] = g * z;
  const float dpn = dn * (1.f - n * n);
  const float dr = dpn * gh[o + 2 * H + u];
  const float dpr = dr * r * (1.f - r);
  const float dpz = dz * z * (1.f - z);
  dgi[o + u] = dpr;
  dgi[o + H + u] = dpz;
  dgi[o + 2 * H + u] = dpn;
  dgh[o + u] = dpr;
  dgh[o + H + u] = dpz;
  dgh[o + 2 * H + u] = dpn * r;
}

}  // namespace grucell
}  // namespace srl

void launch_gru_cell_fwd(const float* gi, const float* gh, const float* h, float* hn, float* rzn, int B, int H, hipStream_t st) {
  hipLaunchKernelGGL(srl::grucell::gru_cell_fwd_kernel, dim3((B * H + 255) / 256), dim3(256), 0, st, gi, gh, h, hn, rzn, B, H);
}

void launch_gru_cell_bwd(const float* gh, const float* h, const float* rzn, const float* dhn, float* dgi, float* dgh, float* dh,
                         int B, int H, hipStream_t st) {
  hipLaunchKernelGGL(srl::grucell::gru_cell_bwd_kernel, dim3((B * H + 255) / 256), dim3(256), 0, st, gh, h, rzn, dhn, dgi, dgh,
                     dh, B, H);
}
