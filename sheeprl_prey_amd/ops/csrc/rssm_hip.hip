#include "hip/hip_runtime.h"
// Small fused kernels of the RSSM posterior scan (see ops/rssm.py):
//   mask_fwd: h' = (1-f) h ; z' = (1-f) z + f z0     (is_first reset, reference dreamer_v3/agent.py:379-384)
//   mask_bwd: dh_prev += (1-f) (dh'_a + dh'_b) ; dz_prev += (1-f) dz'   (accumulating)
// h' is written with a row stride so it lands directly in the [h', feat] GRU input buffer.
#include "common.h"

namespace srl {

__global__ void __launch_bounds__(256) rssm_mask_fwd_kernel(const float* __restrict__ h, int ldh_in,
                                                            const float* __restrict__ z, const float* __restrict__ first,
                                                            const float* __restrict__ z0, float* __restrict__ hout,
                                                            int ldh_out, float* __restrict__ zout, int B, int H, int S) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nh = (int64_t)B * H;
  if (i < nh) {
    int b = i / H, j = i % H;
    float keep = 1.f - first[b];
    hout[(int64_t)b * ldh_out + j] = h ? keep * h[(int64_t)b * ldh_in + j] : 0.f;
  } else if (i < nh + (int64_t)B * S) {
    int64_t k = i - nh;
    int b = k / S, j = k % S;
    float f = first[b];
    float zv = z ? z[k] : 0.f;
    zout[k] = (1.f - f) * zv + f * z0[j];
  }
}

__global__ void __launch_bounds__(256) rssm_mask_bwd_kernel(const float* __restrict__ dha, int ldha,
                                                            const float* __restrict__ dhb, int ldhb,
                                                            const float* __restrict__ dz, const float* __restrict__ first,
                                                            float* __restrict__ dh_acc, float* __restrict__ dz_acc, int B,
                                                            int H, int S) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nh = (int64_t)B * H;
  if (i < nh) {
    int b = i / H, j = i % H;
    dh_acc[i] += (1.f - first[b]) * (dha[(int64_t)b * ldha + j] + dhb[(int64_t)b * ldhb + j]);
  } else if (i < nh + (int64_t)B * S) {
    int64_t k = i - nh;
    int b = k / S;
    dz_acc[k] += (1.f - first[b]) * dz[k];
  }
}

}  // namespace srl

using namespace srl;

void launch_rssm_mask_fwd(const float* h, int ldh_in, const float* z, const float* first, const float* z0, float* hout,
                          int ldh_out, float* zout, int B, int H, int S, hipStream_t st) {
  int64_t n = (int64_t)B * (H + S);
  hipLaunchKernelGGL(rssm_mask_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, h, ldh_in, z, first, z0, hout,
                     ldh_out, zout, B, H, S);
}

void launch_rssm_mask_bwd(const float* dha, int ldha, const float* dhb, int ldhb, const float* dz, const float* first,
                          float* dh_acc, float* dz_acc, int B, int H, int S, hipStream_t st) {
  int64_t n = (int64_t)B * (H + S);
  hipLaunchKernelGGL(rssm_mask_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dha, ldha, dhb, ldhb, dz,
                     first, dh_acc, dz_acc, B, H, S);
}
