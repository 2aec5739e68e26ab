// Flat-slab optimiser kernels: global grad-norm (+clip factor, device-side), fused Adam/AdamW.
// All buffers are fp32, 16-byte aligned, numel % 4 == 0 (FlatOptimizer guarantees it).
// scalars = [step, clip_coef, last_norm, skip] lives on the device so the whole update is
// hipGraph-capturable (no host sync, no per-step kernel-argument changes).
// guard (optional) = the device's fault block [scan health, gather error, skipped updates, -]: when a
// kernel earlier in the step recorded a fault (a timed-out persistent-scan hand-off, an out-of-range
// replay index) the norm/advance kernel sets skip = 1, leaves the step count alone and counts the
// skipped update; Adam then leaves the parameters and moments untouched.
#include "common.h"

namespace srl {

__global__ void __launch_bounds__(256) sqnorm_partial_kernel(const float4* __restrict__ g, int64_t n4,
                                                             float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = g[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = block_sum<4>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__device__ inline bool guard_tripped(int* guard) {
  if (guard == nullptr) return false;
  if ((guard[0] | guard[1]) == 0) return false;
  atomicAdd(guard + 2, 1);
  return true;
}

__global__ void __launch_bounds__(256) sqnorm_finalize_kernel(const float* __restrict__ partial, int np,
                                                              float* __restrict__ scalars, float* __restrict__ out_norm,
                                                              float max_norm, int* guard) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partial[i];
  acc = block_sum<4>(acc, red);
  if (threadIdx.x == 0) {
    float norm = sqrtf(acc);
    float coef = 1.f;
    if (max_norm > 0.f && max_norm < 3.0e38f) {
      coef = max_norm / (norm + 1e-6f);
      coef = (coef > 1.f) ? 1.f : coef;  // NaN propagates like torch's clamp
    }
    out_norm[0] = norm;
    if (guard_tripped(guard)) {
      scalars[3] = 1.f;
    } else {
      scalars[0] += 1.f;
      scalars[1] = coef;
      scalars[2] = norm;
      scalars[3] = 0.f;
    }
  }
}

__global__ void advance_kernel(float* scalars, int* guard) {
  if (guard_tripped(guard)) {
    scalars[3] = 1.f;
    return;
  }
  scalars[0] += 1.f;
  scalars[1] = 1.f;
  scalars[3] = 0.f;
}

__global__ void __launch_bounds__(256) adam_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v,
                                                   const float* __restrict__ scalars, int64_t n4, float lr, float b1,
                                                   float b2, float eps, float wd, int decoupled) {
  if (scalars[3] != 0.f) return;  // a fault earlier in this step: no update
  const float t = scalars[0];
  const float coef = scalars[1];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float step = lr / bc1;
  const float decay = decoupled ? (1.f - lr * wd) : 1.f;
  const float l2 = decoupled ? 0.f : wd;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
    float* pf = reinterpret_cast<float*>(&pp);
    float* gf = reinterpret_cast<float*>(&gg);
    float* mf = reinterpret_cast<float*>(&mm);
    float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gr = gf[k] * coef + l2 * pf[k];
      float w = pf[k] * decay;
      float mk = mf[k] + (1.f - b1) * (gr - mf[k]);
      float vk = vf[k] * b2 + (1.f - b2) * gr * gr;
      float denom = sqrtf(vk) / bc2s + eps;
      pf[k] = w - step * mk / denom;
      mf[k] = mk;
      vf[k] = vk;
    }
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

}  // namespace srl

using namespace srl;

static int grid_for(int64_t n4) {
  int64_t b = (n4 + 255) / 256;
  if (b > 2048) b = 2048;  // 256 CUs x 8 blocks, grid-stride the rest
  return (int)(b < 1 ? 1 : b);
}

void launch_flat_grad_norm(const float* g, int64_t n, float* partial, int np, float* scalars, float* out_norm,
                           float max_norm, int* guard, hipStream_t st) {
  int64_t n4 = n / 4;
  int grid = grid_for(n4);
  if (grid > np) grid = np;
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(grid), dim3(256), 0, st, (const float4*)g, n4, partial);
  hipLaunchKernelGGL(sqnorm_finalize_kernel, dim3(1), dim3(256), 0, st, partial, grid, scalars, out_norm, max_norm,
                     guard);
}

void launch_flat_advance(float* scalars, int* guard, hipStream_t st) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, st, scalars, guard);
}

void launch_flat_adam(float* p, const float* g, float* m, float* v, const float* scalars, int64_t n, float lr, float b1,
                      float b2, float eps, float wd, int decoupled, hipStream_t st) {
  int64_t n4 = n / 4;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n4)), dim3(256), 0, st, (float4*)p, (const float4*)g, (float4*)m,
                     (float4*)v, scalars, n4, lr, b1, b2, eps, wd, decoupled);
}
