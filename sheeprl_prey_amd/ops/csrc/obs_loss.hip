// DreamerV3 observation reconstruction loss (reference dreamer_v3/dreamer_v3.py:186-196 and the
// symlog MSE of utils/distribution.py SymlogDistribution):
//
//   image keys:  loss[r] = sum_i (rec[r,i] - u8[r,i] * scale)^2            (target straight from the
//                uint8 replay bytes: no float copy of the frames is materialised for the loss)
//   vector keys: d = (rec - symlog(x))^2,  d = 0 where d < 1e-8;  loss[r] = sum_i d
//
// fwd: one workgroup per row (t, b), float4 streams, fixed-order block reduction.
// bwd: drec = 2 (rec - target) * g[r]  (zeroed where the vector form zeroed d).
#include "common.h"

namespace srl {
namespace obsloss {

constexpr int NTH = 256;

template <bool U8>
__device__ __forceinline__ float4 target4(const void* t, size_t i4, float scale, bool symlog) {
  float4 v;
  if (U8) {
    const uchar4 b = reinterpret_cast<const uchar4*>(t)[i4];
    v = make_float4(b.x * scale, b.y * scale, b.z * scale, b.w * scale);
  } else {
    v = reinterpret_cast<const float4*>(t)[i4];
  }
  if (symlog) {
    v.x = copysignf(log1pf(fabsf(v.x)), v.x);
    v.y = copysignf(log1pf(fabsf(v.y)), v.y);
    v.z = copysignf(log1pf(fabsf(v.z)), v.z);
    v.w = copysignf(log1pf(fabsf(v.w)), v.w);
  }
  return v;
}

__device__ __forceinline__ float sq(float d, bool thr) {
  const float s = d * d;
  return (thr && s < 1e-8f) ? 0.f : s;
}

template <bool U8>
__global__ __launch_bounds__(NTH) void obs_mse_fwd_kernel(const float* __restrict__ rec, const void* __restrict__ tgt, int n4,
                                                          float scale, int symlog, float* __restrict__ loss) {
  __shared__ float red[NTH / 64];
  const size_t base = (size_t)blockIdx.x * n4;
  const bool sl = symlog != 0;
  float acc = 0.f;
  for (int i = threadIdx.x; i < n4; i += NTH) {
    const float4 r = reinterpret_cast<const float4*>(rec)[base + i];
    const float4 t = target4<U8>(tgt, base + i, scale, sl);
    acc += sq(r.x - t.x, sl) + sq(r.y - t.y, sl) + sq(r.z - t.z, sl) + sq(r.w - t.w, sl);
  }
  acc = block_sum<NTH / 64>(acc, red);
  if (threadIdx.x == 0) loss[blockIdx.x] = acc;
}

template <bool U8>
__global__ __launch_bounds__(NTH) void obs_mse_bwd_kernel(const float* __restrict__ rec, const void* __restrict__ tgt, int n4,
                                                          float scale, int symlog, const float* __restrict__ g,
                                                          float* __restrict__ drec) {
  const size_t base = (size_t)blockIdx.x * n4;
  const bool sl = symlog != 0;
  const float gr = 2.f * g[blockIdx.x];
  for (int i = threadIdx.x; i < n4; i += NTH) {
    const float4 r = reinterpret_cast<const float4*>(rec)[base + i];
    const float4 t = target4<U8>(tgt, base + i, scale, sl);
    float4 d = make_float4(r.x - t.x, r.y - t.y, r.z - t.z, r.w - t.w);
    if (sl) {
      d.x = d.x * d.x < 1e-8f ? 0.f : d.x;
      d.y = d.y * d.y < 1e-8f ? 0.f : d.y;
      d.z = d.z * d.z < 1e-8f ? 0.f : d.z;
      d.w = d.w * d.w < 1e-8f ? 0.f : d.w;
    }
    reinterpret_cast<float4*>(drec)[base + i] = make_float4(gr * d.x, gr * d.y, gr * d.z, gr * d.w);
  }
}

}  // namespace obsloss
}  // namespace srl

// Vector-observation encoder input (reference dreamer_v3/agent.py MLPEncoder: cat of symlog(obs[k]) over the keys):
// the symlog of up to 8 row-major [rows, d_j] inputs written side by side into out [rows, sum d_j] in one pass
// (torch: sign, abs, log1p, mul per key + the concatenation copy).
struct SymlogCat {
  const float* src[8];
  int d[8];
  int off[9];
  int n;
};
__global__ __launch_bounds__(256) void symlog_cat_kernel(SymlogCat s, float* __restrict__ out, int rows, int W) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * W) return;
  const int r = (int)(i / W), c = (int)(i - (long)r * W);
  int j = 0;
  while (j + 1 < s.n && c >= s.off[j + 1]) ++j;
  const float v = s.src[j][(long)r * s.d[j] + (c - s.off[j])];
  out[i] = copysignf(log1pf(fabsf(v)), v);
}

bool launch_symlog_cat(const float* const* src, const int* d, int n, float* out, int rows, hipStream_t st) {
  if (n < 1 || n > 8 || rows < 1) return false;
  SymlogCat s{};
  s.n = n;
  int W = 0;
  for (int j = 0; j < n; ++j) {
    s.src[j] = src[j];
    s.d[j] = d[j];
    s.off[j] = W;
    W += d[j];
  }
  s.off[n] = W;
  const long tot = (long)rows * W;
  hipLaunchKernelGGL(symlog_cat_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, s, out, rows, W);
  return true;
}

void launch_obs_mse_fwd(const float* rec, const void* tgt, bool u8, int rows, int n, float scale, int symlog, float* loss,
                        hipStream_t st) {
  if (u8)
    hipLaunchKernelGGL(srl::obsloss::obs_mse_fwd_kernel<true>, dim3(rows), dim3(srl::obsloss::NTH), 0, st, rec, tgt, n / 4, scale,
                       symlog, loss);
  else
    hipLaunchKernelGGL(srl::obsloss::obs_mse_fwd_kernel<false>, dim3(rows), dim3(srl::obsloss::NTH), 0, st, rec, tgt, n / 4,
                       scale, symlog, loss);
}

void launch_obs_mse_bwd(const float* rec, const void* tgt, bool u8, int rows, int n, float scale, int symlog, const float* g,
                        float* drec, hipStream_t st) {
  if (u8)
    hipLaunchKernelGGL(srl::obsloss::obs_mse_bwd_kernel<true>, dim3(rows), dim3(srl::obsloss::NTH), 0, st, rec, tgt, n / 4, scale,
                       symlog, g, drec);
  else
    hipLaunchKernelGGL(srl::obsloss::obs_mse_bwd_kernel<false>, dim3(rows), dim3(srl::obsloss::NTH), 0, st, rec, tgt, n / 4,
                       scale, symlog, g, drec);
}
