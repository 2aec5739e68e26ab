// Truncated normal N(loc, scale) restricted to [lo, hi]: inverse-CDF reparameterised sample and
// log-density, forward and backward, one elementwise launch each (reference semantics:
// sheeprl/utils/distribution.py:25-147 — Z = max(Phi(beta) - Phi(alpha), eps) with eps the float32
// machine epsilon, the icdf argument Phi(alpha) + u Z is not clamped).
//
// With alpha = (lo - loc) / scale, beta = (hi - loc) / scale, xi = Phi(alpha) + u Z, s = Phi^-1(xi):
//   sample  x = loc + scale s
//   dx/dloc   = 1 - (dxi/dalpha + dxi/dbeta) / phi(s)
//   dx/dscale = s - (alpha dxi/dalpha + beta dxi/dbeta) / phi(s)
//   dxi/dalpha = (1-u) phi(alpha), dxi/dbeta = u phi(beta)   (Z clamped: phi(alpha), 0)
//   log p(v) = -log(sqrt(2 pi)) - log Z - z^2 / 2 - log scale,  z = (v - loc) / scale
//   dlogZ/dloc = (phi(alpha) - phi(beta)) / (Z scale), dlogZ/dscale = (alpha phi(alpha) - beta phi(beta)) / (Z scale)
// Bounds are either one value per element or one scalar (n_lo / n_hi == 1); parameters broadcast over
// leading sample dimensions (element i uses parameter i % np).
#include "common.h"

namespace srl {
namespace tn {

constexpr float INV_SQRT_2PI = 0.3989422804014327f;
constexpr float INV_SQRT_2 = 0.7071067811865476f;
constexpr float SQRT_2 = 1.4142135623730951f;
constexpr float LOG_INV_SQRT_2PI = -0.9189385332046727f;
constexpr float EPS = 1.1920928955078125e-07f;

__device__ __forceinline__ float pdf(float x) { return isfinite(x) ? INV_SQRT_2PI * __expf(-0.5f * x * x) : 0.f; }
__device__ __forceinline__ float cdf(float x) { return 0.5f * (1.f + erff(x * INV_SQRT_2)); }

struct Trunc {
  float alpha, beta, pa, pb, Z;
  bool clamped;
};

__device__ __forceinline__ Trunc bounds(float loc, float scale, float lo, float hi) {
  Trunc t;
  t.alpha = (lo - loc) / scale;
  t.beta = (hi - loc) / scale;
  t.pa = pdf(t.alpha);
  t.pb = pdf(t.beta);
  const float z = cdf(t.beta) - cdf(t.alpha);
  t.clamped = !(z > EPS);
  t.Z = t.clamped ? EPS : z;
  return t;
}

__global__ void rsample_fwd(const float* __restrict__ loc, const float* __restrict__ scale, const float* __restrict__ lo,
                            int nlo, const float* __restrict__ hi, int nhi, const float* __restrict__ u, float* __restrict__ x,
                            int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float l = loc[i], s = scale[i];
    const Trunc t = bounds(l, s, lo[nlo == 1 ? 0 : i], hi[nhi == 1 ? 0 : i]);
    const float xi = cdf(t.alpha) + u[i] * t.Z;
    x[i] = l + s * (SQRT_2 * erfinvf(2.f * xi - 1.f));
  }
}

__global__ void rsample_bwd(const float* __restrict__ loc, const float* __restrict__ scale, const float* __restrict__ lo,
                            int nlo, const float* __restrict__ hi, int nhi, const float* __restrict__ u,
                            const float* __restrict__ gx, float* __restrict__ gloc, float* __restrict__ gscale, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float l = loc[i], sc = scale[i], ui = u[i], g = gx[i];
    const Trunc t = bounds(l, sc, lo[nlo == 1 ? 0 : i], hi[nhi == 1 ? 0 : i]);
    const float xi = cdf(t.alpha) + ui * t.Z;
    const float s = SQRT_2 * erfinvf(2.f * xi - 1.f);
    const float da = t.clamped ? t.pa : (1.f - ui) * t.pa;
    const float db = t.clamped ? 0.f : ui * t.pb;
    const float inv = 1.f / (INV_SQRT_2PI * __expf(-0.5f * s * s));
    const float wa = isfinite(t.alpha) ? t.alpha * da : 0.f, wb = isfinite(t.beta) ? t.beta * db : 0.f;
    gloc[i] = g * (1.f - (da + db) * inv);
    gscale[i] = g * (s - (wa + wb) * inv);
  }
}

__global__ void logprob_fwd(const float* __restrict__ v, const float* __restrict__ loc, const float* __restrict__ scale,
                            const float* __restrict__ lo, int nlo, const float* __restrict__ hi, int nhi, float* __restrict__ lp,
                            int n, int np) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int k = i % np;
    const float l = loc[k], s = scale[k];
    const Trunc t = bounds(l, s, lo[nlo == 1 ? 0 : k], hi[nhi == 1 ? 0 : k]);
    const float z = (v[i] - l) / s;
    lp[i] = LOG_INV_SQRT_2PI - __logf(t.Z) - 0.5f * z * z - __logf(s);
  }
}

// Per-element parameter gradients (summed over sample dimensions by the caller).
__global__ void logprob_bwd(const float* __restrict__ v, const float* __restrict__ loc, const float* __restrict__ scale,
                            const float* __restrict__ lo, int nlo, const float* __restrict__ hi, int nhi,
                            const float* __restrict__ g, float* __restrict__ gv, float* __restrict__ gloc,
                            float* __restrict__ gscale, int n, int np) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int k = i % np;
    const float l = loc[k], s = scale[k], gi = g[i];
    const Trunc t = bounds(l, s, lo[nlo == 1 ? 0 : k], hi[nhi == 1 ? 0 : k]);
    const float z = (v[i] - l) / s;
    float dzl = 0.f, dzs = 0.f;  // dlogZ / dloc, dlogZ / dscale
    if (!t.clamped) {
      const float wa = isfinite(t.alpha) ? t.alpha * t.pa : 0.f, wb = isfinite(t.beta) ? t.beta * t.pb : 0.f;
      dzl = (t.pa - t.pb) / (t.Z * s);
      dzs = (wa - wb) / (t.Z * s);
    }
    gv[i] = -gi * z / s;
    gloc[i] = gi * (z / s - dzl);
    gscale[i] = gi * ((z * z - 1.f) / s - dzs);
  }
}

// DreamerV3 continuous actor head + sample in one pass (reference agent.py:685-700, trunc_normal):
//   loc = tanh(pre[:, a]),  scale = 2 sigmoid((pre[:, A + a] + init_std) / 2) + min_std,  x ~ TN(loc, scale, lo, hi)
// pre [M, 2A] with row stride ldp, u [M, A]; loc / scale [M, A] kept for the backward, x row-strided (ldx).
__global__ void head_sample_fwd(const float* __restrict__ pre, int ldp, const float* __restrict__ u, float init_std,
                                float min_std, float lo, float hi, float* __restrict__ loc_out, float* __restrict__ scale_out,
                                float* __restrict__ x, int ldx, int M, int A) {
  const int n = M * A;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / A, a = i - r * A;
    const float l = tanhf(pre[(int64_t)r * ldp + a]);
    const float sg = 1.f / (1.f + __expf(-0.5f * (pre[(int64_t)r * ldp + A + a] + init_std)));
    const float s = 2.f * sg + min_std;
    const Trunc t = bounds(l, s, lo, hi);
    const float xi = cdf(t.alpha) + u[i] * t.Z;
    loc_out[i] = l;
    scale_out[i] = s;
    x[(int64_t)r * ldx + a] = l + s * (SQRT_2 * erfinvf(2.f * xi - 1.f));
  }
}

// The head Linear folded in: pre = y W^T + b (y [M, K] row-strided, W [2A, K], 2A <= 64, K = 64 KM) computed per
// row by one wave (K products per lane, one DPP wave reduction per head column, W staged per 4-row workgroup in
// LDS under the row loads), written out for the backward, then sampled as head_sample_fwd.  At the continuous imagination shape
// (M = 1024, K = 512, 2A = 12) the library ran this N = 12 GEMM as a 32 x 32-tile kernel at ~26 us per step.
template <int KM>
__global__ void __launch_bounds__(256) head_linear_sample_fwd(const float* __restrict__ y, int ldy, const float* __restrict__ W,
                                                             const float* __restrict__ b, const float* __restrict__ u,
                                                             float init_std, float min_std, float lo, float hi,
                                                             float* __restrict__ pre, float* __restrict__ loc_out,
                                                             float* __restrict__ scale_out, float* __restrict__ x, int ldx,
                                                             int M, int A, const float* __restrict__ lng,
                                                             const float* __restrict__ lnb, float lneps, int act,
                                                             float* __restrict__ yo, int ldyo, float* __restrict__ mean_out,
                                                             float* __restrict__ rstd_out) {
  extern __shared__ float ws[];  // [2A][64 KM]
  const int K = 64 * KM, NA = 2 * A;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wave;  // one row per wave: M / 4 workgroups
  float v[KM], gv[KM], bv[KM];
#pragma unroll
  for (int m = 0; m < KM; ++m) v[m] = r < M ? y[(int64_t)r * ldy + lane + 64 * m] : 0.f;  // in flight under the staging
  // everything read after a reduction is requested now: the LN parameters, this lane's head bias, its uniform
#pragma unroll
  for (int m = 0; m < KM; ++m) {
    gv[m] = lng != nullptr ? lng[lane + 64 * m] : 0.f;
    bv[m] = lng != nullptr ? lnb[lane + 64 * m] : 0.f;
  }
  const float bl = (b != nullptr && lane < NA) ? b[lane] : 0.f;
  const float ul = (r < M && lane < A) ? u[r * A + lane] : 0.f;
  {  // head weights -> LDS, 8 loads in flight per thread before their stores
    const int n = NA * K;
    for (int base = 0; base < n; base += 8 * 256) {
      float t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = base + q * 256 + threadIdx.x;
        t[q] = i < n ? W[i] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = base + q * 256 + threadIdx.x;
        if (i < n) ws[i] = t[q];
      }
    }
  }
  if (lng != nullptr && r < M) {
    // y holds the trunk's last pre-activation: its LayerNorm + activation first (the row is in registers), the
    // normalised row and its statistics written out for the trunk backward
    float a = 0.f;
#pragma unroll
    for (int m = 0; m < KM; ++m) a += v[m];
    const float mu = wave_sum_dpp(a) / K;
    float q = 0.f;
#pragma unroll
    for (int m = 0; m < KM; ++m) q += (v[m] - mu) * (v[m] - mu);
    const float rs = rsqrtf(wave_sum_dpp(q) / K + lneps);
#pragma unroll
    for (int m = 0; m < KM; ++m) {
      const int k = lane + 64 * m;
      v[m] = act_fwd((v[m] - mu) * rs * gv[m] + bv[m], act);
      yo[(int64_t)r * ldyo + k] = v[m];
    }
    if (lane == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rs;
    }
  }
  __syncthreads();
  if (r < M) {
    float mine = 0.f;  // lane j keeps head column j
#pragma unroll 4
    for (int j = 0; j < NA; ++j) {
      float s = 0.f;
#pragma unroll
      for (int m = 0; m < KM; ++m) s += v[m] * ws[j * K + lane + 64 * m];
      s = wave_sum_dpp(s);
      if (lane == j) mine = s + (b ? bl : 0.f);  // lane j: + b[j]
    }
    if (lane < NA) pre[(int64_t)r * NA + lane] = mine;
    const float ps = __shfl(mine, lane + A, 64);  // the log-std column of action `lane`
    if (lane < A) {
      const int i = r * A + lane;
      const float l = tanhf(mine);
      const float sg = 1.f / (1.f + __expf(-0.5f * (ps + init_std)));
      const float sc = 2.f * sg + min_std;
      const Trunc t = bounds(l, sc, lo, hi);
      const float xi = cdf(t.alpha) + ul * t.Z;
      loc_out[i] = l;
      scale_out[i] = sc;
      x[(int64_t)r * ldx + lane] = l + sc * (SQRT_2 * erfinvf(2.f * xi - 1.f));
    }
  }
}

// d pre [M, 2A] = (d loc * (1 - loc^2) | d scale * sg (1 - sg)) (+ dpre_in), with (d loc, d scale) the
// rsample backward of gx (gx may be null: only dpre_in), sg = (scale - min_std) / 2.
__global__ void head_sample_bwd(const float* __restrict__ loc, const float* __restrict__ scale, const float* __restrict__ u,
                                const float* __restrict__ gx, const float* __restrict__ dpre_in, float min_std, float lo,
                                float hi, float* __restrict__ dpre, int M, int A) {
  const int n = M * A;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = i / A, a = i - r * A;
    const float l = loc[i], sc = scale[i];
    float gl = 0.f, gs = 0.f;
    if (gx != nullptr) {
      const float ui = u[i], g = gx[i];
      const Trunc t = bounds(l, sc, lo, hi);
      const float xi = cdf(t.alpha) + ui * t.Z;
      const float s = SQRT_2 * erfinvf(2.f * xi - 1.f);
      const float da = t.clamped ? t.pa : (1.f - ui) * t.pa;
      const float db = t.clamped ? 0.f : ui * t.pb;
      const float inv = 1.f / (INV_SQRT_2PI * __expf(-0.5f * s * s));
      const float wa = isfinite(t.alpha) ? t.alpha * da : 0.f, wb = isfinite(t.beta) ? t.beta * db : 0.f;
      gl = g * (1.f - (da + db) * inv);
      gs = g * (s - (wa + wb) * inv);
    }
    const float sg = 0.5f * (sc - min_std);
    const int64_t o = (int64_t)r * 2 * A + a;
    float dm = gl * (1.f - l * l), ds = gs * sg * (1.f - sg);
    if (dpre_in != nullptr) {
      dm += dpre_in[o];
      ds += dpre_in[o + A];
    }
    dpre[o] = dm;
    dpre[o + A] = ds;
  }
}

inline int grid_for(int n) { return std::max(1, std::min((n + 255) / 256, 2048)); }

}  // namespace tn
}  // namespace srl

using namespace srl::tn;

void launch_truncnorm_rsample_fwd(const float* loc, const float* scale, const float* lo, int nlo, const float* hi, int nhi,
                                  const float* u, float* x, int n, hipStream_t st) {
  hipLaunchKernelGGL(rsample_fwd, dim3(grid_for(n)), dim3(256), 0, st, loc, scale, lo, nlo, hi, nhi, u, x, n);
}

void launch_truncnorm_rsample_bwd(const float* loc, const float* scale, const float* lo, int nlo, const float* hi, int nhi,
                                  const float* u, const float* gx, float* gloc, float* gscale, int n, hipStream_t st) {
  hipLaunchKernelGGL(rsample_bwd, dim3(grid_for(n)), dim3(256), 0, st, loc, scale, lo, nlo, hi, nhi, u, gx, gloc, gscale, n);
}

void launch_truncnorm_logprob_fwd(const float* v, const float* loc, const float* scale, const float* lo, int nlo,
                                  const float* hi, int nhi, float* lp, int n, int np, hipStream_t st) {
  hipLaunchKernelGGL(logprob_fwd, dim3(grid_for(n)), dim3(256), 0, st, v, loc, scale, lo, nlo, hi, nhi, lp, n, np);
}

void launch_truncnorm_logprob_bwd(const float* v, const float* loc, const float* scale, const float* lo, int nlo,
                                  const float* hi, int nhi, const float* g, float* gv, float* gloc, float* gscale, int n, int np,
                                  hipStream_t st) {
  hipLaunchKernelGGL(logprob_bwd, dim3(grid_for(n)), dim3(256), 0, st, v, loc, scale, lo, nlo, hi, nhi, g, gv, gloc, gscale, n,
                     np);
}

void launch_tn_head_sample_fwd(const float* pre, int ldp, const float* u, float init_std, float min_std, float lo, float hi,
                               float* loc, float* scale, float* x, int ldx, int M, int A, hipStream_t st) {
  if (M * A > 0)
    hipLaunchKernelGGL(head_sample_fwd, dim3(grid_for(M * A)), dim3(256), 0, st, pre, ldp, u, init_std, min_std, lo, hi, loc,
                       scale, x, ldx, M, A);
}

bool launch_tn_head_linear_sample_fwd(const float* y, int ldy, const float* W, const float* b, const float* u, float init_std,
                                      float min_std, float lo, float hi, float* pre, float* loc, float* scale, float* x, int ldx,
                                      int M, int K, int A, hipStream_t st, const float* lng, const float* lnb, float lneps,
                                      int act, float* yo, int ldyo, float* mean_out, float* rstd_out) {
  if (lng != nullptr && (lnb == nullptr || yo == nullptr || mean_out == nullptr || rstd_out == nullptr)) return false;
  if (M <= 0 || A < 1 || 2 * A > 64 || K % 64 != 0 || K > 1024 || (size_t)2 * A * K * 4 > 64 * 1024) return false;
  const dim3 grid((M + 3) / 4);
  const size_t shm = (size_t)2 * A * K * sizeof(float);
  switch (K / 64) {
#define HL(KM) \
  case KM: hipLaunchKernelGGL(head_linear_sample_fwd<KM>, grid, dim3(256), shm, st, y, ldy, W, b, u, init_std, min_std, lo, hi, pre, loc, scale, x, ldx, M, A, lng, lnb, lneps, act, yo, ldyo, mean_out, rstd_out); return true;
    HL(1) HL(2) HL(4) HL(8) HL(16)
#undef HL
    default: return false;
  }
}

void launch_tn_head_sample_bwd(const float* loc, const float* scale, const float* u, const float* gx, const float* dpre_in,
                               float min_std, float lo, float hi, float* dpre, int M, int A, hipStream_t st) {
  if (M * A > 0)
    hipLaunchKernelGGL(head_sample_bwd, dim3(grid_for(M * A)), dim3(256), 0, st, loc, scale, u, gx, dpre_in, min_std, lo, hi,
                       dpre, M, A);
}
