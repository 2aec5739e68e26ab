// Device helpers shared by the RSSM scan kernels (rssm_scan.hip: 4+4 launches per step;
// rssm_persist.hip: one persistent launch per direction).  16-row A operands in LDS, weights as
// register tiles of float4 fragments, v_mfma_f32_16x16x4_f32 with K split over the 16 waves.
#pragma once
#include "common.h"

namespace srl {
namespace scandev {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int NTH = 1024;  // threads per workgroup
constexpr int NWV = 16;    // waves per workgroup (== rows of the A tile)

#define FEPS 1.1920928955078125e-07f

__device__ __forceinline__ void chunk(int total, int& lo, int& hi) {
  const int per = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  lo = (int)blockIdx.x * per;
  hi = min(total, lo + per);
  if (lo > hi) lo = hi;
}

// LDS carving shared by all kernels: A [16][K+4] | (kernel extras) | red [16 waves][16][16*NT] | ct [16][16*NT]

// ---------------------------------------------------------------------------------- fast math
// v_exp + v_rcp forms (a few ulp): the prologues are VALU-bound, every workgroup recomputes its tile.
__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 2.f * fsig(2.f * x) - 1.f; }
__device__ __forceinline__ float f_act(float z, int act) {
  switch (act) {
    case ACT_SILU: return z * fsig(z);
    case ACT_ELU: return z > 0.f ? z : __expf(z) - 1.f;
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_TANH: return ftanh(z);
    default: return z;
  }
}
__device__ __forceinline__ float f_act_grad(float z, int act) {
  switch (act) {
    case ACT_SILU: {
      const float sg = fsig(z);
      return sg * (1.f + z * (1.f - sg));
    }
    case ACT_ELU: return z > 0.f ? 1.f : __expf(z);
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_TANH: {
      const float th = ftanh(z);
      return 1.f - th * th;
    }
    default: return 1.f;
  }
}
// compile-time activation forms (common.h SRL_ACT_SPECIALIZE)
template <int ACTC>
__device__ __forceinline__ float f_act_c(float z, int act) {
  if constexpr (ACTC == ACT_SILU) return z * fsig(z);
  else return f_act(z, act);
}
template <int ACTC>
__device__ __forceinline__ float f_act_grad_c(float z, int act) {
  if constexpr (ACTC == ACT_SILU) {
    const float sg = fsig(z);
    return sg * (1.f + z * (1.f - sg));
  } else {
    return f_act_grad(z, act);
  }
}

// ---------------------------------------------------------------------------------- GEMM core
// Weight fragments of one batch of k chunks, loaded at kernel entry so their latency hides behind
// the prologue.  Wave w owns the 16-wide k chunks w, w+16, ...  Default cache policy: the tile a
// workgroup reads is the same every step, so it stays in its XCD's L2 across the scan.
template <int NT, int U>
struct WTile {
  f4 b[U][NT];
};

template <int NT, int U>
__device__ __forceinline__ void wload(WTile<NT, U>& wt, const float* __restrict__ W, int ldw, int K, int c0) {
  const int lane = threadIdx.x & 63;
  const float* wrow = W + (size_t)(lane & 15) * ldw + 4 * (lane >> 4);
  const int nch = K >> 4;
#pragma unroll
  for (int q = 0; q < U; ++q) {
    const int c = c0 + NWV * q;
    if (c < nch) {
#pragma unroll
      for (int t = 0; t < NT; ++t) wt.b[q][t] = *(const f4*)(wrow + (size_t)16 * t * ldw + (c << 4));
    }
  }
}

// C[16][16*NT] (LDS `ct`) = A[16][K] (LDS, row stride lda) x W[16*NT rows][K]^T; `wt` holds the
// first batch (wload(..., c0 = wave)); later batches are streamed here.
template <int NT, int U>
__device__ __forceinline__ void gemm16(WTile<NT, U>& wt, const float* As, int lda, const float* __restrict__ W, int ldw,
                                       int K, float* red, float* ct) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const int nch = K >> 4;
  const float* arow = As + i * lda + 4 * g;
  for (int c0 = w; c0 < nch; c0 += NWV * U) {
    if (c0 != w) wload<NT, U>(wt, W, ldw, K, c0);
    f4 a[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int c = c0 + NWV * q;
      if (c < nch) a[q] = *(const f4*)(arow + (c << 4));
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int c = c0 + NWV * q;
      if (c < nch) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][0], wt.b[q][t][0], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][1], wt.b[q][t][1], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][2], wt.b[q][t][2], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][3], wt.b[q][t][3], acc[t], 0, 0, 0);
        }
      }
    }
  }
  // C/D map: col = lane & 15, row = 4 * (lane >> 4) + reg
  constexpr int NC = 16 * NT;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(w * 16 + 4 * g + r) * NC + 16 * t + i] = acc[t][r];
  __syncthreads();
  if (threadIdx.x < 16 * NC) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) v += red[ww * 16 * NC + threadIdx.x];
    ct[threadIdx.x] = v;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------- staging
// Copy a 16 x cols tile (cols % 4 == 0) from global (row stride ls) into LDS (row stride ld);
// rows >= nvalid are zero.  Each thread issues U float4 loads before its first LDS store.
__device__ __forceinline__ void stage(float* dst, int ld, const float* __restrict__ src, size_t ls, int nvalid, int cols) {
  const int c4 = cols >> 2, n = 16 * c4;
  constexpr int U = 4;
  for (int base = 0; base < n; base += NTH * U) {
    f4 r[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int idx = base + q * NTH + threadIdx.x;
      const int i = idx / c4, k = (idx - i * c4) << 2;
      r[q] = (idx < n && i < nvalid) ? *(const f4*)(src + (size_t)i * ls + k) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int idx = base + q * NTH + threadIdx.x;
      const int i = idx / c4, k = (idx - i * c4) << 2;
      if (idx < n) *(f4*)(dst + i * ld + k) = r[q];
    }
  }
}

// Copy n floats (n % 4 == 0) of a parameter vector into LDS.
__device__ __forceinline__ void stage_vec(float* dst, const float* __restrict__ src, int n) {
  for (int k = threadIdx.x * 4; k < n; k += 4 * NTH) *(f4*)(dst + k) = *(const f4*)(src + k);
}

// Row mean / rstd of r[0:N) by the calling wave.
__device__ __forceinline__ void wave_row_stats(const float* r, int N, float eps, float& mu, float& rs) {
  const int s = threadIdx.x & 63;
  float a = 0.f;
  for (int k = s; k < N; k += 64) a += r[k];
  mu = wave_sum(a) / N;
  float q = 0.f;
  for (int k = s; k < N; k += 64) {
    const float d = r[k] - mu;
    q += d * d;
  }
  rs = rsqrtf(wave_sum(q) / N + eps);
}

// LayerNorm + activation of one row r[0:N) (N <= 64 * M) by the calling wave, the row held in
// registers: one LDS read per element, both statistics from registers, one write.
template <int M, int ACTC>
__device__ __forceinline__ void wave_ln_act_row_t(float* r, int N, float eps, const float* gam, const float* bet, int act,
                                                  float& mu, float& rs) {
  const int s = threadIdx.x & 63;
  float v[M];
  float a = 0.f;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int k = s + 64 * m;
    v[m] = k < N ? r[k] : 0.f;
    a += v[m];
  }
  mu = wave_sum_dpp(a) / N;
  float q = 0.f;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int k = s + 64 * m;
    const float d = k < N ? v[m] - mu : 0.f;
    q += d * d;
  }
  rs = rsqrtf(wave_sum_dpp(q) / N + eps);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int k = s + 64 * m;
    if (k < N) r[k] = f_act_c<ACTC>((v[m] - mu) * rs * gam[k] + bet[k], act);
  }
}
template <int M>
__device__ __forceinline__ void wave_ln_act_row(float* r, int N, float eps, const float* gam, const float* bet, int act,
                                                float& mu, float& rs) {
  SRL_ACT_SPECIALIZE(act, wave_ln_act_row_t<M, ACTC>(r, N, eps, gam, bet, act, mu, rs));
}

// LayerNorm(+act) adjoint of one row, first pass, with the row in registers (N <= 64 * M): loads x
// and dy once, leaves xh / dz in registers AND in place (x <- xh, dy <- dz, for ln_param_partials);
// returns s1 = mean(dz*gamma), s2 = mean(dz*gamma*xh).  Finish with wave_ln_bwd_finish.
template <int M, int ACTC>
__device__ __forceinline__ void wave_ln_bwd_regs_t(float* x, float* dy, const float* gam, const float* bet, int N, int act,
                                                   float mu, float rs, float (&xh)[M], float (&dz)[M], float& s1, float& s2) {
  const int s = threadIdx.x & 63;
  float xv[M], dv[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int k = s + 64 * m;
    xv[m] = k < N ? x[k] : 0.f;
    dv[m] = k < N ? dy[k] : 0.f;
  }
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int k = s + 64 * m;
    if (k < N) {
      xh[m] = (xv[m] - mu) * rs;
      dz[m] = dv[m] * f_act_grad_c<ACTC>(xh[m] * gam[k] + bet[k], act);
      const float dxh = dz[m] * gam[k];
      a += dxh;
      b += dxh * xh[m];
      x[k] = xh[m];
      dy[k] = dz[m];
    } else {
      xh[m] = 0.f;
      dz[m] = 0.f;
    }
  }
  s1 = wave_sum_dpp(a) / N;
  s2 = wave_sum_dpp(b) / N;
}
template <int M>
__device__ __forceinline__ void wave_ln_bwd_regs(float* x, float* dy, const float* gam, const float* bet, int N, int act,
                                                 float mu, float rs, float (&xh)[M], float (&dz)[M], float& s1, float& s2) {
  SRL_ACT_SPECIALIZE(act, wave_ln_bwd_regs_t<M, ACTC>(x, dy, gam, bet, N, act, mu, rs, xh, dz, s1, s2));
}

template <int M>
__device__ __forceinline__ void wave_ln_bwd_finish(float* x, const float* gam, int N, float rs, float s1, float s2,
                                                   const float (&xh)[M], const float (&dz)[M]) {
  const int s = threadIdx.x & 63;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int k = s + 64 * m;
    if (k < N) x[k] = rs * (dz[m] * gam[k] - s1 - xh[m] * s2);
  }
}

// LayerNorm(+act) adjoint, first pass, by the wave owning a row: x <- xh, dy <- dz = dy * act'(z);
// returns (mean(dz*gamma), mean(dz*gamma*xh)).
template <int ACTC>
__device__ __forceinline__ void wave_ln_bwd_prep_t(float* x, float* dy, const float* gam, const float* bet, int N, int act,
                                                   float mu, float rs, float& s1, float& s2) {
  const int s = threadIdx.x & 63;
  float a = 0.f, b = 0.f;
  for (int k = s; k < N; k += 64) {
    const float xh = (x[k] - mu) * rs;
    const float dz = dy[k] * f_act_grad_c<ACTC>(xh * gam[k] + bet[k], act);
    x[k] = xh;
    dy[k] = dz;
    const float dxh = dz * gam[k];
    a += dxh;
    b += dxh * xh;
  }
  s1 = wave_sum(a) / N;
  s2 = wave_sum(b) / N;
}
__device__ __forceinline__ void wave_ln_bwd_prep(float* x, float* dy, const float* gam, const float* bet, int N, int act,
                                                 float mu, float rs, float& s1, float& s2) {
  SRL_ACT_SPECIALIZE(act, wave_ln_bwd_prep_t<ACTC>(x, dy, gam, bet, N, act, mu, rs, s1, s2));
}

// Column sums over the B rows of dz*xh and dz (after wave_ln_bwd_prep) for columns [lo, hi):
// 8 lanes per column (rows r8, r8+8), NTH/8 columns per pass.
__device__ __forceinline__ void ln_param_partials(const float* xh, int ldx, const float* dz, int lddz, int B, int lo, int hi,
                                                  float* pg, float* pb) {
  const int r8 = threadIdx.x & 7;
  for (int base = lo; base < hi; base += NTH / 8) {  // uniform trip count: the shuffles stay converged
    const int col = base + (threadIdx.x >> 3);
    float ag = 0.f, ab = 0.f;
    if (col < hi) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = r8 + 8 * h;
        if (i < B) {
          const float d = dz[i * lddz + col];
          ag += d * xh[i * ldx + col];
          ab += d;
        }
      }
    }
    ag = seg_sum(ag, 8);
    ab = seg_sum(ab, 8);
    if (r8 == 0 && col < hi) {
      pg[col] = ag;
      pb[col] = ab;
    }
  }
}

}  // namespace scandev
}  // namespace srl
