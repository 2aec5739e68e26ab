// Fused LayerNorm + activation kernels (fp32).
//  * row-major:  y[r, :] = act(gamma * (x - mu) * rstd + beta)   (nn.Linear -> LayerNorm -> act)
//    - arbitrary input/output row strides (the RSSM scan writes straight into a concat buffer)
//    - "grouped" mode: M = Bn*G input rows ordered (b, g) with per-group gamma/beta, written
//      group-major (g, b) so the next per-group GEMM reads contiguous operands
//  * NCHW:       normalise over C at every pixel directly in NCHW (the reference permutes to
//                NHWC and back around nn.LayerNorm: LayerNormChannelLast, utils/model.py:225-235;
//                here consecutive threads own consecutive pixels, so the C-strided reads coalesce).
// Rows with N <= 2048 are processed one wave per row, 4 waves per block; wider rows use the whole
// 256-thread block per row.  Backward recomputes x_hat from the saved (mu, rstd); dgamma/dbeta are
// reduced as per-block partial rows -> column sums (row-split blocks + one atomic per column and
// split), optionally into per-call "slots" so a time loop can defer the reduction to one kernel.
#include "common.h"

namespace srl {

// ------------------------------------------------------------------ wave-per-row (N <= 64*MAXV)
template <int MAXV>
__global__ void __launch_bounds__(256) ln_wave_fwd_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y,
                                                          int ldy, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out, int M, int N, int G, float eps,
                                                          int act) {
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * 4;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int Bn = M / G;
  const int g = gw % G;
  const float* gam = gamma ? gamma + (int64_t)g * N : nullptr;
  const float* bet = beta ? beta + (int64_t)g * N : nullptr;
  // every load is unconditional (indices clamped into the row, out-of-row lanes masked after the load): a load
  // under a lane branch made the wait-count pass drain vmcnt per element, one memory round trip each
  float gv[MAXV], bv[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int idx = min(lane + 64 * k, N - 1);
    gv[k] = gam ? gam[idx] : 1.f;
    bv[k] = gam ? bet[idx] : 0.f;
  }
  for (int b = gw / G; b < Bn; b += nwaves / G) {
    const int r = b * G + g;
    const float* xr = x + (int64_t)r * ldx;
    float v[MAXV];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) v[k] = xr[min(lane + 64 * k, N - 1)];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      if (lane + 64 * k >= N) v[k] = 0.f;
      s += v[k];
    }
    const float mu = wave_sum_dpp(s) / N;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const float d = lane + 64 * k < N ? v[k] - mu : 0.f;
      q += d * d;
    }
    const float rs = rsqrtf(wave_sum_dpp(q) / N + eps);
    const int ro = (G == 1) ? r : g * Bn + b;
    float* yr = y + (int64_t)ro * ldy;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = lane + 64 * k;
      if (idx < N) yr[idx] = act_fwd((v[k] - mu) * rs * gv[k] + bv[k], act);
    }
    if (lane == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rs;
    }
  }
}

// Same op, 16-byte form for aligned rows (N % 4 == 0, row strides % 4, 16-B aligned pointers, G dividing
// 4): each lane holds NV4 float4 of the row, and gamma/beta are loaded together with x - before the two
// reductions - so the row costs one memory round trip instead of two.  (The imagination rollout runs ~60 of
// these per step at M = 1024, N = 512, where the kernel is latency-bound; the XL scan's two-group prior /
// posterior LayerNorm, 32 x 1024, ran 9.1 us per step on the scalar form.)  Groups as in ln_wave_fwd_kernel:
// wave gw serves group gw % G, input row b G + g, output row g (M / G) + b when G > 1.
template <int NV4>
__global__ void __launch_bounds__(256) ln_wave4_fwd_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y,
                                                           int ldy, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out, int M, int N, float eps, int act,
                                                           int G) {
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * 4;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int g = gw % G, Bn = M / G;
  const int N4 = N >> 2;
  const float4* gam4 = gamma ? reinterpret_cast<const float4*>(gamma + (int64_t)g * N) : nullptr;
  const float4* bet4 = beta ? reinterpret_cast<const float4*>(beta + (int64_t)g * N) : nullptr;
  float4 gv[NV4], bv[NV4];
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    const int i4 = lane + 64 * k;
    gv[k] = (gam4 && i4 < N4) ? gam4[i4] : make_float4(1.f, 1.f, 1.f, 1.f);
    bv[k] = (bet4 && i4 < N4) ? bet4[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int b = gw / G; b < Bn; b += nwaves / G) {
    const int r = b * G + g;
    const int ro = G == 1 ? r : g * Bn + b;
    const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)r * ldx);
    float4 v[NV4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      const int i4 = lane + 64 * k;
      v[k] = i4 < N4 ? xr[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
      s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    const float mu = wave_sum_dpp(s) / N;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      if (lane + 64 * k < N4) {
        const float a = v[k].x - mu, b = v[k].y - mu, c = v[k].z - mu, d = v[k].w - mu;
        q += (a * a + b * b) + (c * c + d * d);
      }
    }
    const float rs = rsqrtf(wave_sum_dpp(q) / N + eps);
    float4* yr = reinterpret_cast<float4*>(y + (int64_t)ro * ldy);
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      const int i4 = lane + 64 * k;
      if (i4 < N4) {
        float4 o;
        o.x = act_fwd((v[k].x - mu) * rs * gv[k].x + bv[k].x, act);
        o.y = act_fwd((v[k].y - mu) * rs * gv[k].y + bv[k].y, act);
        o.z = act_fwd((v[k].z - mu) * rs * gv[k].z + bv[k].z, act);
        o.w = act_fwd((v[k].w - mu) * rs * gv[k].w + bv[k].w, act);
        yr[i4] = o;
      }
    }
    if (lane == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rs;
    }
  }
}

template <int MAXV>
__global__ void __launch_bounds__(256) ln_wave_bwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ dy,
                                                          int lddy, float* __restrict__ dx, int lddx,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          float* __restrict__ pdg, float* __restrict__ pdb, int M, int N,
                                                          int G, int act) {
  __shared__ float red_g[4][64 * MAXV];
  __shared__ float red_b[4][64 * MAXV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  const int gw = blockIdx.x * 4 + w;
  const int Bn = M / G;
  const int g = gw % G;
  const float* gam = gamma ? gamma + (int64_t)g * N : nullptr;
  const float* bet = beta ? beta + (int64_t)g * N : nullptr;
  float ag[MAXV], ab[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) ag[k] = ab[k] = 0.f;
  float gv[MAXV], bv[MAXV];  // this wave's group parameters, loaded once (clamped, unconditional)
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int idx = min(lane + 64 * k, N - 1);
    gv[k] = gam ? gam[idx] : 1.f;
    bv[k] = gam ? bet[idx] : 0.f;
  }
  for (int b = gw / G; b < Bn; b += nwaves / G) {
    const int r = b * G + g;
    const int ro = (G == 1) ? r : g * Bn + b;
    const float* xr = x + (int64_t)r * ldx;
    const float* dyr = dy + (int64_t)ro * lddy;
    const float mu = mean[r], rs = rstd[r];
    // all of the row's loads first, unconditionally (see the forward)
    float xh[MAXV], dxh[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int idx = min(lane + 64 * k, N - 1);
      xh[k] = xr[idx];
      dxh[k] = dyr[idx];
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const bool ok = lane + 64 * k < N;
      const float h = (xh[k] - mu) * rs;
      const float z = gam ? h * gv[k] + bv[k] : h;
      const float dz = ok ? dxh[k] * act_grad(z, act) : 0.f;
      ag[k] += dz * h;
      ab[k] += dz;
      xh[k] = ok ? h : 0.f;
      dxh[k] = dz * gv[k];
      s1 += dxh[k];
      s2 += dxh[k] * xh[k];
    }
    const float m1 = wave_sum_dpp(s1) / N;
    const float m2 = wave_sum_dpp(s2) / N;
    float* dxr = dx + (int64_t)r * lddx;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = lane + 64 * k;
      if (idx < N) dxr[idx] = rs * (dxh[k] - m1 - xh[k] * m2);
    }
  }
  if (pdg) {
    // block partial per group: waves w with (w % G) == g'
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      red_g[w][lane + 64 * k] = ag[k];
      red_b[w][lane + 64 * k] = ab[k];
    }
    __syncthreads();
    for (int gg = 0; gg < G; ++gg) {
      for (int idx = threadIdx.x; idx < N; idx += 256) {
        float a = 0.f, bb = 0.f;
        for (int ww = gg; ww < 4; ww += G) {
          a += red_g[ww][idx];
          bb += red_b[ww][idx];
        }
        pdg[((int64_t)blockIdx.x * G + gg) * N + idx] = a;
        pdb[((int64_t)blockIdx.x * G + gg) * N + idx] = bb;
      }
    }
  }
}

// 16-byte form of the backward for aligned rows (one group, N % 4 == 0, 16-B aligned operands): each lane
// holds NV4 float4 of x / dy, the next row's loads are issued before this row's two reductions (one memory
// round trip per row is exposed per wave only once), the activation derivative is specialized at compile
// time.  At the imagination heads' 16384 x 512 the scalar form ran 53 us (latency-bound: 4 dependent rows
// per wave, 8 scalar loads each).
template <int NV4, int ACTC>
__global__ void __launch_bounds__(256) ln_wave4_bwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ dy,
                                                           int lddy, float* __restrict__ dx, int lddx,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           float* __restrict__ pdg, float* __restrict__ pdb, int M, int N,
                                                           int act, float* __restrict__ za, float* __restrict__ zb, int G) {
  // za / zb (or null): the dgamma / dbeta targets ([G, N]) the column-sum kernel after this one accumulates
  // into atomically - zeroed here by block 0 instead of by a separate zero kernel (one launch less per call)
  if (za != nullptr && blockIdx.x == 0)
    for (int i = threadIdx.x; i < G * N; i += 256) {
      za[i] = 0.f;
      zb[i] = 0.f;
    }
  __shared__ float4 red_g[4][64 * NV4];
  __shared__ float4 red_b[4][64 * NV4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  // groups as in the forward: wave gw serves group gw % G (= w % G: G divides 4), x / dx row b G + g, dy row
  // g (M / G) + b when G > 1; the block's partial row of group g' sums its waves w with w % G == g'
  const int gw = blockIdx.x * 4 + w;
  const int g = gw % G, Bn = M / G, bstep = nwaves / G;
  const int N4 = N >> 2;
  const float inv_n = 1.f / (float)N;
  const float4* gam4 = gamma ? reinterpret_cast<const float4*>(gamma + (int64_t)g * N) : nullptr;
  const float4* bet4 = beta ? reinterpret_cast<const float4*>(beta + (int64_t)g * N) : nullptr;
  float4 gv[NV4], bv[NV4], ag[NV4], ab[NV4];
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    const int i4 = lane + 64 * k;
    gv[k] = (gam4 && i4 < N4) ? gam4[i4] : make_float4(1.f, 1.f, 1.f, 1.f);
    bv[k] = (bet4 && i4 < N4) ? bet4[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
    ag[k] = ab[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int b = gw / G;
  float4 xv[NV4], dv[NV4];
  float mu = 0.f, rs = 0.f;
  auto load = [&](int bb, float4 (&xa)[NV4], float4 (&da)[NV4], float& m_, float& r_) {
    const int row = bb * G + g;
    const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)row * ldx);
    const float4* dr = reinterpret_cast<const float4*>(dy + (int64_t)(G == 1 ? row : g * Bn + bb) * lddy);
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      const int i4 = lane + 64 * k;
      xa[k] = i4 < N4 ? xr[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
      da[k] = i4 < N4 ? dr[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    m_ = mean[row];
    r_ = rstd[row];
  };
  if (b < Bn) load(b, xv, dv, mu, rs);
  while (b < Bn) {
    const int r = b * G + g;
    const int bn = b + bstep;
    float4 xn[NV4], dn[NV4];
    float mun = 0.f, rsn = 0.f;
    if (bn < Bn) load(bn, xn, dn, mun, rsn);
    float4 h[NV4], g[NV4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      float* hp = &h[k].x;
      float* gp = &g[k].x;
      const float* xp = &xv[k].x;
      const float* dp = &dv[k].x;
      const float* ga = &gv[k].x;
      const float* be = &bv[k].x;
      float* agp = &ag[k].x;
      float* abp = &ab[k].x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float hh = (xp[e] - mu) * rs;
        const float dz = dp[e] * act_grad_c<ACTC>(hh * ga[e] + be[e], act);
        agp[e] += dz * hh;
        abp[e] += dz;
        hp[e] = hh;
        gp[e] = dz * ga[e];
        s1 += gp[e];
        s2 += gp[e] * hh;
      }
    }
    const float m1 = wave_sum_dpp(s1) * inv_n;
    const float m2 = wave_sum_dpp(s2) * inv_n;
    float4* dxr = reinterpret_cast<float4*>(dx + (int64_t)r * lddx);
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      const int i4 = lane + 64 * k;
      if (i4 < N4) {
        float4 o;
        o.x = rs * (g[k].x - m1 - h[k].x * m2);
        o.y = rs * (g[k].y - m1 - h[k].y * m2);
        o.z = rs * (g[k].z - m1 - h[k].z * m2);
        o.w = rs * (g[k].w - m1 - h[k].w * m2);
        dxr[i4] = o;
      }
    }
    b = bn;
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      xv[k] = xn[k];
      dv[k] = dn[k];
    }
    mu = mun;
    rs = rsn;
  }
  if (pdg) {
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      red_g[w][lane + 64 * k] = ag[k];
      red_b[w][lane + 64 * k] = ab[k];
    }
    __syncthreads();
    for (int gg = 0; gg < G; ++gg)
      for (int i4 = threadIdx.x; i4 < N4; i4 += 256) {
        float4 a = red_g[gg][i4], c2 = red_b[gg][i4];
        for (int ww = gg + G; ww < 4; ww += G) {
          const float4 c = red_g[ww][i4], d = red_b[ww][i4];
          a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
          c2.x += d.x; c2.y += d.y; c2.z += d.z; c2.w += d.w;
        }
        reinterpret_cast<float4*>(pdg + ((int64_t)blockIdx.x * G + gg) * N)[i4] = a;
        reinterpret_cast<float4*>(pdb + ((int64_t)blockIdx.x * G + gg) * N)[i4] = c2;
      }
  }
}

// ------------------------------------------------------------------ block-per-row (wide rows, G == 1)
template <int MAXV>
__global__ void __launch_bounds__(256) ln_block_fwd_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y,
                                                           int ldy, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out, int M, int N, float eps, int act) {
  __shared__ float red[4];
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + (int64_t)row * ldx;
    float v[MAXV];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * 256;
      v[k] = idx < N ? xr[idx] : 0.f;
      s += v[k];
    }
    const float mu = block_sum<4>(s, red) / N;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * 256;
      float d = idx < N ? v[k] - mu : 0.f;
      q += d * d;
    }
    const float rs = rsqrtf(block_sum<4>(q, red) / N + eps);
    float* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * 256;
      if (idx < N) {
        float z = (v[k] - mu) * rs;
        if (gamma) z = z * gamma[idx] + beta[idx];
        yr[idx] = act_fwd(z, act);
      }
    }
    if (threadIdx.x == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  }
}

template <int MAXV>
__global__ void __launch_bounds__(256) ln_block_bwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ dy,
                                                           int lddy, float* __restrict__ dx, int lddx,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           float* __restrict__ pdg, float* __restrict__ pdb, int M, int N,
                                                           int act) {
  __shared__ float red[4];
  float ag[MAXV], ab[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) ag[k] = ab[k] = 0.f;
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + (int64_t)row * ldx;
    const float* dyr = dy + (int64_t)row * lddy;
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXV], dxh[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * 256;
      xh[k] = dxh[k] = 0.f;
      if (idx < N) {
        float h = (xr[idx] - mu) * rs;
        float gg = gamma ? gamma[idx] : 1.f;
        float z = gamma ? h * gg + beta[idx] : h;
        float dz = dyr[idx] * act_grad(z, act);
        ag[k] += dz * h;
        ab[k] += dz;
        xh[k] = h;
        dxh[k] = dz * gg;
        s1 += dxh[k];
        s2 += dxh[k] * h;
      }
    }
    const float m1 = block_sum<4>(s1, red) / N;
    const float m2 = block_sum<4>(s2, red) / N;
    float* dxr = dx + (int64_t)row * lddx;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * 256;
      if (idx < N) dxr[idx] = rs * (dxh[k] - m1 - xh[k] * m2);
    }
  }
  if (pdg) {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * 256;
      if (idx < N) {
        pdg[(int64_t)blockIdx.x * N + idx] = ag[k];
        pdb[(int64_t)blockIdx.x * N + idx] = ab[k];
      }
    }
  }
}

// out_a[g*N + n] = sum_{p : p % G == g} pa[p, n]  (deterministic; 4 row-slices per 64 columns)
// Column sums of two partial-row arrays: oa[g][n] = sum_{p = g (mod G)} pa[p][n] (same for b).
// Grid (N/64 column blocks, G, S row splits): each block reduces its split with 4 row slices per
// column, then adds into the (pre-zeroed) outputs with one atomic per column - the split keeps the
// reduction parallel when there are few columns and many partial rows (e.g. 1024 x 512).
__global__ void __launch_bounds__(256) colsum2_kernel(const float* __restrict__ pa, const float* __restrict__ pb,
                                                      float* __restrict__ oa, float* __restrict__ ob, int rows, int N,
                                                      int G) {
  __shared__ float sa[4][64], sb[4][64];
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int slice = threadIdx.x >> 6;
  const int g = blockIdx.y, S = gridDim.z, s = blockIdx.z;
  const int Rg = rows > g ? (rows - g + G - 1) / G : 0;  // partial rows of group g
  const int j0 = (int)((int64_t)Rg * s / S), j1 = (int)((int64_t)Rg * (s + 1) / S);
  float a = 0.f, b = 0.f;
  if (n < N) {
    for (int j = j0 + slice; j < j1; j += 4) {
      const int64_t p = (int64_t)g + (int64_t)G * j;
      a += pa[p * N + n];
      b += pb[p * N + n];
    }
  }
  sa[slice][threadIdx.x & 63] = a;
  sb[slice][threadIdx.x & 63] = b;
  __syncthreads();
  if (slice == 0 && n < N) {
    const int c = threadIdx.x & 63;
    atomicAdd(oa + (int64_t)g * N + n, sa[0][c] + sa[1][c] + sa[2][c] + sa[3][c]);
    atomicAdd(ob + (int64_t)g * N + n, sb[0][c] + sb[1][c] + sb[2][c] + sb[3][c]);
  }
}

// Single-array column sum out[n] = sum_r x[r * ldx + n] (bias gradients: dY summed over rows),
// same row-split + atomic layout as colsum2.
__global__ void __launch_bounds__(256) colsum1_kernel(const float* __restrict__ x, int ldx, float* __restrict__ out,
                                                      int rows, int N) {
  __shared__ float sa[4][64];
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int slice = threadIdx.x >> 6;
  const int S = gridDim.z, s = blockIdx.z;
  const int j0 = (int)((int64_t)rows * s / S), j1 = (int)((int64_t)rows * (s + 1) / S);
  float a = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int j = j0 + slice; j < j1; j += 4) a += x[(int64_t)j * ldx + n];
  }
  sa[slice][threadIdx.x & 63] = a;
  __syncthreads();
  if (slice == 0 && n < N) {
    const int c = threadIdx.x & 63;
    atomicAdd(out + n, sa[0][c] + sa[1][c] + sa[2][c] + sa[3][c]);
  }
}

// Ticket-combined form of both column sums (no zero kernel, no float atomics, deterministic): each split block
// stores its 64-column partial write-through (agent-scope relaxed stores = sc1), drains, joins and draws a ticket
// from its column tile's counter; the block drawing S - 1 sums the S partials in split order (each wave a fixed
// quarter of the splits, combined in LDS in wave order) and writes the result, then returns the counter to zero
// (cdna_hip_programming.md section 6 Guideline 16, split-K counter form).  Rows: r(j) = g + G j, row stride ld.
__global__ void __launch_bounds__(256) colsum_t_kernel(const float* __restrict__ pa, const float* __restrict__ pb, int ld,
                                                       float* __restrict__ oa, float* __restrict__ ob, int rows, int N,
                                                       int G, float* __restrict__ ws, int* __restrict__ cnt) {
  __shared__ float sa[4][64], sb[4][64];
  __shared__ int last;
  const int c = threadIdx.x & 63, n = blockIdx.x * 64 + c;
  const int slice = threadIdx.x >> 6;
  const int g = blockIdx.y, S = gridDim.z, s = blockIdx.z;
  const int Rg = rows > g ? (rows - g + G - 1) / G : 0;
  const int j0 = (int)((int64_t)Rg * s / S), j1 = (int)((int64_t)Rg * (s + 1) / S);
  float a = 0.f, b = 0.f;
  if (n < N) {
    // rows summed in row order; 8 rows' loads issued before their adds (one memory latency per 8 rows, not per 2)
    int j = j0 + slice;
    if (pb) {
      for (; j + 7 * 4 < j1; j += 8 * 4) {
        float va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t p = (int64_t)g + (int64_t)G * (j + 4 * u);
          va[u] = pa[p * ld + n];
          vb[u] = pb[p * ld + n];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a += va[u];
          b += vb[u];
        }
      }
    } else {
      for (; j + 7 * 4 < j1; j += 8 * 4) {
        float va[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) va[u] = pa[((int64_t)g + (int64_t)G * (j + 4 * u)) * ld + n];
#pragma unroll
        for (int u = 0; u < 8; ++u) a += va[u];
      }
    }
    for (; j < j1; j += 4) {
      const int64_t p = (int64_t)g + (int64_t)G * j;
      a += pa[p * ld + n];
      if (pb) b += pb[p * ld + n];
    }
  }
  sa[slice][c] = a;
  sb[slice][c] = b;
  __syncthreads();
  const float ta = (sa[0][c] + sa[1][c]) + (sa[2][c] + sa[3][c]);
  const float tb = (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]);
  if (S == 1) {
    if (slice == 0 && n < N) {
      oa[(int64_t)g * N + n] = ta;
      if (ob) ob[(int64_t)g * N + n] = tb;
    }
    return;
  }
  const int64_t plane = (int64_t)S * G * N;  // ws: [2][S][G][N]
  if (slice == 0 && n < N) {
    __hip_atomic_store(ws + ((int64_t)s * G + g) * N + n, ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (pb) __hip_atomic_store(ws + plane + ((int64_t)s * G + g) * N + n, tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains its write-through stores
  __syncthreads();
  int* ctr = cnt + (int64_t)g * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: every read below is sc1
  a = 0.f;
  b = 0.f;
  if (n < N) {  // the S partials summed in order, 8 requested before their adds
    for (int q0 = slice; q0 < S; q0 += 8 * 4) {
      float va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = q0 + 4 * u;
        va[u] = q < S ? __hip_atomic_load(ws + ((int64_t)q * G + g) * N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        vb[u] = (q < S && pb)
                    ? __hip_atomic_load(ws + plane + ((int64_t)q * G + g) * N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (q0 + 4 * u < S) {
          a += va[u];
          b += vb[u];
        }
      }
    }
  }
  __syncthreads();  // every wave has read its ta / tb out of sa / sb
  sa[slice][c] = a;
  sb[slice][c] = b;
  __syncthreads();
  if (slice == 0 && n < N) {
    oa[(int64_t)g * N + n] = (sa[0][c] + sa[1][c]) + (sa[2][c] + sa[3][c]);
    if (ob) ob[(int64_t)g * N + n] = (sb[0][c] + sb[1][c]) + (sb[2][c] + sb[3][c]);
  }
}

// ---------------------------------------------------------------- NCHW (normalise over C)
// One thread per pixel.  C <= MAXC: the pixel's C values stay in registers (1 read + 1 write of the
// tensor); otherwise 3 passes over global memory.
template <int MAXC>
__global__ void __launch_bounds__(256) ln_nchw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int B, int C, int HW, float eps, int act) {
  int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pix >= (int64_t)B * HW) return;
  int b = pix / HW, p = pix % HW;
  const float* xb = x + (int64_t)b * C * HW + p;
  float* yb = y + (int64_t)b * C * HW + p;
  float mu, rs;
  if (MAXC > 0 && C <= MAXC) {
    float v[MAXC > 0 ? MAXC : 1];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      v[c] = c < C ? xb[(int64_t)c * HW] : 0.f;
      s += v[c];
    }
    mu = s / C;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      float d = c < C ? v[c] - mu : 0.f;
      q += d * d;
    }
    rs = rsqrtf(q / C + eps);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        float z = (v[c] - mu) * rs;
        if (gamma) z = z * gamma[c] + beta[c];
        yb[(int64_t)c * HW] = act_fwd(z, act);
      }
    }
  } else {
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += xb[(int64_t)c * HW];
    mu = s / C;
    float q = 0.f;
    for (int c = 0; c < C; ++c) {
      float d = xb[(int64_t)c * HW] - mu;
      q += d * d;
    }
    rs = rsqrtf(q / C + eps);
    for (int c = 0; c < C; ++c) {
      float z = (xb[(int64_t)c * HW] - mu) * rs;
      if (gamma) z = z * gamma[c] + beta[c];
      yb[(int64_t)c * HW] = act_fwd(z, act);
    }
  }
  mean_out[pix] = mu;
  rstd_out[pix] = rs;
}

template <int MAXC>
__global__ void __launch_bounds__(256) ln_nchw_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          float* __restrict__ dx, int B, int C, int HW, int act) {
  int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pix >= (int64_t)B * HW) return;
  int b = pix / HW, p = pix % HW;
  const int64_t base = (int64_t)b * C * HW + p;
  const float mu = mean[pix], rs = rstd[pix];
  float s1 = 0.f, s2 = 0.f;
  if (MAXC > 0 && C <= MAXC) {
    float hv[MAXC > 0 ? MAXC : 1], dv[MAXC > 0 ? MAXC : 1];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      hv[c] = dv[c] = 0.f;
      if (c < C) {
        int64_t o = base + (int64_t)c * HW;
        float h = (x[o] - mu) * rs;
        float g = gamma ? gamma[c] : 1.f;
        float z = gamma ? h * g + beta[c] : h;
        float dxh = dy[o] * act_grad(z, act) * g;
        hv[c] = h;
        dv[c] = dxh;
        s1 += dxh;
        s2 += dxh * h;
      }
    }
    s1 /= C;
    s2 /= C;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c < C) dx[base + (int64_t)c * HW] = rs * (dv[c] - s1 - hv[c] * s2);
    return;
  }
  for (int c = 0; c < C; ++c) {
    int64_t o = base + (int64_t)c * HW;
    float h = (x[o] - mu) * rs;
    float g = gamma ? gamma[c] : 1.f;
    float z = gamma ? h * g + beta[c] : h;
    float dxh = dy[o] * act_grad(z, act) * g;
    s1 += dxh;
    s2 += dxh * h;
  }
  s1 /= C;
  s2 /= C;
  for (int c = 0; c < C; ++c) {
    int64_t o = base + (int64_t)c * HW;
    float h = (x[o] - mu) * rs;
    float g = gamma ? gamma[c] : 1.f;
    float z = gamma ? h * g + beta[c] : h;
    float dxh = dy[o] * act_grad(z, act) * g;
    dx[o] = rs * (dxh - s1 - h * s2);
  }
}

// grid (C, S): partial sums of dz*x_hat and dz for channel c over a 1/S slice of the pixels
__global__ void __launch_bounds__(256) ln_nchw_dgb_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          float* __restrict__ pdg, float* __restrict__ pdb, int B, int C,
                                                          int HW, int act) {
  __shared__ float red[4];
  const int c = blockIdx.x, S = gridDim.y, sidx = blockIdx.y;
  const int64_t P = (int64_t)B * HW;
  const float g = gamma[c], bt = beta[c];
  float a = 0.f, bsum = 0.f;
  for (int64_t pix = sidx * (int64_t)blockDim.x + threadIdx.x; pix < P; pix += (int64_t)S * blockDim.x) {
    int b = pix / HW, p = pix % HW;
    int64_t o = ((int64_t)b * C + c) * HW + p;
    float h = (x[o] - mean[pix]) * rstd[pix];
    float dz = dy[o] * act_grad(h * g + bt, act);
    a += dz * h;
    bsum += dz;
  }
  a = block_sum<4>(a, red);
  bsum = block_sum<4>(bsum, red);
  if (threadIdx.x == 0) {
    pdg[(int64_t)sidx * C + c] = a;
    pdb[(int64_t)sidx * C + c] = bsum;
  }
}

}  // namespace srl

using namespace srl;

// ---------------------------------------------------------------- launch configuration (shared with bindings)
// mode 0: wave-per-row with MAXV = 64*k; mode 1: block-per-row.  Returns false if unsupported.
static bool ln_mode(int N, int G, int& mode, int& maxv) {
  if (N <= 256) { mode = 0; maxv = 4; }
  else if (N <= 512) { mode = 0; maxv = 8; }
  else if (N <= 1024) { mode = 0; maxv = 16; }
  else if (N <= 2048) { mode = 0; maxv = 32; }
  else if (G != 1) return false;
  else if (N <= 4096) { mode = 1; maxv = 16; }
  else if (N <= 12288) { mode = 1; maxv = 48; }
  else return false;
  return true;
}

// Number of blocks (== partial rows per group) the backward uses for M rows.
int ln_bwd_grid(int M, int N, int G) {
  int mode, maxv;
  if (!ln_mode(N, G, mode, maxv)) return 0;
  if (mode == 0) {
    int waves = M;                      // one wave per row
    int g = cdiv(waves, 4);
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    if (G > 1 && (g * 4) % G) g += 1;   // nwaves must be a multiple of G
    return g;
  }
  return M < 512 ? M : 512;
}

// grouped (G = 2 / 4) rows on the 16-byte wave kernels (profiles/r4_ln_grouped.md)
static constexpr bool g_ln_vec_groups = true;

bool launch_ln_act_fwd(const float* x, int ldx, float* y, int ldy, const float* gamma, const float* beta, float* mean,
                       float* rstd, int M, int N, int G, float eps, int act, hipStream_t st) {
  int mode, maxv;
  if (!ln_mode(N, G, mode, maxv)) return false;
  if (mode == 0) {
    int grid = cdiv(M, 4);
    if (grid > 4096) grid = 4096;
    const bool al16 = ((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) % 16 == 0;
    if ((G == 1 || (g_ln_vec_groups && (G == 2 || G == 4) && M % G == 0)) && N % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 &&
        al16 && (gamma != nullptr) == (beta != nullptr)) {
#define F4(NV) if (maxv == 4 * NV) { hipLaunchKernelGGL(ln_wave4_fwd_kernel<NV>, dim3(grid), dim3(256), 0, st, x, ldx, y, ldy, gamma, beta, mean, rstd, M, N, eps, act, G); return true; }
      F4(1) F4(2) F4(4) F4(8)
#undef F4
    }
    if (G > 1 && (grid * 4) % G) grid += 1;
#define F(MV) if (maxv == MV) { hipLaunchKernelGGL(ln_wave_fwd_kernel<MV>, dim3(grid), dim3(256), 0, st, x, ldx, y, ldy, gamma, beta, mean, rstd, M, N, G, eps, act); return true; }
    F(4) F(8) F(16) F(32)
#undef F
  } else {
    int grid = M < 8192 ? M : 8192;
#define F(MV) if (maxv == MV) { hipLaunchKernelGGL(ln_block_fwd_kernel<MV>, dim3(grid), dim3(256), 0, st, x, ldx, y, ldy, gamma, beta, mean, rstd, M, N, eps, act); return true; }
    F(16) F(48)
#undef F
  }
  return false;
}

// Zero the atomic-accumulation targets with a kernel, not hipMemsetAsync: under hipGraph stream
// capture the memset did not reliably precede the atomics (stale sums showed up as garbage bias
// gradients, up to 1.5e38, in replayed DreamerV3 steps; eager runs were clean).
__global__ void __launch_bounds__(256) zero2_kernel(float* __restrict__ a, float* __restrict__ b, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    a[i] = 0.f;
    if (b) b[i] = 0.f;
  }
}

static void launch_zero2(float* a, float* b, int n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(zero2_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, a, b, n);
}

// Workspace + ticket counters of colsum_t_kernel (set once per process by ops.init_reduce_workspace on the device
// it trains on; until then - or on another device - the zero kernel + atomic form runs).  Launches take rotating
// slices so launches close together never share one, and the pool is split in two halves by stream: launches on
// the registered side stream (ops/sidestream.py: parameter gradients beside the scan backward) rotate through the
// second half, so a side launch can never share a slice with a main-stream launch running at the same time, however
// often either cursor wraps.
static float* g_cs_ws = nullptr;
static int* g_cs_cnt = nullptr;
static int64_t g_cs_ws_n = 0, g_cs_cnt_n = 0, g_cs_ws_cur[2] = {0, 0}, g_cs_cnt_cur[2] = {0, 0};
static int g_cs_dev = -1;
static hipStream_t g_cs_side = nullptr;

void set_colsum_workspace(float* ws, int64_t ws_n, int* cnt, int64_t cnt_n) {
  // the cursors survive a re-init with the same buffers (captured graphs keep their slices; a reset would hand
  // a live slice out again)
  if (ws != g_cs_ws || cnt != g_cs_cnt) g_cs_ws_cur[0] = g_cs_ws_cur[1] = g_cs_cnt_cur[0] = g_cs_cnt_cur[1] = 0;
  g_cs_ws = ws;
  g_cs_ws_n = ws_n;
  g_cs_cnt = cnt;
  g_cs_cnt_n = cnt_n;
  g_cs_dev = -1;
  if (ws != nullptr) (void)hipGetDevice(&g_cs_dev);
}

void set_colsum_side_stream(hipStream_t st) { g_cs_side = st; }

static int colsum_S2(int rows, int G) {
  const int Rg = cdiv(rows, G > 0 ? G : 1);
  int S = cdiv(Rg, 64);
  if (S > 32) S = 32;
  if (S < 1) S = 1;
  return S;
}

// slice sizes of one ticket launch; false when the workspace is absent / on another device / too small
static bool colsum_ticket_fits(int N, int G, int S, int64_t& need, int64_t& nc) {
  if (g_cs_ws == nullptr) return false;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != g_cs_dev) return false;
  const int nx = cdiv(N, 64);
  need = S > 1 ? 2LL * S * G * N : 0;
  nc = S > 1 ? (int64_t)G * nx : 0;
  return need <= g_cs_ws_n / 2 && nc <= g_cs_cnt_n / 2;
}

// true: launched the ticket form (out written directly, no zeroing needed)
static bool colsum_ticket(const float* pa, const float* pb, int ld, float* oa, float* ob, int rows, int N, int G, int S,
                          hipStream_t st) {
  int64_t need, nc;
  if (!colsum_ticket_fits(N, G, S, need, nc)) return false;
  const int h = (g_cs_side != nullptr && st == g_cs_side) ? 1 : 0;
  const int64_t wsh = g_cs_ws_n / 2, cnh = g_cs_cnt_n / 2;
  if (g_cs_ws_cur[h] + need > wsh) g_cs_ws_cur[h] = 0;
  if (g_cs_cnt_cur[h] + nc > cnh) g_cs_cnt_cur[h] = 0;
  float* ws = g_cs_ws + h * wsh + g_cs_ws_cur[h];
  int* cnt = g_cs_cnt + h * cnh + g_cs_cnt_cur[h];
  g_cs_ws_cur[h] += (need + 63) / 64 * 64;
  g_cs_cnt_cur[h] += (nc + 63) / 64 * 64;
  hipLaunchKernelGGL(colsum_t_kernel, dim3(cdiv(N, 64), G, S), dim3(256), 0, st, pa, pb, ld, oa, ob, rows, N, G, ws, cnt);
  return true;
}

void launch_colsum1(const float* x, int ldx, float* out, int rows, int N, hipStream_t st) {
  int S = cdiv(rows, 128);
  if (S > 64) S = 64;
  if (S < 1) S = 1;
  if (colsum_ticket(x, nullptr, ldx, out, nullptr, rows, N, 1, S, st)) return;
  launch_zero2(out, nullptr, N, st);
  hipLaunchKernelGGL(colsum1_kernel, dim3(cdiv(N, 64), 1, S), dim3(256), 0, st, x, ldx, out, rows, N);
}

// the reduction alone: oa / ob already zeroed (by the producing kernel)
static void launch_colsum2_nz(const float* pa, const float* pb, float* oa, float* ob, int rows, int N, int G, hipStream_t st) {
  const int Rg = cdiv(rows, G > 0 ? G : 1);
  int S = cdiv(Rg, 64);
  if (S > 32) S = 32;
  if (S < 1) S = 1;
  hipLaunchKernelGGL(colsum2_kernel, dim3(cdiv(N, 64), G, S), dim3(256), 0, st, pa, pb, oa, ob, rows, N, G);
}

void launch_colsum2(const float* pa, const float* pb, float* oa, float* ob, int rows, int N, int G, hipStream_t st) {
  // ticket form (one launch, deterministic), else zero kernel + one atomic reduction kernel (graph-capturable); ~64
  // partial rows per split
  const int S = colsum_S2(rows, G);
  if (colsum_ticket(pa, pb, N, oa, ob, rows, N, G, S, st)) return;
  launch_zero2(oa, ob, G * N, st);
  hipLaunchKernelGGL(colsum2_kernel, dim3(cdiv(N, 64), G, S), dim3(256), 0, st, pa, pb, oa, ob, rows, N, G);
}

// pdg/pdb: [grid*G, N] partial rows (required if gamma != null).  If dgamma != null the partials
// are reduced into dgamma/dbeta [G, N] right away; otherwise the caller reduces them later.
bool launch_ln_act_bwd(const float* x, int ldx, const float* dy, int lddy, float* dx, int lddx, const float* gamma,
                       const float* beta, const float* mean, const float* rstd, float* pdg, float* pdb, float* dgamma,
                       float* dbeta, int M, int N, int G, int act, hipStream_t st) {
  int mode, maxv;
  if (!ln_mode(N, G, mode, maxv)) return false;
  const int grid = ln_bwd_grid(M, N, G);
  float* pg = gamma ? pdg : nullptr;
  float* pb = gamma ? pdb : nullptr;
  if (mode == 0) {
    const bool al16 = ((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)gamma | (uintptr_t)beta) % 16 == 0;
    if ((G == 1 || (g_ln_vec_groups && (G == 2 || G == 4) && M % G == 0)) && N % 4 == 0 && ldx % 4 == 0 &&
        lddy % 4 == 0 && lddx % 4 == 0 && al16 && (gamma != nullptr) == (beta != nullptr) && maxv <= 16) {
      // the deterministic one-launch ticket reduction when its workspace is set (no zeroing needed); else the LN
      // kernel zeroes dgamma / dbeta itself and the atomic reduction follows
      int64_t tneed, tnc;
      const bool tk = gamma && dgamma && colsum_ticket_fits(N, G, colsum_S2(grid * G, G), tneed, tnc);
      float* za = (gamma && dgamma && !tk) ? dgamma : nullptr;
      float* zb = (gamma && dgamma && !tk) ? dbeta : nullptr;
#define F4(NV) if (maxv == 4 * NV) { SRL_ACT_SPECIALIZE(act, hipLaunchKernelGGL((ln_wave4_bwd_kernel<NV, ACTC>), dim3(grid), dim3(256), 0, st, x, ldx, dy, lddy, dx, lddx, gamma, beta, mean, rstd, pg, pb, M, N, act, za, zb, G)); if (tk) goto reduce; goto reduce_zeroed; }
      F4(1) F4(2) F4(4)
#undef F4
    }
#define F(MV) if (maxv == MV) { hipLaunchKernelGGL(ln_wave_bwd_kernel<MV>, dim3(grid), dim3(256), 0, st, x, ldx, dy, lddy, dx, lddx, gamma, beta, mean, rstd, pg, pb, M, N, G, act); goto reduce; }
    F(4) F(8) F(16) F(32)
#undef F
    return false;
  } else {
#define F(MV) if (maxv == MV) { hipLaunchKernelGGL(ln_block_bwd_kernel<MV>, dim3(grid), dim3(256), 0, st, x, ldx, dy, lddy, dx, lddx, gamma, beta, mean, rstd, pg, pb, M, N, act); goto reduce; }
    F(16) F(48)
#undef F
    return false;
  }
reduce:
  if (gamma && dgamma) launch_colsum2(pdg, pdb, dgamma, dbeta, grid * G, N, G, st);
  return true;
reduce_zeroed:  // the LN kernel zeroed dgamma / dbeta itself
  if (gamma && dgamma) launch_colsum2_nz(pdg, pdb, dgamma, dbeta, grid * G, N, G, st);
  return true;
}

void launch_ln_nchw_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int B,
                        int C, int HW, float eps, int act, hipStream_t st) {
  int64_t P = (int64_t)B * HW;
  dim3 g((unsigned)((P + 255) / 256)), b(256);
  if (C <= 32) hipLaunchKernelGGL(ln_nchw_fwd_kernel<32>, g, b, 0, st, x, gamma, beta, y, mean, rstd, B, C, HW, eps, act);
  else if (C <= 64) hipLaunchKernelGGL(ln_nchw_fwd_kernel<64>, g, b, 0, st, x, gamma, beta, y, mean, rstd, B, C, HW, eps, act);
  else hipLaunchKernelGGL(ln_nchw_fwd_kernel<0>, g, b, 0, st, x, gamma, beta, y, mean, rstd, B, C, HW, eps, act);
}

int ln_nchw_splits(int B, int HW) {
  int64_t P = (int64_t)B * HW;
  int64_t s = (P + 4095) / 4096;
  if (s > 64) s = 64;
  return (int)(s < 1 ? 1 : s);
}

void launch_ln_nchw_bwd(const float* x, const float* dy, const float* gamma, const float* beta, const float* mean,
                        const float* rstd, float* dx, float* pdg, float* pdb, float* dgamma, float* dbeta, int B, int C,
                        int HW, int act, hipStream_t st) {
  int64_t P = (int64_t)B * HW;
  dim3 gg((unsigned)((P + 255) / 256)), bb(256);
  if (C <= 32) hipLaunchKernelGGL(ln_nchw_bwd_kernel<32>, gg, bb, 0, st, x, dy, gamma, beta, mean, rstd, dx, B, C, HW, act);
  else hipLaunchKernelGGL(ln_nchw_bwd_kernel<0>, gg, bb, 0, st, x, dy, gamma, beta, mean, rstd, dx, B, C, HW, act);
  if (gamma) {
    int S = ln_nchw_splits(B, HW);
    hipLaunchKernelGGL(ln_nchw_dgb_kernel, dim3(C, S), dim3(256), 0, st, x, dy, gamma, beta, mean, rstd, pdg, pdb, B, C, HW,
                       act);
    launch_colsum2(pdg, pdb, dgamma, dbeta, S, C, 1, st);
  }
}
