// LayerNorm-GRU cell epilogue (reference: LayerNormGRUCell, sheeprl/models/models.py:362-402):
//   x = [h, in] @ W            (GEMM, done by the caller)
//   z = LN(x) * gamma + beta   over 3H
//   r = sig(z_r); c = tanh(r * z_c); u = sig(z_u - 1); h' = u * c + (1 - u) * h
// One block per row; thread t owns hidden units t, t+T, ... and reads their r/c/u columns,
// so every load is coalesced.  Backward recomputes z from (x, mean, rstd).
#include "common.h"

#include <cstdint>
#include <cstdlib>

namespace srl {

template <int MAXH>
// xsum (may alias x): the summed input x + x2 written back (the split-GEMM caller whose backward reads the whole gx)
__global__ void __launch_bounds__(256) ln_gru_fwd_kernel(const float* x, const float* __restrict__ h, int ldh,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float* __restrict__ hn, float* __restrict__ mean_out,
                                                         float* __restrict__ rstd_out, int M, int H, float eps,
                                                         int ldo, const float* __restrict__ x2, int ldx2, float* xsum) {
  __shared__ float red[4];
  const int T = 256, N = 3 * H;
  // LayerNorm parameters (and, per row, h) requested before the row loads: used after the two block reductions,
  // they no longer add a memory latency there
  float gm[3][MAXH], bt[3][MAXH];
#pragma unroll
  for (int k = 0; k < MAXH; ++k) {
    const int j = threadIdx.x + k * T;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      gm[g][k] = j < H ? gamma[g * H + j] : 0.f;
      bt[g][k] = j < H ? beta[g * H + j] : 0.f;
    }
  }
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + (int64_t)row * N;
    const float* x2r = x2 ? x2 + (int64_t)row * ldx2 : nullptr;  // optional second GEMM part (row-strided)
    float hp[MAXH];
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      const int j = threadIdx.x + k * T;
      hp[k] = j < H ? h[(int64_t)row * ldh + j] : 0.f;
    }
    float v[3][MAXH];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      int j = threadIdx.x + k * T;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        v[g][k] = j < H ? xr[g * H + j] + (x2r ? x2r[g * H + j] : 0.f) : 0.f;
        s += v[g][k];
        if (xsum && j < H) xsum[(int64_t)row * N + g * H + j] = v[g][k];  // same element this thread just read
      }
    }
    const float mu = block_sum<4>(s, red) / N;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      int j = threadIdx.x + k * T;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        float d = j < H ? v[g][k] - mu : 0.f;
        q += d * d;
      }
    }
    const float rs = rsqrtf(block_sum<4>(q, red) / N + eps);
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      int j = threadIdx.x + k * T;
      if (j < H) {
        float zr = (v[0][k] - mu) * rs * gm[0][k] + bt[0][k];
        float zc = (v[1][k] - mu) * rs * gm[1][k] + bt[1][k];
        float zu = (v[2][k] - mu) * rs * gm[2][k] + bt[2][k];
        float r = sigmoidf_(zr);
        float c = tanhf(r * zc);
        float u = sigmoidf_(zu - 1.f);
        hn[(int64_t)row * ldo + j] = u * c + (1.f - u) * hp[k];
      }
    }
    if (threadIdx.x == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  }
}

// Wide-row forms (H a multiple of 1024: the L / XL deter sizes): one float4 per gate per thread, H / 4 threads
// (NW = H / 256 waves) per row, so a 16-row scan step still runs 16 x NW waves, and every load is a 16-byte
// vector load issued before the row statistics reduce.  The scalar forms issue 3 * MAXH four-byte loads per
// thread per row from 256 threads.
template <int NW>
__global__ void __launch_bounds__(64 * NW) ln_gru_fwd4_kernel(const float* x, const float* __restrict__ h, int ldh,
                                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                                              float* __restrict__ hn, float* __restrict__ mean_out,
                                                              float* __restrict__ rstd_out, int M, int H, float eps,
                                                              int ldo, const float* __restrict__ x2, int ldx2, float* xsum) {
  __shared__ float red[NW];
  const int N = 3 * H, H4 = H >> 2, j4 = threadIdx.x;
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  const float4* b4 = reinterpret_cast<const float4*>(beta);
  const float4 gr = g4[j4], gc = g4[H4 + j4], gu = g4[2 * H4 + j4];
  const float4 br = b4[j4], bc = b4[H4 + j4], bu = b4[2 * H4 + j4];
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)row * N);
    const float4* x2r = x2 ? reinterpret_cast<const float4*>(x2 + (int64_t)row * ldx2) : nullptr;
    float4 v[3];
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      float4 a = xr[g * H4 + j4];
      if (x2r) {
        const float4 b = x2r[g * H4 + j4];
        a.x += b.x, a.y += b.y, a.z += b.z, a.w += b.w;
      }
      v[g] = a;
      s += (a.x + a.y) + (a.z + a.w);
      if (xsum) reinterpret_cast<float4*>(xsum + (int64_t)row * N)[g * H4 + j4] = a;
    }
    const float4 hp = reinterpret_cast<const float4*>(h + (int64_t)row * ldh)[j4];
    const float mu = block_sum<NW>(s, red) / N;
    float q = 0.f;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      const float a = v[g].x - mu, b = v[g].y - mu, c = v[g].z - mu, d = v[g].w - mu;
      q += (a * a + b * b) + (c * c + d * d);
    }
    const float rs = rsqrtf(block_sum<NW>(q, red) / N + eps);
    float4 o;
#define SRL_GRU_LANE(C)                                                   \
  {                                                                       \
    const float r = sigmoidf_((v[0].C - mu) * rs * gr.C + br.C);          \
    const float c = tanhf(r * ((v[1].C - mu) * rs * gc.C + bc.C));        \
    const float u = sigmoidf_((v[2].C - mu) * rs * gu.C + bu.C - 1.f);    \
    o.C = u * c + (1.f - u) * hp.C;                                       \
  }
    SRL_GRU_LANE(x) SRL_GRU_LANE(y) SRL_GRU_LANE(z) SRL_GRU_LANE(w)
#undef SRL_GRU_LANE
    reinterpret_cast<float4*>(hn + (int64_t)row * ldo)[j4] = o;
    if (threadIdx.x == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  }
}

// Backward of the wide-row form: same thread map; per-block LN-GRU parameter partials kept in registers across
// the block's rows ([grid, 3H] partial rows, reduced by colsum2 as for the scalar form).
template <int NW>
__global__ void __launch_bounds__(64 * NW) ln_gru_bwd4_kernel(const float* __restrict__ x, const float* __restrict__ h, int ldh,
                                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                                              const float* __restrict__ mean, const float* __restrict__ rstd,
                                                              const float* __restrict__ dhn, float* __restrict__ dx,
                                                              float* __restrict__ dh, float* __restrict__ pdg,
                                                              float* __restrict__ pdb, int M, int H,
                                                              const float* __restrict__ dadd, int ldadd) {
  __shared__ float red[NW];
  const int N = 3 * H, H4 = H >> 2, j4 = threadIdx.x;
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  const float4* b4 = reinterpret_cast<const float4*>(beta);
  const float4 G0 = g4[j4], G1 = g4[H4 + j4], G2 = g4[2 * H4 + j4];
  const float4 B0 = b4[j4], B1 = b4[H4 + j4], B2 = b4[2 * H4 + j4];
  float4 ag0 = {0.f, 0.f, 0.f, 0.f}, ag1 = ag0, ag2 = ag0, ab0 = ag0, ab1 = ag0, ab2 = ag0;
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)row * N);
    const float4 X0 = xr[j4], X1 = xr[H4 + j4], X2 = xr[2 * H4 + j4];
    const float4 hp = reinterpret_cast<const float4*>(h + (int64_t)row * ldh)[j4];
    const float4 go = reinterpret_cast<const float4*>(dhn + (int64_t)row * H)[j4];
    const float mu = mean[row], rs = rstd[row];
    float4 xh0, xh1, xh2, d0, d1, d2, dho;
    float s1 = 0.f, s2 = 0.f;
#define SRL_GRU_BWD_LANE(C)                                                       \
  {                                                                               \
    const float hr = (X0.C - mu) * rs, hc = (X1.C - mu) * rs, hu = (X2.C - mu) * rs; \
    const float zc = hc * G1.C + B1.C;                                            \
    const float r = sigmoidf_(hr * G0.C + B0.C);                                  \
    const float c = tanhf(r * zc);                                                \
    const float u = sigmoidf_(hu * G2.C + B2.C - 1.f);                            \
    const float g = go.C;                                                         \
    dho.C = g * (1.f - u);                                                        \
    const float dzu = g * (c - hp.C) * u * (1.f - u);                             \
    const float da = g * u * (1.f - c * c);                                       \
    const float dzc = da * r;                                                     \
    const float dzr = da * zc * r * (1.f - r);                                    \
    ag0.C += dzr * hr, ag1.C += dzc * hc, ag2.C += dzu * hu;                      \
    ab0.C += dzr, ab1.C += dzc, ab2.C += dzu;                                     \
    xh0.C = hr, xh1.C = hc, xh2.C = hu;                                           \
    d0.C = dzr * G0.C, d1.C = dzc * G1.C, d2.C = dzu * G2.C;                      \
    s1 += d0.C + d1.C + d2.C;                                                     \
    s2 += d0.C * hr + d1.C * hc + d2.C * hu;                                      \
  }
    SRL_GRU_BWD_LANE(x) SRL_GRU_BWD_LANE(y) SRL_GRU_BWD_LANE(z) SRL_GRU_BWD_LANE(w)
#undef SRL_GRU_BWD_LANE
    if (dadd) {  // an extra gradient into h_{t-1} (row-strided), added here instead of by a separate kernel
      const float4 e = reinterpret_cast<const float4*>(dadd + (int64_t)row * ldadd)[j4];
      dho.x += e.x, dho.y += e.y, dho.z += e.z, dho.w += e.w;
    }
    reinterpret_cast<float4*>(dh + (int64_t)row * H)[j4] = dho;
    const float m1 = block_sum<NW>(s1, red) / N;
    const float m2 = block_sum<NW>(s2, red) / N;
    float4* dxr = reinterpret_cast<float4*>(dx + (int64_t)row * N);
    float4 o;
#define SRL_DX(D, XH, OUTI)                                       \
  o.x = rs * (D.x - m1 - XH.x * m2), o.y = rs * (D.y - m1 - XH.y * m2); \
  o.z = rs * (D.z - m1 - XH.z * m2), o.w = rs * (D.w - m1 - XH.w * m2); \
  dxr[OUTI] = o;
    SRL_DX(d0, xh0, j4)
    SRL_DX(d1, xh1, H4 + j4)
    SRL_DX(d2, xh2, 2 * H4 + j4)
#undef SRL_DX
  }
  float4* pg = reinterpret_cast<float4*>(pdg + (int64_t)blockIdx.x * N);
  float4* pb = reinterpret_cast<float4*>(pdb + (int64_t)blockIdx.x * N);
  pg[j4] = ag0, pg[H4 + j4] = ag1, pg[2 * H4 + j4] = ag2;
  pb[j4] = ab0, pb[H4 + j4] = ab1, pb[2 * H4 + j4] = ab2;
}

template <int MAXH>
__global__ void __launch_bounds__(256) ln_gru_bwd_kernel(const float* __restrict__ x, const float* __restrict__ h, int ldh,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         const float* __restrict__ dhn, float* __restrict__ dx,
                                                         float* __restrict__ dh, float* __restrict__ pdg,
                                                         float* __restrict__ pdb, int M, int H,
                                                         const float* __restrict__ dadd, int ldadd) {
  __shared__ float red[4];
  const int T = 256, N = 3 * H;
  float ag[3][MAXH], ab[3][MAXH];
#pragma unroll
  for (int k = 0; k < MAXH; ++k)
#pragma unroll
    for (int g = 0; g < 3; ++g) ag[g][k] = ab[g][k] = 0.f;
  // row-invariant LN parameters hoisted; the next row's inputs are requested before this row's math (a block walks
  // M / grid rows: at M = 15360 one memory latency per row was the kernel's time)
  float gm[3][MAXH], bt[3][MAXH];
#pragma unroll
  for (int k = 0; k < MAXH; ++k) {
    const int j = threadIdx.x + k * T;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      gm[g][k] = j < H ? gamma[g * H + j] : 0.f;
      bt[g][k] = j < H ? beta[g * H + j] : 0.f;
    }
  }
  struct RowIn {
    float x[3][MAXH], h[MAXH], go[MAXH], ad[MAXH], mu, rs;
  };
  auto load = [&](int row, RowIn& in) {
    const float* xr = x + (int64_t)row * N;
    in.mu = mean[row];
    in.rs = rstd[row];
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      const int j = threadIdx.x + k * T;
      const bool ok = j < H;
#pragma unroll
      for (int g = 0; g < 3; ++g) in.x[g][k] = ok ? xr[g * H + j] : 0.f;
      in.h[k] = ok ? h[(int64_t)row * ldh + j] : 0.f;
      in.go[k] = ok ? dhn[(int64_t)row * H + j] : 0.f;
      in.ad[k] = (ok && dadd) ? dadd[(int64_t)row * ldadd + j] : 0.f;
    }
  };
  constexpr bool PF = MAXH <= 4;  // (wider rows: no second row of registers, one row at a time as before)
  RowIn cur, nxt;
  if (PF && blockIdx.x < M) load(blockIdx.x, cur);
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    if (!PF) load(row, cur);
    if (PF && row + (int)gridDim.x < M) load(row + gridDim.x, nxt);
    const float mu = cur.mu, rs = cur.rs;
    float xh[3][MAXH], dxh[3][MAXH];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      int j = threadIdx.x + k * T;
#pragma unroll
      for (int g = 0; g < 3; ++g) xh[g][k] = dxh[g][k] = 0.f;
      if (j < H) {
        float hr = (cur.x[0][k] - mu) * rs, hc = (cur.x[1][k] - mu) * rs, hu = (cur.x[2][k] - mu) * rs;
        float gr = gm[0][k], gc = gm[1][k], gu = gm[2][k];
        float zr = hr * gr + bt[0][k], zc = hc * gc + bt[1][k], zu = hu * gu + bt[2][k];
        float r = sigmoidf_(zr);
        float c = tanhf(r * zc);
        float u = sigmoidf_(zu - 1.f);
        float hp = cur.h[k];
        float g_out = cur.go[k];
        dh[(int64_t)row * H + j] = g_out * (1.f - u) + (dadd ? cur.ad[k] : 0.f);
        float du = g_out * (c - hp);
        float dc = g_out * u;
        float dzu = du * u * (1.f - u);
        float da = dc * (1.f - c * c);
        float dzc = da * r;
        float dr = da * zc;
        float dzr = dr * r * (1.f - r);
        ag[0][k] += dzr * hr; ag[1][k] += dzc * hc; ag[2][k] += dzu * hu;
        ab[0][k] += dzr; ab[1][k] += dzc; ab[2][k] += dzu;
        xh[0][k] = hr; xh[1][k] = hc; xh[2][k] = hu;
        dxh[0][k] = dzr * gr; dxh[1][k] = dzc * gc; dxh[2][k] = dzu * gu;
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          s1 += dxh[g][k];
          s2 += dxh[g][k] * xh[g][k];
        }
      }
    }
    const float m1 = block_sum<4>(s1, red) / N;
    const float m2 = block_sum<4>(s2, red) / N;
    float* dxr = dx + (int64_t)row * N;
#pragma unroll
    for (int k = 0; k < MAXH; ++k) {
      int j = threadIdx.x + k * T;
      if (j < H) {
#pragma unroll
        for (int g = 0; g < 3; ++g) dxr[g * H + j] = rs * (dxh[g][k] - m1 - xh[g][k] * m2);
      }
    }
    if (PF) cur = nxt;
  }
#pragma unroll
  for (int k = 0; k < MAXH; ++k) {
    int j = threadIdx.x + k * T;
    if (j < H) {
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        pdg[(int64_t)blockIdx.x * N + g * H + j] = ag[g][k];
        pdb[(int64_t)blockIdx.x * N + g * H + j] = ab[g][k];
      }
    }
  }
}

}  // namespace srl

using namespace srl;

// the float4 wide-row forward / backward where the shape allows (set_gru_vec(false): the scalar kernels for every H,
// tests only)
static bool g_gru_vec = true;
void set_gru_vec(bool on) { g_gru_vec = on; }

static int gru_maxh(int H) {
  if (H <= 512) return 2;
  if (H <= 1024) return 4;
  if (H <= 2048) return 8;
  if (H <= 4096) return 16;
  return 0;
}

bool launch_ln_gru_fwd(const float* x, const float* h, int ldh, const float* gamma, const float* beta, float* hn,
                       float* mean, float* rstd, int M, int H, float eps, hipStream_t st, int ldo, const float* x2, int ldx2,
                       float* xsum) {
  if (ldo <= 0) ldo = H;
  int mh = gru_maxh(H);
  dim3 g(M < 8192 ? M : 8192), b(256);
  const bool al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(hn) |
                    reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) |
                    reinterpret_cast<uintptr_t>(x2) | reinterpret_cast<uintptr_t>(xsum)) & 15) == 0 && ldh % 4 == 0 && ldo % 4 == 0 && (!x2 || ldx2 % 4 == 0);
  if (g_gru_vec && al && H % 1024 == 0 && H <= 4096) {
    const dim3 bw(H / 4);
    switch (H / 1024) {
      case 1: hipLaunchKernelGGL(ln_gru_fwd4_kernel<4>, g, bw, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
      case 2: hipLaunchKernelGGL(ln_gru_fwd4_kernel<8>, g, bw, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
      case 4: hipLaunchKernelGGL(ln_gru_fwd4_kernel<16>, g, bw, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
      default: break;
    }
  }
  switch (mh) {
    case 2: hipLaunchKernelGGL(ln_gru_fwd_kernel<2>, g, b, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
    case 4: hipLaunchKernelGGL(ln_gru_fwd_kernel<4>, g, b, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
    case 8: hipLaunchKernelGGL(ln_gru_fwd_kernel<8>, g, b, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
    case 16: hipLaunchKernelGGL(ln_gru_fwd_kernel<16>, g, b, 0, st, x, h, ldh, gamma, beta, hn, mean, rstd, M, H, eps, ldo, x2, ldx2, xsum); return true;
    default: return false;
  }
}

int ln_gru_bwd_grid(int M) { return M < 256 ? M : 256; }

void launch_colsum2(const float* pa, const float* pb, float* oa, float* ob, int rows, int N, int G, hipStream_t st);

// pdg/pdb: [grid, 3H] partial rows; reduced into dgamma/dbeta when those are non-null.
bool launch_ln_gru_bwd(const float* x, const float* h, int ldh, const float* gamma, const float* beta, const float* mean,
                       const float* rstd, const float* dhn, float* dx, float* dh, float* pdg, float* pdb, float* dgamma,
                       float* dbeta, int M, int H, hipStream_t st, const float* dadd, int ldadd) {
  int mh = gru_maxh(H);
  int grid = ln_gru_bwd_grid(M);
  dim3 g(grid), b(256);
  const bool al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(dhn) |
                    reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(dh) | reinterpret_cast<uintptr_t>(pdg) |
                    reinterpret_cast<uintptr_t>(pdb) | reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta)) &
                   15) == 0 && ldh % 4 == 0 && (!dadd || ((reinterpret_cast<uintptr_t>(dadd) & 15) == 0 && ldadd % 4 == 0));
  if (g_gru_vec && al && H % 1024 == 0 && H <= 4096 && (H / 1024 == 1 || H / 1024 == 2 || H / 1024 == 4)) {
    const dim3 bw(H / 4);
    if (H == 1024) hipLaunchKernelGGL(ln_gru_bwd4_kernel<4>, g, bw, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd);
    else if (H == 2048) hipLaunchKernelGGL(ln_gru_bwd4_kernel<8>, g, bw, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd);
    else hipLaunchKernelGGL(ln_gru_bwd4_kernel<16>, g, bw, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd);
    if (dgamma) launch_colsum2(pdg, pdb, dgamma, dbeta, grid, 3 * H, 1, st);
    return true;
  }
  switch (mh) {
    case 2: hipLaunchKernelGGL(ln_gru_bwd_kernel<2>, g, b, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd); break;
    case 4: hipLaunchKernelGGL(ln_gru_bwd_kernel<4>, g, b, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd); break;
    case 8: hipLaunchKernelGGL(ln_gru_bwd_kernel<8>, g, b, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd); break;
    case 16: hipLaunchKernelGGL(ln_gru_bwd_kernel<16>, g, b, 0, st, x, h, ldh, gamma, beta, mean, rstd, dhn, dx, dh, pdg, pdb, M, H, dadd, ldadd); break;
    default: return false;
  }
  if (dgamma) launch_colsum2(pdg, pdb, dgamma, dbeta, grid, 3 * H, 1, st);
  return true;
}
