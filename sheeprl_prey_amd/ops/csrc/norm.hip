// Fused LayerNorm + activation kernels (fp32).
//  * row-major:  y[m, :] = act(gamma * (x - mu) * rstd + beta)   (nn.Linear -> LayerNorm -> act)
//  * NCHW:       normalise over C at every pixel directly in NCHW (the reference permutes to
//                NHWC and back around nn.LayerNorm: LayerNormChannelLast, utils/model.py:225-235;
//                here consecutive threads own consecutive pixels, so the C-strided reads coalesce).
// Backward recomputes x_hat from the saved (mu, rstd); dgamma/dbeta are reduced
// deterministically: per-block partial rows, then a column-sum kernel.
#include "common.h"

namespace srl {

template <int NW, int MAXV>
__global__ void __launch_bounds__(64 * NW) ln_act_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ y,
                                                             float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                             int M, int N, float eps, int act) {
  __shared__ float red[NW];
  const int T = 64 * NW;
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + (int64_t)row * N;
    float v[MAXV];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * T;
      v[k] = idx < N ? xr[idx] : 0.f;
      s += v[k];
    }
    const float mu = block_sum<NW>(s, red) / N;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * T;
      float d = idx < N ? v[k] - mu : 0.f;
      q += d * d;
    }
    const float var = block_sum<NW>(q, red) / N;
    const float rs = rsqrtf(var + eps);
    float* yr = y + (int64_t)row * N;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * T;
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

template <int NW, int MAXV>
__global__ void __launch_bounds__(64 * NW) ln_act_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                                             const float* __restrict__ mean, const float* __restrict__ rstd,
                                                             float* __restrict__ dx, float* __restrict__ pdg,
                                                             float* __restrict__ pdb, int M, int N, int act) {
  __shared__ float red[NW];
  const int T = 64 * NW;
  float ag[MAXV], ab[MAXV];
#pragma unroll
  for (int k = 0; k < MAXV; ++k) ag[k] = ab[k] = 0.f;
  for (int row = blockIdx.x; row < M; row += gridDim.x) {
    const float* xr = x + (int64_t)row * N;
    const float* dyr = dy + (int64_t)row * N;
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXV], dxh[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * T;
      xh[k] = 0.f;
      dxh[k] = 0.f;
      if (idx < N) {
        float h = (xr[idx] - mu) * rs;
        float g = gamma ? gamma[idx] : 1.f;
        float z = gamma ? h * g + beta[idx] : h;
        float dz = dyr[idx] * act_grad(z, act);
        ag[k] += dz * h;
        ab[k] += dz;
        xh[k] = h;
        dxh[k] = dz * g;
        s1 += dxh[k];
        s2 += dxh[k] * h;
      }
    }
    const float m1 = block_sum<NW>(s1, red) / N;
    const float m2 = block_sum<NW>(s2, red) / N;
    float* dxr = dx + (int64_t)row * N;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * T;
      if (idx < N) dxr[idx] = rs * (dxh[k] - m1 - xh[k] * m2);
    }
  }
  if (pdg) {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      int idx = threadIdx.x + k * T;
      if (idx < N) {
        pdg[(int64_t)blockIdx.x * N + idx] = ag[k];
        pdb[(int64_t)blockIdx.x * N + idx] = ab[k];
      }
    }
  }
}

// out_a[n] = sum_b pa[b, n]; out_b likewise (deterministic order)
__global__ void __launch_bounds__(256) colsum2_kernel(const float* __restrict__ pa, const float* __restrict__ pb,
                                                      float* __restrict__ oa, float* __restrict__ ob, int rows, int N) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float a = 0.f, b = 0.f;
  for (int r = 0; r < rows; ++r) {
    a += pa[(int64_t)r * N + n];
    b += pb[(int64_t)r * N + n];
  }
  oa[n] = a;
  ob[n] = b;
}

// ---------------------------------------------------------------- NCHW (normalise over C)
__global__ void __launch_bounds__(256) ln_nchw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int B, int C, int HW, float eps, int act) {
  int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pix >= (int64_t)B * HW) return;
  int b = pix / HW, p = pix % HW;
  const float* xb = x + (int64_t)b * C * HW + p;
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += xb[(int64_t)c * HW];
  float mu = s / C;
  float q = 0.f;
  for (int c = 0; c < C; ++c) {
    float d = xb[(int64_t)c * HW] - mu;
    q += d * d;
  }
  float rs = rsqrtf(q / C + eps);
  float* yb = y + (int64_t)b * C * HW + p;
  for (int c = 0; c < C; ++c) {
    float z = (xb[(int64_t)c * HW] - mu) * rs;
    if (gamma) z = z * gamma[c] + beta[c];
    yb[(int64_t)c * HW] = act_fwd(z, act);
  }
  mean_out[pix] = mu;
  rstd_out[pix] = rs;
}

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

#define LN_DISPATCH(NW, MAXV, KERNEL, ...) \
  hipLaunchKernelGGL((KERNEL<NW, MAXV>), dim3(grid), dim3(64 * NW), 0, st, __VA_ARGS__)

// Picks (waves per row, values per thread).  Returns false if N is unsupported.
static bool ln_config(int N, int& nw, int& maxv) {
  if (N <= 256) { nw = 1; maxv = 4; }
  else if (N <= 512) { nw = 1; maxv = 8; }
  else if (N <= 1024) { nw = 2; maxv = 8; }
  else if (N <= 2048) { nw = 4; maxv = 8; }
  else if (N <= 4096) { nw = 4; maxv = 16; }
  else if (N <= 12288) { nw = 4; maxv = 48; }
  else return false;
  return true;
}

bool launch_ln_act_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int M,
                       int N, float eps, int act, hipStream_t st) {
  int nw, maxv;
  if (!ln_config(N, nw, maxv)) return false;
  int grid = M;
#define F(NW_, MV_) if (nw == NW_ && maxv == MV_) { LN_DISPATCH(NW_, MV_, ln_act_fwd_kernel, x, gamma, beta, y, mean, rstd, M, N, eps, act); return true; }
  F(1, 4) F(1, 8) F(2, 8) F(4, 8) F(4, 16) F(4, 48)
#undef F
  return false;
}

int ln_act_bwd_grid(int M) { return M < 512 ? M : 512; }

bool launch_ln_act_bwd(const float* x, const float* dy, const float* gamma, const float* beta, const float* mean,
                       const float* rstd, float* dx, float* pdg, float* pdb, float* dgamma, float* dbeta, int M, int N,
                       int act, hipStream_t st) {
  int nw, maxv;
  if (!ln_config(N, nw, maxv)) return false;
  int grid = ln_act_bwd_grid(M);
#define F(NW_, MV_) if (nw == NW_ && maxv == MV_) { LN_DISPATCH(NW_, MV_, ln_act_bwd_kernel, x, dy, gamma, beta, mean, rstd, dx, pdg, pdb, M, N, act); goto reduce; }
  F(1, 4) F(1, 8) F(2, 8) F(4, 8) F(4, 16) F(4, 48)
#undef F
  return false;
reduce:
  if (dgamma) hipLaunchKernelGGL(colsum2_kernel, dim3(cdiv(N, 256)), dim3(256), 0, st, pdg, pdb, dgamma, dbeta, grid, N);
  return true;
}

void launch_ln_nchw_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int B,
                        int C, int HW, float eps, int act, hipStream_t st) {
  int64_t P = (int64_t)B * HW;
  hipLaunchKernelGGL(ln_nchw_fwd_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, x, gamma, beta, y, mean, rstd,
                     B, C, HW, eps, act);
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
  hipLaunchKernelGGL(ln_nchw_bwd_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, x, dy, gamma, beta, mean, rstd,
                     dx, B, C, HW, act);
  if (gamma) {
    int S = ln_nchw_splits(B, HW);
    hipLaunchKernelGGL(ln_nchw_dgb_kernel, dim3(C, S), dim3(256), 0, st, x, dy, gamma, beta, mean, rstd, pdg, pdb, B, C, HW,
                       act);
    hipLaunchKernelGGL(colsum2_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, pdg, pdb, dgamma, dbeta, S, C);
  }
}
