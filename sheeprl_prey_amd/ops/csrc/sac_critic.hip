// Fused SAC twin-Q critic update, forward + loss + backward (K15; reference sac/agent.py:256-275 critic
// evaluation, sac/loss.py:15-20 critic loss, sac/sac.py:36-52 the update):
//
//   h1_c = relu(W1_c [obs, act] + b1_c),  h2_c = relu(W2_c h1_c + b2_c),  q_c = w3_c . h2_c + b3_c
//   loss = sum_c mean_b (q_c - y)^2
//
// Two launches instead of ~20 (concat, 3 GEMM layers, 2 ReLUs, the loss reduction and their autograd
// backward: GEMM pairs, ReLU masks, bias column sums):
//   fwd kernel   (grid: 16-row blocks x critics, 8 waves): the whole forward of one critic on 16 rows,
//                the loss partial, dq = 2 (q - y) / B, dh2 = dq w3 * [h2 > 0] and dh1 = (dh2 W2) * [h1 > 0]
//                (a 16-row GEMM against W2 read K-major) - activations stay in LDS, the operands of
//                the weight gradients (x, h1, h2, dh1, dh2, dq) are written once to global;
//   wgrad kernel (grid: 16x16 output tiles of dW2 / dW1 per critic, 8 per workgroup, + one
//                bias workgroup per critic): dW = dh^T act over the batch (fp32 MFMA 16x16x4, K = batch
//                rows), bias / head gradients as column sums, all scaled by the loss gradient (device
//                scalar: the launch is graph-capturable).
// Weights are the stacked ensemble layout [n, out, in] (models/ensemble.py).
#include "common.h"
#include "sac_tiles.h"

namespace srl {
namespace saccrit {

constexpr int NTH = 512;
constexpr int NW = NTH / 64;
constexpr int ROWS = 16;

using namespace sactile;

struct FP {
  const float* obs;
  const float* act;
  const float* y;   // [M] Bellman targets
  const float* W1;  // [n, H, IN]
  const float* b1;  // [n, H]
  const float* W2;  // [n, H, H]
  const float* b2;  // [n, H]
  const float* W3;  // [n, 1, H]
  const float* b3;  // [n, 1]
  float* X;         // [M, INp]  (critic-0 workgroups write it)
  float* H1;        // [n, M, H]
  float* H2;        // [n, M, H]
  float* DH1;       // [n, M, H]
  float* DH2;       // [n, M, H]
  float* DQ;        // [n, M]
  float* Q;         // [M, n]  (the critics' values, for metrics / tests)
  float* lossp;     // [n * blocks] partial losses
  int M, OD, AD, IN, INp, H, n;
};

__global__ __launch_bounds__(NTH) void critic_fwd_kernel(FP p) {
  extern __shared__ float sm[];
  const int ldx = p.INp + 4, ldh = p.H + 4, H = p.H, M = p.M;
  float* xs = sm;                 // [16][INp + 4]
  float* h1s = xs + ROWS * ldx;   // [16][H + 4]
  float* h2s = h1s + ROWS * ldh;  // [16][H + 4]  h2, then dh2 in place
  float* qp = h2s + ROWS * ldh;   // [NW][16]
  float* dqs = qp + NW * ROWS;    // [16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y, r0 = blockIdx.x * ROWS;
  const int j = lane & 15, q = lane >> 4;
  for (int i = tid; i < ROWS * p.INp; i += NTH) {  // x = [obs, act], zero padded (rows and columns)
    const int r = i / p.INp, k = i - r * p.INp, row = r0 + r;
    float v = 0.f;
    if (row < M) v = k < p.OD ? p.obs[(long)row * p.OD + k] : (k < p.IN ? p.act[(long)row * p.AD + k - p.OD] : 0.f);
    xs[r * ldx + k] = v;
    if (c == 0 && row < M) p.X[(long)row * p.INp + k] = v;
  }
  __syncthreads();
  const int tiles = H / (16 * NW);
  const float* W1 = p.W1 + (long)c * H * p.IN;
  float* H1 = p.H1 + (long)c * M * H;
  // first layer: the whole (small) K of both tiles' weights in flight at once
  wave_tiles<2, NW>(xs, ldx, W1, p.IN, H, p.IN, lane, wave, [&](int n0, const floatx4& acc) {
    const float bb = p.b1[c * H + n0 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float h = fmaxf(acc[e] + bb, 0.f);
      h1s[(4 * q + e) * ldh + n0 + j] = h;
      if (r0 + 4 * q + e < M) H1[(long)(r0 + 4 * q + e) * H + n0 + j] = h;
    }
  });
  __syncthreads();
  const float* W2 = p.W2 + (long)c * H * H;
  float* H2 = p.H2 + (long)c * M * H;
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  wave_tiles<0, NW>(h1s, ldh, W2, H, H, H, lane, wave, [&](int n0, const floatx4& acc) {
    const float bb = p.b2[c * H + n0 + j], w3 = p.W3[c * H + n0 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float h = fmaxf(acc[e] + bb, 0.f);
      part[e] += h * w3;
      h2s[(4 * q + e) * ldh + n0 + j] = h;
      if (r0 + 4 * q + e < M) H2[(long)(r0 + 4 * q + e) * H + n0 + j] = h;
    }
  });
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v = part[e];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (j == 0) qp[wave * ROWS + 4 * q + e] = v;
  }
  __syncthreads();
  if (tid < 64) {  // q, dq, and the block's loss partial (one wave)
    float d2 = 0.f;
    if (tid < ROWS) {
      const int row = r0 + tid;
      float qv = p.b3[c];
      for (int w = 0; w < NW; ++w) qv += qp[w * ROWS + tid];
      float dq = 0.f;
      if (row < M) {
        const float d = qv - p.y[row];
        d2 = d * d;
        dq = 2.f * d / (float)M;
        p.DQ[(long)c * M + row] = dq;
        p.Q[(long)row * p.n + c] = qv;
      }
      dqs[tid] = dq;
    }
    const float s = wave_sum(d2);
    if (tid == 0) p.lossp[(long)c * gridDim.x + blockIdx.x] = s / (float)M;
  }
  __syncthreads();
  // dh2 = dq * w3 * [h2 > 0], in place of h2
  const float* w3 = p.W3 + (long)c * H;
  float* DH2 = p.DH2 + (long)c * M * H;
  for (int i = tid; i < ROWS * H; i += NTH) {
    const int r = i / H, k = i - r * H;
    float* hp = h2s + r * ldh + k;
    const float d = *hp > 0.f ? dqs[r] * w3[k] : 0.f;
    *hp = d;
    if (r0 + r < M) DH2[(long)(r0 + r) * H + k] = d;
  }
  __syncthreads();
  // dh1 = (dh2 W2) * [h1 > 0]
  float* DH1 = p.DH1 + (long)c * M * H;
  wave_tiles<1, NW>(h2s, ldh, W2, H, H, H, lane, wave, [&](int n0, const floatx4& acc) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * q + e;
      if (r0 + r < M) DH1[(long)(r0 + r) * H + n0 + j] = h1s[r * ldh + n0 + j] > 0.f ? acc[e] : 0.f;
    }
  });
}

struct GP {
  const float* X;
  const float* H1;
  const float* H2;
  const float* DH1;
  const float* DH2;
  const float* DQ;
  const float* g;  // loss gradient (device scalar)
  float* dW1;      // [n, H, IN]
  float* db1;      // [n, H]
  float* dW2;      // [n, H, H]
  float* db2;      // [n, H]
  float* dW3;      // [n, 1, H]
  float* db3;      // [n, 1]
  const float* lossp;  // [nlp] partial losses of the forward kernel, or null
  float* loss;         // their sum (the loss value), written by one extra workgroup when lossp is set
  int M, IN, INp, H, n, nlp;
  int nb2, nb1;    // workgroups of the dW2 / dW1 roles
};

__global__ __launch_bounds__(NTH) void critic_wgrad_kernel(GP p) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = p.H, M = p.M, j = lane & 15, q = lane >> 4;
  const float g = *p.g;
  int b = blockIdx.x;
  if (b < p.nb2) {  // dW2 tiles: (critic, i-tile, j-tile), 8 per workgroup
    const int nt = H / 16;
    const int tile = b * NW + wave;
    if (tile >= p.n * nt * nt) return;
    const int c = tile / (nt * nt), ij = tile - c * nt * nt, i0 = (ij / nt) * 16, j0 = (ij % nt) * 16;
    const floatx4 acc = tile_wgrad(p.DH2 + (long)c * M * H, H, p.H1 + (long)c * M * H, H, i0, j0, M, lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) p.dW2[((long)c * H + i0 + 4 * q + e) * H + j0 + j] = g * acc[e];
    return;
  }
  b -= p.nb2;
  if (b < p.nb1) {  // dW1 tiles over the padded input width
    const int ni = H / 16, nj = p.INp / 16;
    const int tile = b * NW + wave;
    if (tile >= p.n * ni * nj) return;
    const int c = tile / (ni * nj), ij = tile - c * ni * nj, i0 = (ij / nj) * 16, j0 = (ij % nj) * 16;
    const floatx4 acc = tile_wgrad(p.DH1 + (long)c * M * H, H, p.X, p.INp, i0, j0, M, lane);
    if (j0 + j < p.IN) {
#pragma unroll
      for (int e = 0; e < 4; ++e) p.dW1[((long)c * H + i0 + 4 * q + e) * p.IN + j0 + j] = g * acc[e];
    }
    return;
  }
  b -= p.nb1;  // bias / head workgroups (critic, 64 columns): column sums over the batch, rows split over waves
  __shared__ float red[NW][3][64];
  const int nch = H / 64;
  if (b == p.n * nch) {  // loss workgroup: the forward's partial losses summed in a fixed order (one wave)
    if (wave == 0) {
      float s = 0.f;
      for (int i = lane; i < p.nlp; i += 64) s += p.lossp[i];
      s = wave_sum(s);
      if (lane == 0) *p.loss = s;
    }
    return;
  }
  const int c = b / nch, k = (b - c * nch) * 64 + lane;
  const float* DH1 = p.DH1 + (long)c * M * H;
  const float* DH2 = p.DH2 + (long)c * M * H;
  const float* H2 = p.H2 + (long)c * M * H;
  const float* DQ = p.DQ + (long)c * M;
  float s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
  for (int r = wave; r < M; r += NW) {
    const float dq = DQ[r];
    s1 += DH1[(long)r * H + k];
    s2 += DH2[(long)r * H + k];
    s3 += dq * H2[(long)r * H + k];
    s4 += lane == 0 ? dq : 0.f;
  }
  red[wave][0][lane] = s1;
  red[wave][1][lane] = s2;
  red[wave][2][lane] = s3;
  s4 = __shfl(s4, 0, 64);
  __syncthreads();
  if (wave == 0) {
    float a = 0.f, bb = 0.f, cc = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      a += red[w][0][lane];
      bb += red[w][1][lane];
      cc += red[w][2][lane];
    }
    p.db1[(long)c * H + k] = g * a;
    p.db2[(long)c * H + k] = g * bb;
    p.dW3[(long)c * H + k] = g * cc;
  }
  __syncthreads();
  if (k == 0 && lane == 0) red[wave][0][0] = s4;  // (k == 0: the first column chunk's waves)
  __syncthreads();
  if (k == 0 && wave == 0) {
    float t = 0.f;
    for (int w = 0; w < NW; ++w) t += red[w][0][0];
    p.db3[c] = g * t;
  }
}

}  // namespace saccrit
}  // namespace srl

using namespace srl::saccrit;

size_t sac_critic_fwd_lds(int INp, int H) {
  return sizeof(float) * (16 * (size_t)(INp + 4) + 32 * (size_t)(H + 4) + NW * 16 + 16);
}

int sac_critic_blocks(int M) { return (M + ROWS - 1) / ROWS; }

void launch_sac_critic_fwd(const float* obs, const float* act, const float* y, const float* W1, const float* b1,
                           const float* W2, const float* b2, const float* W3, const float* b3, float* X, float* H1, float* H2,
                           float* DH1, float* DH2, float* DQ, float* Q, float* lossp, int M, int OD, int AD, int H, int n,
                           hipStream_t st) {
  FP p;
  p.obs = obs;
  p.act = act;
  p.y = y;
  p.W1 = W1;
  p.b1 = b1;
  p.W2 = W2;
  p.b2 = b2;
  p.W3 = W3;
  p.b3 = b3;
  p.X = X;
  p.H1 = H1;
  p.H2 = H2;
  p.DH1 = DH1;
  p.DH2 = DH2;
  p.DQ = DQ;
  p.Q = Q;
  p.lossp = lossp;
  p.M = M;
  p.OD = OD;
  p.AD = AD;
  p.IN = OD + AD;
  p.INp = (p.IN + 15) / 16 * 16;
  p.H = H;
  p.n = n;
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute((const void*)critic_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    init = true;
  }
  hipLaunchKernelGGL(critic_fwd_kernel, dim3(sac_critic_blocks(M), n), dim3(NTH), sac_critic_fwd_lds(p.INp, H), st, p);
}

void launch_sac_critic_wgrad(const float* X, const float* H1, const float* H2, const float* DH1, const float* DH2,
                             const float* DQ, const float* g, float* dW1, float* db1, float* dW2, float* db2, float* dW3,
                             float* db3, int M, int IN, int H, int n, const float* lossp, int nlp, float* loss,
                             hipStream_t st) {
  GP p;
  p.X = X;
  p.H1 = H1;
  p.H2 = H2;
  p.DH1 = DH1;
  p.DH2 = DH2;
  p.DQ = DQ;
  p.g = g;
  p.dW1 = dW1;
  p.db1 = db1;
  p.dW2 = dW2;
  p.db2 = db2;
  p.dW3 = dW3;
  p.db3 = db3;
  p.M = M;
  p.IN = IN;
  p.INp = (IN + 15) / 16 * 16;
  p.H = H;
  p.n = n;
  p.lossp = lossp;
  p.loss = loss;
  p.nlp = nlp;
  const int nt = H / 16;
  p.nb2 = (n * nt * nt + NW - 1) / NW;
  p.nb1 = (n * nt * (p.INp / 16) + NW - 1) / NW;
  hipLaunchKernelGGL(critic_wgrad_kernel, dim3(p.nb2 + p.nb1 + n * (H / 64) + (lossp && loss ? 1 : 0)), dim3(NTH), 0, st, p);
}
