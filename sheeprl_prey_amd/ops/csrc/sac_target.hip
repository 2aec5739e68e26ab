// Fused SAC twin-Q target (reference sac/agent.py:256-275, sac/sac.py:36-52):
//
//   q_c   = w3_c . relu(W2_c relu(W1_c [obs, act] + b1_c) + b2_c) + b3_c        c = 0..n-1
//   y     = r + (1 - done) * gamma * (min_c q_c - exp(log_alpha) * logp)
//
// One workgroup per 16 batch rows evaluates every target critic of the ensemble (stacked weights
// [n, out, in], models/ensemble.py) and writes y directly: the concatenation, 3 n GEMM layers,
// the ReLUs, the min over critics and the entropy-regularised Bellman target in ONE launch instead
// of ~10 (no autograd: the target path runs under no_grad).
//
// 8 waves per workgroup; layer l output columns are split into 16-wide MFMA tiles across the waves
// (H / 128 tiles per wave).  Activations (x, h1) live in LDS; weights are read from L2 with one
// 64-byte float4 row segment per lane and a permuted K order (lane (j, q) of MFMA e takes
// k = k0 + 4q + e for both operands), so no operand shuffles are needed.  fp32 MFMA 16x16x4.
#include "common.h"

namespace srl {
namespace sactgt {

constexpr int NTH = 512;
constexpr int NW = NTH / 64;
constexpr int ROWS = 16;
constexpr int MAXC = 4;

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct TP {
  const float* obs;
  const float* act;
  const float* logp;
  const float* rew;
  const float* done;
  const float* log_alpha;
  const float* W1;  // [n, H, IN]
  const float* b1;  // [n, H]
  const float* W2;  // [n, H, H]
  const float* b2;  // [n, H]
  const float* W3;  // [n, 1, H]
  const float* b3;  // [n, 1]
  float* y;         // [M, 1]
  int M, OD, AD, IN, INp, H, n;
  float gamma;
};

__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

// acc (16 rows x 16 cols of tile starting at weight row n0) += act[16][K] . W[n0.., K]^T
// act: LDS, row stride lda (floats); W global row-major with row stride ldw.  K % 16 == 0.  The weight
// loads of KC K-steps are issued before the MFMAs that use them (one L2 latency per chunk).
constexpr int KC = 8;
__device__ __forceinline__ floatx4 tile_gemm(const float* act, int lda, const float* W, int ldw, int n0, int K, int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* wr = W + (long)(n0 + j) * ldw + 4 * q;
  const float* ar = act + j * lda + 4 * q;
  for (int kb = 0; kb < K; kb += 16 * KC) {
    float4 w[KC];
#pragma unroll
    for (int u = 0; u < KC; ++u)
      if (kb + 16 * u < K) w[u] = *reinterpret_cast<const float4*>(wr + kb + 16 * u);
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (kb + 16 * u < K) {
        const float4 a = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), comp(w[u], e), acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

__global__ __launch_bounds__(NTH) void sac_target_kernel(TP p) {
  extern __shared__ float sm[];
  const int ldx = p.INp + 4, ldh = p.H + 4;
  float* xs = sm;                    // [16][INp + 4]
  float* hs = xs + ROWS * ldx;       // [16][H + 4]
  float* qp = hs + ROWS * ldh;       // [NW][16] per-wave partial q
  float* qmin = qp + NW * ROWS;      // [16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * ROWS;
  for (int i = tid; i < ROWS * p.INp; i += NTH) {  // x = [obs, act], zero padded (rows and columns)
    const int r = i / p.INp, c = i - r * p.INp, row = r0 + r;
    float v = 0.f;
    if (row < p.M) v = c < p.OD ? p.obs[(long)row * p.OD + c] : (c < p.IN ? p.act[(long)row * p.AD + c - p.OD] : 0.f);
    xs[r * ldx + c] = v;
  }
  if (tid < ROWS) qmin[tid] = INFINITY;
  const int tiles = p.H / (16 * NW);  // 16-column tiles per wave
  const int j = lane & 15, q = lane >> 4;
  for (int c = 0; c < p.n; ++c) {
    __syncthreads();  // xs ready / previous critic's hs consumers done
    const float* W1 = p.W1 + (long)c * p.H * p.IN;
    for (int t = 0; t < tiles; ++t) {
      const int n0 = (wave * tiles + t) * 16;
      // layer 1 reads W1 rows of length IN (not padded): stage through the padded-K loop only when
      // IN % 16 == 0; otherwise a guarded scalar path (IN is small: obs + action dims)
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      if ((p.IN & 15) == 0) {
        acc = tile_gemm(xs, ldx, W1, p.IN, n0, p.IN, lane);
      } else {
        for (int k0 = 0; k0 < p.INp; k0 += 4) {
          const int k = k0 + q;
          const float w = k < p.IN ? W1[(long)(n0 + j) * p.IN + k] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[j * ldx + k], w, acc, 0, 0, 0);
        }
      }
      const float bb = p.b1[c * p.H + n0 + j];
#pragma unroll
      for (int e = 0; e < 4; ++e) hs[(4 * q + e) * ldh + n0 + j] = fmaxf(acc[e] + bb, 0.f);
    }
    __syncthreads();
    const float* W2 = p.W2 + (long)c * p.H * p.H;
    float part[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < tiles; ++t) {
      const int n0 = (wave * tiles + t) * 16;
      const floatx4 acc = tile_gemm(hs, ldh, W2, p.H, n0, p.H, lane);
      const float bb = p.b2[c * p.H + n0 + j], w3 = p.W3[c * p.H + n0 + j];
#pragma unroll
      for (int e = 0; e < 4; ++e) part[e] += fmaxf(acc[e] + bb, 0.f) * w3;
    }
    // sum over the 16 columns held by lanes j = 0..15 (same q), then over waves
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = part[e];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (j == 0) qp[wave * ROWS + 4 * q + e] = v;
    }
    __syncthreads();
    if (tid < ROWS) {
      float s = p.b3[c];
      for (int w = 0; w < NW; ++w) s += qp[w * ROWS + tid];
      qmin[tid] = fminf(qmin[tid], s);
    }
  }
  __syncthreads();
  if (tid < ROWS && r0 + tid < p.M) {
    const int row = r0 + tid;
    const float alpha = __expf(*p.log_alpha);
    p.y[row] = p.rew[row] + (1.f - p.done[row]) * p.gamma * (qmin[tid] - alpha * p.logp[row]);
  }
}

}  // namespace sactgt
}  // namespace srl

size_t sac_target_lds(int INp, int H) {
  return sizeof(float) * (16 * (size_t)(INp + 4) + 16 * (size_t)(H + 4) + srl::sactgt::NW * 16 + 16);
}

void launch_sac_target(const float* obs, const float* act, const float* logp, const float* rew, const float* done,
                       const float* log_alpha, const float* W1, const float* b1, const float* W2, const float* b2,
                       const float* W3, const float* b3, float* y, int M, int OD, int AD, int H, int n, float gamma,
                       hipStream_t st) {
  srl::sactgt::TP p;
  p.obs = obs;
  p.act = act;
  p.logp = logp;
  p.rew = rew;
  p.done = done;
  p.log_alpha = log_alpha;
  p.W1 = W1;
  p.b1 = b1;
  p.W2 = W2;
  p.b2 = b2;
  p.W3 = W3;
  p.b3 = b3;
  p.y = y;
  p.M = M;
  p.OD = OD;
  p.AD = AD;
  p.IN = OD + AD;
  p.INp = (p.IN + 15) / 16 * 16;
  p.H = H;
  p.n = n;
  p.gamma = gamma;
  hipLaunchKernelGGL(srl::sactgt::sac_target_kernel, dim3((M + 15) / 16), dim3(srl::sactgt::NTH), sac_target_lds(p.INp, H),
                     st, p);
}
