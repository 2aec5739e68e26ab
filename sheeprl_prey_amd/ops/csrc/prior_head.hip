// Prior (transition) head of the DreamerV3 imagination step in ONE launch (reference: RSSM._transition ->
// transition_model MLP -> _uniform_mix -> OneHotCategoricalStraightThrough sample, dreamer_v3/agent.py:439-455
// and utils/distribution.py:380-393, once per imagined step at dreamer_v3.py:235-257):
//
//   y = act(LN(x))                      x: the transition's first-layer pre-activations [M, K] (row-strided: a
//                                       column block of the rollout's merged h_{t+1} GEMM output)
//   l = y W^T + b                       W [N, K], N = G categoricals x 32 classes
//   sample ~ Categorical(unimix(l))     one-hot rows into the rollout buffer + each categorical's hot column
//
// was three launches per step (LayerNorm, hipBLASLt GEMM + bias, sampler) on the rollout's critical path.  The
// imagination is no-grad (the discrete objective never back-propagates through the dynamics), so neither y nor
// the logits are stored.
//
// Tiling: one workgroup = 16 rows x 256 logit columns (8 waves; wave w = ONE categorical group of 32 classes = two
// 16-column MFMA tiles), grid (M / 16, N / 256) = 256 workgroups at M = 1024 (one per CU).  The 16 x K row tile
// is staged in LDS once and LayerNorm-ed in place (each of the N / 256 column workgroups of a row tile repeats
// the row statistics: 16 rows, trivial).  B fragments (W rows) stream from L2 (W = 2 MB stays resident in each
// XCD's L2) through a double-buffered register batch of UK chunks; v_mfma_f32_16x16x4_f32 with the
// float4-permuted K order of scan_dev.h (a[j] / b[j] = K index 16c + 4g + j on both operands).  The accumulator
// map (col = lane & 15, row = 4 (lane >> 4) + r) puts a row's 32 classes on the 16 lanes of one DPP row x two
// registers, so the unimix / softmax / CDF of the sampler are DPP row reductions with no LDS round trip.
#include "common.h"
#include "scan_dev.h"

namespace srl {
namespace phead {

using scandev::f4;

constexpr int NT = 512;  // 8 waves
constexpr int CL = 32;   // classes per categorical
constexpr int UK = 8;    // 16-wide K chunks of B fragments per register batch

struct HP {
  const float* x;
  long ldx;
  const float* gamma;
  const float* beta;
  const float* W;  // [N, K]
  const float* b;  // [N] or null
  const float* uni;  // [M * G]: uniform of (row m, categorical g) at m * G + g
  float* sample;     // [M, >= N] row-strided
  long lds;
  int* idx;          // [M, >= G] row-strided or null: ioff + g * 32 + pick
  long ldi;
  int ioff, M, K, N, act;
  float eps, alpha;
  // optional saved forward state for a backward through the head (continuous imagination, imagine_cont.py):
  float* logits;     // [M, >= N] row-strided pre-unimix logits, or null
  long ldl;
  float* mean_out;   // [M] LayerNorm row statistics of x, or null
  float* rstd_out;
};

// 16-lane (DPP row) reductions / scan: no LDS-crossbar shuffles (common.h row16_*); the row's last lane by readlanes
__device__ __forceinline__ float row16_last(float v) {
  const float a = lane_f(v, 15), b = lane_f(v, 31), c = lane_f(v, 47), d = lane_f(v, 63);
  const int r = (threadIdx.x >> 4) & 3;
  return r == 0 ? a : (r == 1 ? b : (r == 2 ? c : d));
}

// LayerNorm + act of one LDS row of K = 64 KV with this lane's gamma / beta columns (s + 64 m) already in registers
// (scan_dev.h wave_ln_act_row reads them from global memory after the row reductions: one more memory latency per
// row on the kernel's serial prologue); same arithmetic
template <int KV, int ACTC>
__device__ __forceinline__ void ln_act_row_regs(float* r, int N, float eps, const float (&gm)[KV], const float (&bt)[KV],
                                                int act, float& mu, float& rs) {
  const int s = threadIdx.x & 63;  // N = 64 KV (runtime value: the same division as wave_ln_act_row)
  float v[KV];
  float a = 0.f;
#pragma unroll
  for (int m = 0; m < KV; ++m) {
    v[m] = r[s + 64 * m];
    a += v[m];
  }
  mu = wave_sum_dpp(a) / N;
  float q = 0.f;
#pragma unroll
  for (int m = 0; m < KV; ++m) {
    const float d = v[m] - mu;
    q += d * d;
  }
  rs = rsqrtf(wave_sum_dpp(q) / N + eps);
#pragma unroll
  for (int m = 0; m < KV; ++m) r[s + 64 * m] = scandev::f_act_c<ACTC>((v[m] - mu) * rs * gm[m] + bt[m], act);
}

template <int KV>
__global__ void __launch_bounds__(NT) prior_head_kernel(HP p) {
  extern __shared__ float sm[];
  const int lda = p.K + 4;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * 16;
  const int nrow = min(16, p.M - r0);
  const int G = p.N / CL;
  const int gg = blockIdx.y * 8 + w;  // this wave's categorical
  const int n0 = gg * CL;
  // first B batch requested before anything else: its latency hides behind the staging and the LayerNorm
  const float* wr0 = p.W + (long)(n0 + i) * p.K + 4 * g;
  const float* wr1 = wr0 + 16L * p.K;
  f4 cb0[UK], cb1[UK];
#pragma unroll
  for (int q = 0; q < UK; ++q) {
    cb0[q] = *(const f4*)(wr0 + 16 * q);
    cb1[q] = *(const f4*)(wr1 + 16 * q);
  }
  const float bb0 = p.b ? p.b[n0 + i] : 0.f, bb1 = p.b ? p.b[n0 + 16 + i] : 0.f;
  // everything else the prologue and the sampler read from global memory is requested here too, so the serial
  // part of the kernel (stage -> LayerNorm -> K loop -> sample) waits on one memory latency, not one per use:
  // the LN parameters of this lane's columns and the uniforms of this lane's four (row, categorical) draws
  float gm[KV], bt[KV];
#pragma unroll
  for (int m = 0; m < KV; ++m) {
    gm[m] = p.gamma[lane + 64 * m];
    bt[m] = p.beta[lane + 64 * m];
  }
  float un[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) un[r] = 4 * g + r < nrow ? p.uni[(long)(r0 + 4 * g + r) * G + gg] : 0.f;
  // 16 x K row tile -> LDS (rows past M zero; all of a thread's loads in flight together), then LayerNorm + act in
  // place (two rows per wave)
  constexpr int C4 = 16 * KV, PER = 16 * C4 / NT;  // K / 4 float4 per row; float4 per thread
  static_assert(PER * NT == 16 * C4, "row tile per thread");
  f4 xv[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + j * NT, r = e / C4, k = (e - r * C4) << 2;
    xv[j] = r < nrow ? *(const f4*)(p.x + (long)(r0 + r) * p.ldx + k) : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = threadIdx.x + j * NT, r = e / C4, k = (e - r * C4) << 2;
    *(f4*)(sm + r * lda + k) = xv[j];
  }
  __syncthreads();
  for (int r = w; r < 16; r += NT / 64) {
    float mu, rs;
    SRL_ACT_SPECIALIZE(p.act, (ln_act_row_regs<KV, ACTC>(sm + r * lda, p.K, p.eps, gm, bt, p.act, mu, rs)));
    if (p.mean_out != nullptr && blockIdx.y == 0 && lane == 0 && r < nrow) {
      p.mean_out[r0 + r] = mu;
      p.rstd_out[r0 + r] = rs;
    }
  }
  __syncthreads();
  // logits tile [16 rows x 32 classes] of this wave's categorical.  K = 64 * KV exactly (compile-time trip count,
  // fully unrolled) and every B load unconditional (the last batch re-reads itself): an exec-masked or branched
  // load makes the wait-count pass drain vmcnt before the next batch, serialising load latency with the MFMAs
  // (the conv.hip main-loop lesson)
  const float* arow = sm + i * lda + 4 * g;
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  constexpr int NCH = 4 * KV;
  static_assert(NCH % UK == 0, "K chunks per batch");
#pragma unroll
  for (int c0 = 0; c0 < NCH; c0 += UK) {
    f4 nb0[UK], nb1[UK];
    const int cn = c0 + UK < NCH ? c0 + UK : c0;
#pragma unroll
    for (int q = 0; q < UK; ++q) {
      nb0[q] = *(const f4*)(wr0 + 16 * (cn + q));
      nb1[q] = *(const f4*)(wr1 + 16 * (cn + q));
    }
#pragma unroll
    for (int q = 0; q < UK; ++q) {
      const f4 a = *(const f4*)(arow + 16 * (c0 + q));
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], cb0[q][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], cb1[q][0], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], cb0[q][1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], cb1[q][1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], cb0[q][2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], cb1[q][2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], cb0[q][3], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], cb1[q][3], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < UK; ++q) {
      cb0[q] = nb0[q];
      cb1[q] = nb1[q];
    }
  }
  // unimix + categorical sample per (row, categorical): class j on lane i of register 0, class 16 + j on register 1
  const float inv = 1.f / CL;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * g + r;
    const float l0 = acc0[r] + bb0, l1 = acc1[r] + bb1;
    if (p.logits != nullptr && row < nrow) {
      float* lrow = p.logits + (long)(r0 + row) * p.ldl + n0;
      lrow[i] = l0;
      lrow[16 + i] = l1;
    }
    float m0 = l0, m1 = l1;
    if (p.alpha > 0.f) {
      const float mx = row16_max(fmaxf(l0, l1));
      const float e0 = __expf(l0 - mx), e1 = __expf(l1 - mx);
      const float s = row16_sum(e0 + e1);
      float q0 = (1.f - p.alpha) * (e0 / s) + p.alpha * inv;
      float q1 = (1.f - p.alpha) * (e1 / s) + p.alpha * inv;
      q0 = fminf(fmaxf(q0, FEPS), 1.f - FEPS);
      q1 = fminf(fmaxf(q1, FEPS), 1.f - FEPS);
      m0 = logf(q0);
      m1 = logf(q1);
    }
    const float mx2 = row16_max(fmaxf(m0, m1));
    const float e0 = __expf(m0 - mx2), e1 = __expf(m1 - mx2);
    const float s2 = row16_sum(e0 + e1);
    const float cdf0 = row16_scan(e0 / s2);
    const float cdf1 = row16_last(cdf0) + row16_scan(e1 / s2);
    const float cmax = row16_last(cdf1);
    const float thr = un[r] * cmax;
    int pick = (int)row16_sum((cdf0 < thr ? 1.f : 0.f) + (cdf1 < thr ? 1.f : 0.f));
    if (pick > CL - 1) pick = CL - 1;
    if (row < nrow) {
      float* srow = p.sample + (long)(r0 + row) * p.lds + n0;
      srow[i] = i == pick ? 1.f : 0.f;
      srow[16 + i] = 16 + i == pick ? 1.f : 0.f;
      if (p.idx != nullptr && i == 0) p.idx[(long)(r0 + row) * p.ldi + gg] = p.ioff + n0 + pick;
    }
  }
}

}  // namespace phead
}  // namespace srl

// false: shape not covered (caller runs the three-launch path)
bool launch_prior_head(const float* x, long ldx, const float* gamma, const float* beta, float eps, int act, const float* W,
                       const float* b, const float* uni, float alpha, float* sample, long lds, int* idx, long ldi, int ioff,
                       int M, int K, int N, hipStream_t st, float* logits, long ldl, float* mean_out, float* rstd_out) {
  using namespace srl::phead;
  if (M <= 0 || (K != 256 && K != 512 && K != 1024) || N % 256 != 0 || ldx % 4 != 0 || !gamma || !beta) return false;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W)) & 15) return false;
  if ((mean_out == nullptr) != (rstd_out == nullptr)) return false;
  HP p{x, ldx, gamma, beta, W, b, uni, sample, lds, idx, ldi, ioff, M, K, N, act, eps, alpha, logits, ldl, mean_out, rstd_out};
  const dim3 grid((M + 15) / 16, N / 256);
  const size_t shm = (size_t)16 * (K + 4) * sizeof(float);
  static const bool lds_set = [] {  // K = 1024 needs 65.8 KB of the 160 KB
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(prior_head_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              16 * 260 * 4);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(prior_head_kernel<8>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              16 * 516 * 4);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(prior_head_kernel<16>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              16 * 1028 * 4);
    return true;
  }();
  (void)lds_set;
  if (K == 256)
    hipLaunchKernelGGL(prior_head_kernel<4>, grid, dim3(NT), shm, st, p);
  else if (K == 512)
    hipLaunchKernelGGL(prior_head_kernel<8>, grid, dim3(NT), shm, st, p);
  else
    hipLaunchKernelGGL(prior_head_kernel<16>, grid, dim3(NT), shm, st, p);
  return true;
}
