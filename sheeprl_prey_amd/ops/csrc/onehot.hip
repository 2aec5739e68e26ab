// One-hot input columns as row gathers (DreamerV3 latents, reference dreamer_v3/agent.py:312-455, 602-828).
//
// Every DreamerV3 latent is [z | h] with z the straight-through sample of 32 categoricals x 32 classes:
// its forward value is EXACTLY one-hot (32 ones among 1024 columns).  The first Linear of every MLP that
// reads a latent (actor trunk, critic, target critic, reward, continue, the decoder's Linear, the
// recurrent model's [z | a] input) therefore computes, for its z columns,
//     z W_z^T = sum over the 32 groups g of  W_z^T[g*32 + k_g]        (k_g = the hot class of group g)
// i.e. 32 row reads of the transposed weight instead of a K = 1024 GEMM slice: 2/3 of the K = 1536
// GEMM of a 512-unit layer.  The dense h columns stay a library GEMM (K = 512); this kernel adds the
// gathered rows to it and applies the layer's LayerNorm + activation in the same pass (one wave per row,
// the whole row in registers), writing the pre-norm value (for the backward), the row statistics and
// the activation.  Summation order differs from the dense GEMM only by fp32 rounding.
//
//   onehot_index_kernel   : one-hot rows (row-strided) -> int32 hot column per group (+ offset)
//   onehot_gather_ln_kernel: y = act(LN(Y + sum_j T[idx_j - off] + bias)) per row (LN optional)
#include "common.h"

namespace srl {
namespace onehot {

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// idx[r * ldi + g] = off + g * C + argmax_k x[r * ldx + g * C + k]   (one lane per (row, group))
__global__ void __launch_bounds__(256) onehot_index_kernel(const float* __restrict__ x, int ldx, int M, int G, int C,
                                                           int* __restrict__ idx, int ldi, int off) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= M * G) return;
  const int r = t / G, g = t - r * G;
  const float* p = x + (int64_t)r * ldx + g * C;
  int best = 0;
  float bv = p[0];
  for (int k = 1; k < C; ++k) {
    const float v = p[k];
    if (v > bv) {
      bv = v;
      best = k;
    }
  }
  idx[(int64_t)r * ldi + g] = off + g * C + best;
}

// y = act(LN(acc)) for one wave's float4 columns c4 + lane + 64 v (ACTC: common.h SRL_ACT_SPECIALIZE)
// (gp / bp: this lane's LayerNorm parameters, loaded in the kernel prologue)
template <int NV4, int ACTC>
__device__ __forceinline__ void store_rows(const f4 (&acc)[NV4], int c4, int lane, int N4, int ln, float mu, float rs,
                                           const f4 (&gp)[NV4], const f4 (&bp)[NV4], int act, float* yrow) {
#pragma unroll
  for (int v = 0; v < NV4; ++v) {
    const int i4 = c4 + lane + 64 * v;
    if (i4 < N4) {
      f4 o = acc[v];
      if (ln) o = (o - mu) * rs * gp[v] + bp[v];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act_fwd_c<ACTC>(o[e], act);
      reinterpret_cast<f4*>(yrow)[i4] = o;
    }
  }
}

// WPR waves per row (4 / WPR rows per 256-thread block); wave part p of a row owns float4 columns
// p * 64 * NV4 + l + 64 v (v < NV4): N <= 256 * NV4 * WPR.  WPR = 2 at the 512-wide rollout layers (M = B*T =
// 1024 rows): each lane keeps 16 table rows in flight instead of 8, so the 32 gathers of a row take two L2 round
// trips instead of four (this kernel is latency-bound at that size: ~10 us per call with one wave per row).
template <int NV4, int WPR>
__global__ void __launch_bounds__(256) onehot_gather_ln_kernel(
    const float* __restrict__ Y, int ldy, const int* __restrict__ idx, int ldi, int G, int off,
    const float* __restrict__ T, int K, const float* __restrict__ bias, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int act, int ln, float* __restrict__ z_out, int ldz,
    float* __restrict__ y_out, int ldo, float* __restrict__ mean_out, float* __restrict__ rstd_out, int M, int N,
    int* __restrict__ err, const float* __restrict__ xa, int ldxa, int nA, const float* __restrict__ Wa) {
  static_assert(WPR == 1 || WPR == 2 || WPR == 4, "onehot_gather_ln: 1, 2 or 4 waves per row");
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, part = wave % WPR;
  const int r = blockIdx.x * (4 / WPR) + wave / WPR;
  const bool live = r < M;  // (no early return: the WPR = 2 row reduction joins the block)
  const int N4 = N >> 2, c4 = part * 64 * NV4;
  f4 acc[NV4], gp[NV4], bp[NV4];
#pragma unroll
  for (int v = 0; v < NV4; ++v) {
    const int i4 = c4 + lane + 64 * v;
    // the LayerNorm parameters are requested with the first loads: used only after the gathers and the row
    // reductions, they no longer add a memory latency at the end of the kernel
    const bool pv = ln && live && i4 < N4;
    gp[v] = (pv && gamma) ? reinterpret_cast<const f4*>(gamma)[i4] : f4{1.f, 1.f, 1.f, 1.f};
    bp[v] = (pv && beta) ? reinterpret_cast<const f4*>(beta)[i4] : zero4();
    acc[v] = (live && Y != nullptr && i4 < N4) ? reinterpret_cast<const f4*>(Y + (int64_t)r * ldy)[i4] : zero4();
    if (live && bias != nullptr && i4 < N4) acc[v] += reinterpret_cast<const f4*>(bias)[i4];
  }
  // dense columns of the layer's input (the action part of the recurrent input: nA <= 64 small products per
  // element, in place of a K = nA library GEMM launch): acc += sum_a xa[r, a] Wa[a, :]
  for (int a = 0; a < nA; ++a) {
    const float w = live ? xa[(int64_t)r * ldxa + a] : 0.f;
#pragma unroll
    for (int v = 0; v < NV4; ++v) {
      const int i4 = c4 + lane + 64 * v;
      if (i4 < N4) acc[v] += w * reinterpret_cast<const f4*>(Wa + (int64_t)a * N)[i4];
    }
  }
  const int* ir = idx + (int64_t)(live ? r : 0) * ldi;
  // the row's hot indices: lanes < G load one each, then broadcast (wave-uniform loop below)
  int my = (live && lane < G) ? ir[lane] - off : -1;
  if (live && lane < G && (my < 0 || my >= K)) {  // a caller bug: skip the row read, report it
    if (err) atomicOr(err, 1);
    my = -1;
  }
  // QB table rows in flight per lane at a time (QB * NV4 = 16 float4 temporaries)
  constexpr int QB = NV4 <= 1 ? 16 : (NV4 <= 2 ? 8 : 16 / NV4);
  for (int j = 0; j < G; j += QB) {
    f4 t[QB][NV4];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int row = __shfl(my, j + q, 64);
      const bool ok = (j + q < G) && row >= 0;
      const f4* src = reinterpret_cast<const f4*>(T + (int64_t)(ok ? row : 0) * N);
#pragma unroll
      for (int v = 0; v < NV4; ++v) {
        const int i4 = c4 + lane + 64 * v;
        t[q][v] = (ok && i4 < N4) ? src[i4] : zero4();
      }
    }
#pragma unroll
    for (int q = 0; q < QB; ++q)
#pragma unroll
      for (int v = 0; v < NV4; ++v) acc[v] += t[q][v];
  }
  if (live && z_out != nullptr) {
#pragma unroll
    for (int v = 0; v < NV4; ++v) {
      const int i4 = c4 + lane + 64 * v;
      if (i4 < N4) reinterpret_cast<f4*>(z_out + (int64_t)r * ldz)[i4] = acc[v];
    }
  }
  float mu = 0.f, rs = 1.f;
  if (ln) {  // (ln is a kernel argument: uniform over the block)
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NV4; ++v) s += (acc[v][0] + acc[v][1]) + (acc[v][2] + acc[v][3]);
    s = wave_sum_dpp(s);
    if (WPR == 2) {
      if (lane == 0) red[0][wave] = s;
      __syncthreads();
      s = red[0][wave & ~1] + red[0][wave | 1];
    } else if (WPR == 4) {
      if (lane == 0) red[0][wave] = s;
      __syncthreads();
      s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    }
    mu = s / N;
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < NV4; ++v) {
      if (c4 + lane + 64 * v < N4) {
        const f4 d = acc[v] - mu;
        q += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
      }
    }
    q = wave_sum_dpp(q);
    if (WPR == 2) {
      if (lane == 0) red[1][wave] = q;
      __syncthreads();
      q = red[1][wave & ~1] + red[1][wave | 1];
    } else if (WPR == 4) {
      if (lane == 0) red[1][wave] = q;
      __syncthreads();
      q = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
    rs = rsqrtf(q / N + eps);
    if (live && lane == 0 && part == 0) {
      if (mean_out) mean_out[r] = mu;
      if (rstd_out) rstd_out[r] = rs;
    }
  }
  if (!live) return;
  SRL_ACT_SPECIALIZE(act, store_rows<NV4, ACTC>(acc, c4, lane, N4, ln, mu, rs, gp, bp, act, y_out + (int64_t)r * ldo));
}

}  // namespace onehot
}  // namespace srl

void launch_onehot_index(const float* x, int ldx, int M, int G, int C, int* idx, int ldi, int off, hipStream_t st) {
  const int n = M * G;
  if (n > 0) hipLaunchKernelGGL(srl::onehot::onehot_index_kernel, dim3((n + 255) / 256), dim3(256), 0, st, x, ldx, M, G, C, idx, ldi, off);
}

bool launch_onehot_gather_ln(const float* Y, int ldy, const int* idx, int ldi, int G, int off, const float* T, int K,
                             const float* bias, const float* gamma, const float* beta, float eps, int act, int ln,
                             float* z_out, int ldz, float* y_out, int ldo, float* mean, float* rstd, int M, int N, int* err,
                             hipStream_t st, const float* xa, int ldxa, int nA, const float* Wa) {
  if (nA < 0 || nA > 64 || (nA > 0 && (xa == nullptr || Wa == nullptr))) return false;
  if (N % 4 != 0 || N > 4096 || G > 64 || M <= 0) return false;
  const int nv = (N + 255) / 256;
  const dim3 block(256);
  if (nv == 2 && M <= 4096) {  // latency-bound rollout sizes: two waves per 512-wide row
    hipLaunchKernelGGL((srl::onehot::onehot_gather_ln_kernel<1, 2>), dim3((M + 1) / 2), block, 0, st, Y, ldy, idx, ldi, G, off,
                       T, K, bias, gamma, beta, eps, act, ln, z_out, ldz, y_out, ldo, mean, rstd, M, N, err, xa, ldxa, nA, Wa);
    return true;
  }
  if (nv == 4 && M <= 16384) {  // 1024-wide rows (exp=dreamer_v3_prey, dense 1024): four waves per row, 2 L2 round trips
    hipLaunchKernelGGL((srl::onehot::onehot_gather_ln_kernel<1, 4>), dim3(M), block, 0, st, Y, ldy, idx, ldi, G, off,
                       T, K, bias, gamma, beta, eps, act, ln, z_out, ldz, y_out, ldo, mean, rstd, M, N, err, xa, ldxa, nA, Wa);
    return true;
  }
  const dim3 grid((M + 3) / 4);
#define OG(NV)                                                                                                          \
  if (nv <= NV) {                                                                                                       \
    hipLaunchKernelGGL((srl::onehot::onehot_gather_ln_kernel<NV, 1>), grid, block, 0, st, Y, ldy, idx, ldi, G, off, T, K, \
                       bias, gamma, beta, eps, act, ln, z_out, ldz, y_out, ldo, mean, rstd, M, N, err, xa, ldxa, nA, Wa); \
    return true;                                                                                                        \
  }
  OG(1) OG(2) OG(4) OG(8) OG(16)
#undef OG
  return false;
}
