// Tail of the discrete actor inside the imagination rollout, one launch per step (reference: the actor's last
// hidden block + head + OneHotCategoricalStraightThrough sample with unimix, dreamer_v3/agent.py:682-739 and
// utils/distribution.py:380-393, called once per imagined step at dreamer_v3.py:235-257):
//
//   y = act(LN(pre))                  (the trunk's last LayerNorm; y, mean, rstd recorded for the backward)
//   l[a] = y . Wh[a] + bh[a]          (the head, A <= 16 actions)
//   sample ~ Categorical(unimix(l))   (one-hot into the rollout buffer + its hot column index)
//
// was three launches per step (LayerNorm kernel, hipBLASLt GEMM with N = 9, sampler) at M = 1024 rows, each
// latency-bound (~5 us).  One wave per row: the row's N <= 1024 values stay in registers (16-byte loads), the A
// head dot products are wave reductions (DPP), and the sampler runs on the first 16-lane row of the wave with
// exactly the segment arithmetic of dist.hip's unimix_sample_fwd_kernel.
#include "common.h"

namespace srl {
namespace atail {

#define FEPS 1.1920928955078125e-07f

struct TP {
  const float* pre;
  float* y;
  const float* gamma;
  const float* beta;
  float* mean;
  float* rstd;
  const float* Wh;  // [A, N]
  const float* bh;  // [A] or null
  const float* uniform;  // [M] or null (mode)
  float* sample;    // [M, >= A] row-strided
  int* idx;         // [M, >= 1] row-strided or null
  float* logits;    // [M, A] or null
  long ldp, ldy, lds, ldi;
  int M, N, A, ioff, act;
  float eps, alpha;
};

template <int NV4, int AMAX, int ACTC>
__global__ void __launch_bounds__(256) tail_kernel(TP p) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= p.M) return;  // whole wave
  const int N4 = p.N >> 2;
  // the head rows are requested first (unconditional loads, rows past A clamped to A - 1: their dot products are
  // dropped), so their latency overlaps the row's load and the LayerNorm instead of 9 serial round trips (the
  // first version waited on each head row in turn: 11.8 us per step at M = 1024)
  float4 wv[AMAX][NV4];
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    const float4* wr = reinterpret_cast<const float4*>(p.Wh + (long)min(a, p.A - 1) * p.N);
#pragma unroll
    for (int k = 0; k < NV4; ++k) wv[a][k] = wr[min(lane + 64 * k, N4 - 1)];
  }
  // the LayerNorm parameters, this lane's head bias and the row's uniform: requested here too, so the row statistics,
  // the head and the draw below wait on no further memory latency
  float4 gv[NV4], bv4[NV4];
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    const int i4 = min(lane + 64 * k, N4 - 1);
    gv[k] = p.gamma ? reinterpret_cast<const float4*>(p.gamma)[i4] : make_float4(1.f, 1.f, 1.f, 1.f);
    bv4[k] = p.beta ? reinterpret_cast<const float4*>(p.beta)[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float bhl = (p.bh && lane < p.A) ? p.bh[lane] : 0.f;
  const float ur = p.uniform != nullptr ? p.uniform[r] : 0.f;
  const float4* xr = reinterpret_cast<const float4*>(p.pre + (long)r * p.ldp);
  float4 v[NV4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    const int i4 = lane + 64 * k;
    v[k] = i4 < N4 ? xr[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
  }
  const float mu = wave_sum_dpp(s) / p.N;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    if (lane + 64 * k < N4) {
      const float a = v[k].x - mu, b = v[k].y - mu, c = v[k].z - mu, d = v[k].w - mu;
      q += (a * a + b * b) + (c * c + d * d);
    }
  }
  const float rs = rsqrtf(wave_sum_dpp(q) / p.N + p.eps);
  float4* yr = reinterpret_cast<float4*>(p.y + (long)r * p.ldy);
#pragma unroll
  for (int k = 0; k < NV4; ++k) {
    const int i4 = lane + 64 * k;
    if (i4 < N4) {
      const float4 g = gv[k], b = bv4[k];
      float4 o;
      o.x = act_fwd_c<ACTC>((v[k].x - mu) * rs * g.x + b.x, p.act);
      o.y = act_fwd_c<ACTC>((v[k].y - mu) * rs * g.y + b.y, p.act);
      o.z = act_fwd_c<ACTC>((v[k].z - mu) * rs * g.z + b.z, p.act);
      o.w = act_fwd_c<ACTC>((v[k].w - mu) * rs * g.w + b.w, p.act);
      yr[i4] = o;
      v[k] = o;  // y stays in registers for the head
    }
  }
  if (lane == 0) {
    p.mean[r] = mu;
    p.rstd[r] = rs;
  }
  // head: lane a (< A) ends up holding l[a]
  float la = -INFINITY;
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    if (a < p.A) {  // wave-uniform
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        if (lane + 64 * k < N4) {
          const float4 w = wv[a][k];
          d += (v[k].x * w.x + v[k].y * w.y) + (v[k].z * w.z + v[k].w * w.w);
        }
      }
      const float l = wave_sum_dpp(d) + bhl;  // lane a: + bh[a]
      if (lane == a) la = l;
    }
  }
  // unimix sample on lanes 0..15 (segment width 16 >= A): dist.hip unimix_sample_fwd_kernel's arithmetic
  constexpr int W = 16;
  const int k = lane & (W - 1);
  const bool valid = lane < p.A;
  const int C = p.A;
  float m = la;
  if (p.alpha > 0.f) {
    const float mx = seg_max_f(la, W);
    const float e = valid ? __expf(la - mx) : 0.f;
    const float ssum = seg_sum_f(e, W);
    float pm = (1.f - p.alpha) * (e / ssum) + p.alpha / C;
    pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
    m = valid ? logf(pm) : -INFINITY;
  }
  const float mx2 = seg_max_f(m, W);
  const float e2 = valid ? __expf(m - mx2) : 0.f;
  const float s2 = seg_sum_f(e2, W);
  const float pr = e2 / s2;
  int pick;
  if (p.uniform != nullptr) {
    const float cdf = row16_scan(pr);
    const float u = ur;
    const float cmax = seg_max_f(cdf, W);
    const float below = (valid && cdf < u * cmax) ? 1.f : 0.f;
    pick = (int)seg_sum_f(below, W);
    if (pick > C - 1) pick = C - 1;
  } else {
    // mode: first index of the max probability
    float bv = valid ? pr : -1.f;
    int bi = k;
    for (int o = W >> 1; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    pick = bi;
  }
  if (valid) {
    p.sample[(long)r * p.lds + k] = (k == pick) ? 1.f : 0.f;
    if (p.logits) p.logits[(long)r * C + k] = la;
    if (p.idx != nullptr && k == 0) p.idx[(long)r * p.ldi] = p.ioff + pick;
  }
}

}  // namespace atail
}  // namespace srl

using namespace srl;

// false: shape not covered (A > 16, N % 4, N > 1024, misaligned rows) - the caller runs the three-launch path
bool launch_actor_tail(const float* pre, long ldp, float* y, long ldy, const float* gamma, const float* beta, float* mean,
                       float* rstd, float eps, int act, const float* Wh, const float* bh, int A, const float* uniform,
                       float alpha, float* sample, long lds, int* idx, long ldi, int ioff, float* logits, int M, int N,
                       hipStream_t st) {
  if (A < 1 || A > 16 || (N & 3) || N > 1024 || (ldp & 3) || (ldy & 3) ||
      (((uintptr_t)pre | (uintptr_t)y | (uintptr_t)Wh | (uintptr_t)gamma | (uintptr_t)beta) & 15))
    return false;
  atail::TP p;
  p.pre = pre;
  p.y = y;
  p.gamma = gamma;
  p.beta = beta;
  p.mean = mean;
  p.rstd = rstd;
  p.Wh = Wh;
  p.bh = bh;
  p.uniform = uniform;
  p.sample = sample;
  p.idx = idx;
  p.logits = logits;
  p.ldp = ldp;
  p.ldy = ldy;
  p.lds = lds;
  p.ldi = ldi;
  p.M = M;
  p.N = N;
  p.A = A;
  p.ioff = ioff;
  p.act = act;
  p.eps = eps;
  p.alpha = alpha;
  const int nv4 = cdiv(N / 4, 64);
  const dim3 grid(cdiv(M, 4));
#define F(NV, AM)                                                                                              \
  if (nv4 <= NV && A <= AM) {                                                                                  \
    SRL_ACT_SPECIALIZE(act, hipLaunchKernelGGL((atail::tail_kernel<NV, AM, ACTC>), grid, dim3(256), 0, st, p)); \
    return true;                                                                                               \
  }
  F(1, 8) F(1, 16) F(2, 8) F(2, 16) F(4, 4) F(4, 8)  // N > 512 with A > 8: too many head registers
#undef F
  return false;
}
