// Distribution-head kernels for the world-model / actor-critic losses (fp32):
//  * unimix + straight-through one-hot sampling (reference RSSM._uniform_mix + compute_stochastic_state,
//    dreamer_v3/agent.py:390-437; OneHotCategoricalStraightThrough, utils/distribution.py:380-393)
//  * two-hot symlog NLL and two-hot mean (TwoHotEncodingDistribution, utils/distribution.py:224-270)
//  * categorical KL summed over groups (dreamer_v3/loss.py:65-110)
// Categorical rows are mapped onto aligned lane segments of W = next_pow2(C) <= 64 lanes, so a
// wave64 processes 64/W groups at once and every reduction is a segmented xor-shuffle.
#include "common.h"

#include <cstdlib>

namespace srl {

__device__ __forceinline__ float seg_prefix_sum(float v, int width, int lane_in_seg) {
  if (width == 32) return seg32_scan(v);  // DPP forms (common.h): no LDS-crossbar round trips
  if (width == 16) return row16_scan(v);
  for (int o = 1; o < width; o <<= 1) {
    float t = __shfl_up(v, o, width);
    if (lane_in_seg >= o) v += t;
  }
  return v;
}

// argmax (first index on ties) over a segment
__device__ __forceinline__ int seg_argmax(float v, int idx, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) {
    float ov = __shfl_xor(v, o, SRL_WAVE);
    int oi = __shfl_xor(idx, o, SRL_WAVE);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  return idx;
}

#define FEPS 1.1920928955078125e-07f

// One segment = one categorical of C classes.  uniform == nullptr -> mode (argmax).
__global__ void __launch_bounds__(256) unimix_sample_fwd_kernel(const float* __restrict__ logits,
                                                                const float* __restrict__ uniform,
                                                                float* __restrict__ mixed, float* __restrict__ sample,
                                                                int R, int C, int W, float alpha, int G, int lds,
                                                                int* __restrict__ idx, int ldi, int ioff) {
  const int lane = threadIdx.x & 63;
  const int seg_per_wave = 64 / W;
  const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int r = gwave * seg_per_wave + lane / W;
  const int k = lane % W;
  const bool row_ok = r < R;
  const bool valid = row_ok && k < C;
  const int64_t off = (int64_t)r * C + k;
  float l = valid ? logits[off] : -INFINITY;
  float m = l;
  if (alpha > 0.f) {
    float mx = seg_max_f(l, W);
    float e = valid ? __expf(l - mx) : 0.f;
    float s = seg_sum_f(e, W);
    float q = e / s;
    float pm = (1.f - alpha) * q + alpha / C;
    pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
    m = valid ? logf(pm) : -INFINITY;
  }
  // probabilities of Categorical(logits=m)
  float mx2 = seg_max_f(m, W);
  float e2 = valid ? __expf(m - mx2) : 0.f;
  float s2 = seg_sum_f(e2, W);
  float p = e2 / s2;
  int pick;
  if (uniform != nullptr) {
    float cdf = seg_prefix_sum(p, W, k);
    float u = row_ok ? uniform[r] : 0.f;
    // every cross-lane reduction runs with the whole wave active: a DPP operand from a lane masked off by
    // a divergent branch (e.g. the short-circuit of `valid && ...`) reads 0, not the lane's value
    const float cmax = seg_max_f(cdf, W);
    float below = (valid && cdf < u * cmax) ? 1.f : 0.f;
    pick = (int)seg_sum_f(below, W);
    if (pick > C - 1) pick = C - 1;
  } else {
    pick = seg_argmax(valid ? p : -1.f, k, W);
  }
  if (valid) {
    if (mixed) mixed[off] = m;
    // sample rows may be strided: G categoricals per row, row stride lds (G*C when contiguous)
    const int64_t so = (int64_t)(r / G) * lds + (int64_t)(r % G) * C + k;
    sample[so] = (k == pick) ? 1.f : 0.f;
    // optional hot-column index of the sample (ops/csrc/onehot.hip consumers): ioff + g * C + pick
    if (idx != nullptr && k == 0) idx[(int64_t)(r / G) * ldi + (r % G)] = ioff + (r % G) * C + pick;
  }
}

// d(loss)/d(logits) given g_mixed (may be null) and g_sample (straight-through path, may be null)
__global__ void __launch_bounds__(256) unimix_sample_bwd_kernel(const float* __restrict__ logits,
                                                                const float* __restrict__ g_mixed,
                                                                const float* __restrict__ g_sample,
                                                                float* __restrict__ dlogits, int R, int C, int W,
                                                                float alpha) {
  const int lane = threadIdx.x & 63;
  const int seg_per_wave = 64 / W;
  const int gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int r = gwave * seg_per_wave + lane / W;
  const int k = lane % W;
  const bool valid = r < R && k < C;
  const int64_t off = (int64_t)r * C + k;
  float l = valid ? logits[off] : -INFINITY;
  float q = 0.f, pm = 0.f, m = l;
  bool clamped = false;
  if (alpha > 0.f) {
    float mx = seg_max_f(l, W);
    float e = valid ? __expf(l - mx) : 0.f;
    float s = seg_sum_f(e, W);
    q = e / s;
    pm = (1.f - alpha) * q + alpha / C;
    clamped = pm <= FEPS || pm >= 1.f - FEPS;
    m = valid ? logf(fminf(fmaxf(pm, FEPS), 1.f - FEPS)) : -INFINITY;
  }
  float gm = (valid && g_mixed) ? g_mixed[off] : 0.f;
  if (g_sample) {
    float mx2 = seg_max_f(m, W);
    float e2 = valid ? __expf(m - mx2) : 0.f;
    float p = e2 / seg_sum_f(e2, W);
    float gs = valid ? g_sample[off] : 0.f;
    float dot = seg_sum_f(p * gs, W);
    gm += p * (gs - dot);
  }
  float dl;
  if (alpha > 0.f) {
    float w = (valid && !clamped) ? (1.f - alpha) * gm / pm : 0.f;
    float dot = seg_sum_f(q * w, W);
    dl = q * (w - dot);
  } else {
    dl = gm;
  }
  if (valid) dlogits[off] = dl;
}

// ---------------------------------------------------------------- wide categoricals (64 < C <= 64 V)
// One wave per categorical (the fork's prey_d_1 actor has Discrete(100)): lane l holds classes l + 64 v.  Same
// arithmetic as the segment form above; the sampler's CDF is each 64-class chunk's wave scan plus the running total
// of the chunks before it.
template <int V>
__global__ void __launch_bounds__(256) unimix_sample_wide_fwd_kernel(const float* __restrict__ logits,
                                                                     const float* __restrict__ uniform,
                                                                     float* __restrict__ mixed, float* __restrict__ sample,
                                                                     int R, int C, float alpha, int G, int lds,
                                                                     int* __restrict__ idx, int ldi, int ioff) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;  // wave-uniform
  const float* lr = logits + (int64_t)r * C;
  float l[V], m[V];
  bool ok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int k = lane + 64 * v;
    ok[v] = k < C;
    const float x = lr[k < C ? k : C - 1];  // unconditional (clamped) load
    l[v] = ok[v] ? x : -INFINITY;
    m[v] = l[v];
  }
  if (alpha > 0.f) {
    float mx = -INFINITY;
#pragma unroll
    for (int v = 0; v < V; ++v) mx = fmaxf(mx, l[v]);
    mx = seg_max_f(mx, 64);
    float e[V], s = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      e[v] = ok[v] ? __expf(l[v] - mx) : 0.f;
      s += e[v];
    }
    s = seg_sum_f(s, 64);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float pm = (1.f - alpha) * (e[v] / s) + alpha / C;
      pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
      m[v] = ok[v] ? logf(pm) : -INFINITY;
    }
  }
  float mx2 = -INFINITY;
#pragma unroll
  for (int v = 0; v < V; ++v) mx2 = fmaxf(mx2, m[v]);
  mx2 = seg_max_f(mx2, 64);
  float p[V], s2 = 0.f;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    p[v] = ok[v] ? __expf(m[v] - mx2) : 0.f;
    s2 += p[v];
  }
  s2 = seg_sum_f(s2, 64);
#pragma unroll
  for (int v = 0; v < V; ++v) p[v] /= s2;
  int pick;
  if (uniform != nullptr) {
    float cdf[V], run = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      cdf[v] = seg_prefix_sum(p[v], 64, lane) + run;
      run = __shfl(cdf[v], 63, 64);
    }
    const float thr = uniform[r] * run;  // run = the last class's CDF (the segment form's max of the CDF)
    float below = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) below += (ok[v] && cdf[v] < thr) ? 1.f : 0.f;
    pick = (int)seg_sum_f(below, 64);
    if (pick > C - 1) pick = C - 1;
  } else {
    float bv = -1.f;
    int bi = 0;
#pragma unroll
    for (int v = 0; v < V; ++v)
      if (ok[v] && p[v] > bv) {  // ascending k within a lane: first index on ties
        bv = p[v];
        bi = lane + 64 * v;
      }
    pick = seg_argmax(bv, bi, 64);
  }
  const int64_t srow = (int64_t)(r / G) * lds + (int64_t)(r % G) * C;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int k = lane + 64 * v;
    if (ok[v]) {
      if (mixed) mixed[(int64_t)r * C + k] = m[v];
      sample[srow + k] = k == pick ? 1.f : 0.f;
    }
  }
  if (idx != nullptr && lane == 0) idx[(int64_t)(r / G) * ldi + (r % G)] = ioff + (r % G) * C + pick;
}

template <int V>
__global__ void __launch_bounds__(256) unimix_sample_wide_bwd_kernel(const float* __restrict__ logits,
                                                                     const float* __restrict__ g_mixed,
                                                                     const float* __restrict__ g_sample,
                                                                     float* __restrict__ dlogits, int R, int C, float alpha) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;  // wave-uniform
  const int64_t base = (int64_t)r * C;
  float l[V], q[V], pm[V], m[V], gm[V];
  bool ok[V], clamped[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int k = lane + 64 * v;
    ok[v] = k < C;
    const int kc = k < C ? k : C - 1;
    const float x = logits[base + kc];
    l[v] = ok[v] ? x : -INFINITY;
    m[v] = l[v];
    q[v] = pm[v] = 0.f;
    clamped[v] = false;
    const float g = g_mixed ? g_mixed[base + kc] : 0.f;
    gm[v] = ok[v] ? g : 0.f;
  }
  if (alpha > 0.f) {
    float mx = -INFINITY;
#pragma unroll
    for (int v = 0; v < V; ++v) mx = fmaxf(mx, l[v]);
    mx = seg_max_f(mx, 64);
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      q[v] = ok[v] ? __expf(l[v] - mx) : 0.f;
      s += q[v];
    }
    s = seg_sum_f(s, 64);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      q[v] /= s;
      pm[v] = (1.f - alpha) * q[v] + alpha / C;
      clamped[v] = pm[v] <= FEPS || pm[v] >= 1.f - FEPS;
      m[v] = ok[v] ? logf(fminf(fmaxf(pm[v], FEPS), 1.f - FEPS)) : -INFINITY;
    }
  }
  if (g_sample) {
    float mx2 = -INFINITY;
#pragma unroll
    for (int v = 0; v < V; ++v) mx2 = fmaxf(mx2, m[v]);
    mx2 = seg_max_f(mx2, 64);
    float p[V], gs[V], s2 = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      p[v] = ok[v] ? __expf(m[v] - mx2) : 0.f;
      s2 += p[v];
      const int k = lane + 64 * v;
      const float g = g_sample[base + (k < C ? k : C - 1)];
      gs[v] = ok[v] ? g : 0.f;
    }
    s2 = seg_sum_f(s2, 64);
    float dot = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      p[v] /= s2;
      dot += p[v] * gs[v];
    }
    dot = seg_sum_f(dot, 64);
#pragma unroll
    for (int v = 0; v < V; ++v) gm[v] += p[v] * (gs[v] - dot);
  }
  float dl[V];
  if (alpha > 0.f) {
    float w[V], dot = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      w[v] = (ok[v] && !clamped[v]) ? (1.f - alpha) * gm[v] / pm[v] : 0.f;
      dot += q[v] * w[v];
    }
    dot = seg_sum_f(dot, 64);
#pragma unroll
    for (int v = 0; v < V; ++v) dl[v] = q[v] * (w[v] - dot);
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) dl[v] = gm[v];
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int k = lane + 64 * v;
    if (ok[v]) dlogits[base + k] = dl[v];
  }
}

// ---------------------------------------------------------------- two-hot (one wave per row)
template <int MAXK>
__global__ void __launch_bounds__(256) twohot_nll_fwd_kernel(const float* __restrict__ logits, const float* __restrict__ y,
                                                             const float* __restrict__ bins, float* __restrict__ loss,
                                                             int R, int K) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const float* lr = logits + (int64_t)r * K;
  float yv = y[r];
  float x = copysignf(log1pf(fabsf(yv)), yv);
  float lv[MAXK], bv[MAXK];
  float mx = -INFINITY;
  int cle = 0, cgt = 0;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    bool ok = k < K;
    lv[i] = ok ? lr[k] : -INFINITY;
    bv[i] = ok ? bins[k] : 0.f;
    mx = fmaxf(mx, lv[i]);
    cle += (ok && bv[i] <= x) ? 1 : 0;
    cgt += (ok && bv[i] > x) ? 1 : 0;
  }
  mx = wave_max(mx);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) se += (lane + 64 * i < K) ? __expf(lv[i] - mx) : 0.f;
  const float lse = mx + logf(wave_sum(se));
  int below = (int)wave_sum((float)cle) - 1;
  int above = K - (int)wave_sum((float)cgt);
  below = below < 0 ? 0 : (below > K - 1 ? K - 1 : below);
  above = above < 0 ? 0 : (above > K - 1 ? K - 1 : above);
  const float bb = bins[below], ba = bins[above];
  const bool eq = below == above;
  const float db = eq ? 1.f : fabsf(bb - x), da = eq ? 1.f : fabsf(ba - x);
  const float tot = db + da;
  const float wb = da / tot, wa = db / tot;
  if (lane == 0) {
    float lpb = lr[below] - lse, lpa = lr[above] - lse;
    loss[r] = -(wb * lpb + wa * lpa);
  }
}

template <int MAXK>
__global__ void __launch_bounds__(256) twohot_nll_bwd_kernel(const float* __restrict__ logits, const float* __restrict__ y,
                                                             const float* __restrict__ bins, const float* __restrict__ gl,
                                                             float* __restrict__ dlogits, int R, int K) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const float* lr = logits + (int64_t)r * K;
  float yv = y[r];
  float x = copysignf(log1pf(fabsf(yv)), yv);
  float lv[MAXK];
  float mx = -INFINITY;
  int cle = 0, cgt = 0;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    bool ok = k < K;
    lv[i] = ok ? lr[k] : -INFINITY;
    float b = ok ? bins[k] : 0.f;
    mx = fmaxf(mx, lv[i]);
    cle += (ok && b <= x) ? 1 : 0;
    cgt += (ok && b > x) ? 1 : 0;
  }
  mx = wave_max(mx);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) se += (lane + 64 * i < K) ? __expf(lv[i] - mx) : 0.f;
  se = wave_sum(se);
  int below = (int)wave_sum((float)cle) - 1;
  int above = K - (int)wave_sum((float)cgt);
  below = below < 0 ? 0 : (below > K - 1 ? K - 1 : below);
  above = above < 0 ? 0 : (above > K - 1 ? K - 1 : above);
  const float bb = bins[below], ba = bins[above];
  const bool eq = below == above;
  const float db = eq ? 1.f : fabsf(bb - x), da = eq ? 1.f : fabsf(ba - x);
  const float tot = db + da;
  const float wb = da / tot, wa = db / tot;
  const float g = gl[r];
  float* dr = dlogits + (int64_t)r * K;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    if (k < K) {
      float t = (k == below ? wb : 0.f) + (k == above ? wa : 0.f);
      dr[k] = g * (__expf(lv[i] - mx) / se - t);
    }
  }
}

// out[r] = symexp(sum_k softmax(l)_k * bins_k); also stores s = sum p*b for the backward
// wave max through DPP row reductions + readlanes (max is exact, so the result equals wave_max's)
__device__ __forceinline__ float wave_max_exact(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

template <int MAXK>
__global__ void __launch_bounds__(256) twohot_mean_fwd_kernel(const float* __restrict__ logits,
                                                              const float* __restrict__ bins, float* __restrict__ out,
                                                              float* __restrict__ s_out, int R, int K) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const float* lr = logits + (int64_t)r * K;
  float lv[MAXK], bv[MAXK];  // (the bins requested with the row: no second memory latency after the max)
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    lv[i] = k < K ? lr[k] : -INFINITY;
    bv[i] = k < K ? bins[k] : 0.f;
    mx = fmaxf(mx, lv[i]);
  }
  mx = wave_max_exact(mx);
  float se = 0.f, sb = 0.f;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    if (k < K) {
      float e = __expf(lv[i] - mx);
      se += e;
      sb += e * bv[i];
    }
  }
  se = wave_sum(se);
  sb = wave_sum(sb);
  if (lane == 0) {
    float s = sb / se;
    s_out[r] = s;
    out[r] = copysignf(expm1f(fabsf(s)), s);
  }
}

template <int MAXK>
__global__ void __launch_bounds__(256) twohot_mean_bwd_kernel(const float* __restrict__ logits,
                                                              const float* __restrict__ bins, const float* __restrict__ s_in,
                                                              const float* __restrict__ gout, float* __restrict__ dlogits,
                                                              int R, int K) {
  const int lane = threadIdx.x & 63;
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const float* lr = logits + (int64_t)r * K;
  float lv[MAXK], bv[MAXK];
  float mx = -INFINITY;
  const float s = s_in[r], go = gout[r];  // requested with the row (used after the reductions)
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    lv[i] = k < K ? lr[k] : -INFINITY;
    bv[i] = k < K ? bins[k] : 0.f;
    mx = fmaxf(mx, lv[i]);
  }
  mx = wave_max_exact(mx);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) se += (lane + 64 * i < K) ? __expf(lv[i] - mx) : 0.f;
  se = wave_sum(se);
  const float g = go * __expf(fabsf(s));
  float* dr = dlogits + (int64_t)r * K;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    int k = lane + 64 * i;
    if (k < K) dr[k] = g * (__expf(lv[i] - mx) / se) * (bv[i] - s);
  }
}

// ---------------------------------------------------------------- categorical KL(post || prior)
// one block per row; row holds G groups of C classes; loss = (dyn + rep) * max(kl, free)
// also the row's summed categorical entropies of a and b (the posterior / prior entropy metrics of
// reference dreamer_v3.py:512-515) when ent_a / ent_b are given: they reuse the log-softmaxes.
__global__ void __launch_bounds__(256) kl_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     float* __restrict__ kl_out, float* __restrict__ loss_out,
                                                     float* __restrict__ ent_a, float* __restrict__ ent_b, int R, int G,
                                                     int C, int W, float dyn, float rep, float free_nats) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int spw = 64 / W;
  const int k = lane % W;
  const int r = blockIdx.x;
  float acc = 0.f, hA = 0.f, hB = 0.f;
  for (int g0 = 0; g0 < G; g0 += 4 * spw) {
    const int g = g0 + wid * spw + lane / W;
    const bool valid = g < G && k < C;
    const int64_t off = ((int64_t)r * G + g) * C + k;
    float av = valid ? a[off] : -INFINITY, bv = valid ? b[off] : -INFINITY;
    float ma = seg_max(av, W), mb = seg_max(bv, W);
    float ea = valid ? __expf(av - ma) : 0.f, eb = valid ? __expf(bv - mb) : 0.f;
    float la = logf(seg_sum(ea, W)) + ma, lb = logf(seg_sum(eb, W)) + mb;
    float lpa = av - la, lpb = bv - lb;
    float p = valid ? __expf(lpa) : 0.f;
    acc += valid ? p * (lpa - lpb) : 0.f;
    if (ent_a) {
      hA -= valid ? p * lpa : 0.f;
      hB -= valid ? __expf(lpb) * lpb : 0.f;
    }
  }
  float kl = block_sum<4>(acc, red);
  if (ent_a) {
    hA = block_sum<4>(hA, red);
    hB = block_sum<4>(hB, red);
  }
  if (threadIdx.x == 0) {
    kl_out[r] = kl;
    loss_out[r] = (dyn + rep) * fmaxf(kl, free_nats);
    if (ent_a) {
      ent_a[r] = hA;
      ent_b[r] = hB;
    }
  }
}

__global__ void __launch_bounds__(256) kl_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     const float* __restrict__ kl_in, const float* __restrict__ gl,
                                                     float* __restrict__ da, float* __restrict__ db, int R, int G, int C,
                                                     int W, float dyn, float rep, float free_nats) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int spw = 64 / W;
  const int k = lane % W;
  const int r = blockIdx.x;
  const bool active = kl_in[r] > free_nats;
  const float g = active ? gl[r] : 0.f;
  for (int g0 = 0; g0 < G; g0 += 4 * spw) {
    const int grp = g0 + wid * spw + lane / W;
    const bool valid = grp < G && k < C;
    const int64_t off = ((int64_t)r * G + grp) * C + k;
    float av = valid ? a[off] : -INFINITY, bv = valid ? b[off] : -INFINITY;
    float ma = seg_max(av, W), mb = seg_max(bv, W);
    float ea = valid ? __expf(av - ma) : 0.f, eb = valid ? __expf(bv - mb) : 0.f;
    float sa = seg_sum(ea, W), sb = seg_sum(eb, W);
    float lpa = av - (logf(sa) + ma), lpb = bv - (logf(sb) + mb);
    float p = ea / sa, q = eb / sb;
    float klg = seg_sum(valid ? p * (lpa - lpb) : 0.f, W);
    if (valid) {
      da[off] = rep * g * p * ((lpa - lpb) - klg);
      db[off] = dyn * g * (q - p);
    }
  }
}

}  // namespace srl

using namespace srl;

static int next_pow2(int c) {
  int w = 1;
  while (w < c) w <<= 1;
  return w;
}

bool launch_unimix_sample_fwd(const float* logits, const float* uniform, float* mixed, float* sample, int R, int C,
                              float alpha, hipStream_t st, int G, int lds, int* idx, int ldi, int ioff) {
  if (C < 1 || C > 1024) return false;
  if (G <= 0) {
    G = 1;
    lds = C;
  }
  if (C > 64) {  // one wave per categorical, 4 per block
    const dim3 g(cdiv(R, 4)), b(256);
#define SRL_UW(V) hipLaunchKernelGGL(unimix_sample_wide_fwd_kernel<V>, g, b, 0, st, logits, uniform, mixed, sample, R, C, alpha, G, lds, idx, ldi, ioff)
    if (C <= 128) SRL_UW(2);
    else if (C <= 256) SRL_UW(4);
    else if (C <= 512) SRL_UW(8);
    else SRL_UW(16);
#undef SRL_UW
    return true;
  }
  int W = next_pow2(C);
  int segs_per_block = 4 * (64 / W);
  hipLaunchKernelGGL(unimix_sample_fwd_kernel, dim3(cdiv(R, segs_per_block)), dim3(256), 0, st, logits, uniform, mixed,
                     sample, R, C, W, alpha, G, lds, idx, ldi, ioff);
  return true;
}

bool launch_unimix_sample_bwd(const float* logits, const float* g_mixed, const float* g_sample, float* dlogits, int R,
                              int C, float alpha, hipStream_t st) {
  if (C < 1 || C > 1024) return false;
  if (C > 64) {
    const dim3 g(cdiv(R, 4)), b(256);
#define SRL_UW(V) hipLaunchKernelGGL(unimix_sample_wide_bwd_kernel<V>, g, b, 0, st, logits, g_mixed, g_sample, dlogits, R, C, alpha)
    if (C <= 128) SRL_UW(2);
    else if (C <= 256) SRL_UW(4);
    else if (C <= 512) SRL_UW(8);
    else SRL_UW(16);
#undef SRL_UW
    return true;
  }
  int W = next_pow2(C);
  int segs_per_block = 4 * (64 / W);
  hipLaunchKernelGGL(unimix_sample_bwd_kernel, dim3(cdiv(R, segs_per_block)), dim3(256), 0, st, logits, g_mixed, g_sample,
                     dlogits, R, C, W, alpha);
  return true;
}

// DreamerV3 critic objective (reference dreamer_v3.py:327-336): loss = mean_r w_r (nll(l_r, y1_r) + nll(l_r, y2_r)) over
// the two-hot encodings of the lambda returns y1 and the target critic's values y2, one wave per row.  The logits
// gradient is written in the same pass (d/dl_rk = scale w_r (2 softmax_rk - t1_rk - t2_rk)); the autograd backward only
// scales it by the incoming gradient.  Per-block partials (4 rows, fixed order) -> fixed-order final sum (value_loss_final).
__device__ __forceinline__ void th_interp(const float* __restrict__ bins, int K, float x, int cle, int cgt, int& below,
                                          int& above, float& wb, float& wa) {
  below = cle - 1;
  above = K - cgt;
  below = below < 0 ? 0 : (below > K - 1 ? K - 1 : below);
  above = above < 0 ? 0 : (above > K - 1 ? K - 1 : above);
  const float bb = bins[below], ba = bins[above];
  const bool eq = below == above;
  const float db = eq ? 1.f : fabsf(bb - x), da = eq ? 1.f : fabsf(ba - x);
  const float tot = db + da;
  wb = da / tot;
  wa = db / tot;
}

template <int MAXK>
__global__ void __launch_bounds__(256) value_loss2_kernel(const float* __restrict__ logits, const float* __restrict__ y1,
                                                          const float* __restrict__ y2, const float* __restrict__ w,
                                                          const float* __restrict__ bins, float* __restrict__ dlogits,
                                                          float* __restrict__ partial, int R, int K, float scale) {
  __shared__ float rowv[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wv;
  float v = 0.f;
  if (r < R) {
    const float* lr = logits + (int64_t)r * K;
    const float a = y1[r], b = y2[r];
    const float x1 = copysignf(log1pf(fabsf(a)), a), x2 = copysignf(log1pf(fabsf(b)), b);
    float lv[MAXK];
    float mx = -INFINITY;
    int c1le = 0, c1gt = 0, c2le = 0, c2gt = 0;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const int k = lane + 64 * i;
      const bool ok = k < K;
      lv[i] = ok ? lr[k] : -INFINITY;
      const float bk = ok ? bins[k] : 0.f;
      mx = fmaxf(mx, lv[i]);
      c1le += (ok && bk <= x1) ? 1 : 0;
      c1gt += (ok && bk > x1) ? 1 : 0;
      c2le += (ok && bk <= x2) ? 1 : 0;
      c2gt += (ok && bk > x2) ? 1 : 0;
    }
    mx = wave_max(mx);
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) se += (lane + 64 * i < K) ? __expf(lv[i] - mx) : 0.f;
    se = wave_sum(se);
    const float lse = mx + logf(se);
    int b1, a1, b2, a2;
    float wb1, wa1, wb2, wa2;
    th_interp(bins, K, x1, (int)wave_sum((float)c1le), (int)wave_sum((float)c1gt), b1, a1, wb1, wa1);
    th_interp(bins, K, x2, (int)wave_sum((float)c2le), (int)wave_sum((float)c2gt), b2, a2, wb2, wa2);
    const float wr = w[r];
    // the same per-term arithmetic as twohot_nll_fwd_kernel, then w * (nll1 + nll2) as the torch composite
    const float n1 = -(wb1 * (lr[b1] - lse) + wa1 * (lr[a1] - lse));
    const float n2 = -(wb2 * (lr[b2] - lse) + wa2 * (lr[a2] - lse));
    v = (n1 + n2) * wr;
    const float g = scale * wr;
    float* dr = dlogits + (int64_t)r * K;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const int k = lane + 64 * i;
      if (k < K) {
        const float t = (k == b1 ? wb1 : 0.f) + (k == a1 ? wa1 : 0.f) + (k == b2 ? wb2 : 0.f) + (k == a2 ? wa2 : 0.f);
        dr[k] = g * (2.f * (__expf(lv[i] - mx) / se) - t);
      }
    }
  }
  if (lane == 0) rowv[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (rowv[0] + rowv[1]) + (rowv[2] + rowv[3]);
}

// fixed-order tree: lane-strided sums (each thread's elements in index order), a butterfly wave sum, then the 4 wave
// totals in order - bitwise reproducible run to run, ~n/256 dependent adds per lane instead of n in one lane
__global__ void __launch_bounds__(256) value_loss_final(const float* __restrict__ partial, int n, float scale,
                                                        float* __restrict__ loss) {
  __shared__ float wsum[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *loss = ((wsum[0] + wsum[1]) + (wsum[2] + wsum[3])) * scale;
}

#define TH_DISPATCH(KERNEL, ...)                                                                       \
  do {                                                                                                 \
    dim3 g(cdiv(R, 4)), b(256);                                                                        \
    if (K <= 64) hipLaunchKernelGGL(KERNEL<1>, g, b, 0, st, __VA_ARGS__);                              \
    else if (K <= 128) hipLaunchKernelGGL(KERNEL<2>, g, b, 0, st, __VA_ARGS__);                        \
    else if (K <= 256) hipLaunchKernelGGL(KERNEL<4>, g, b, 0, st, __VA_ARGS__);                        \
    else if (K <= 512) hipLaunchKernelGGL(KERNEL<8>, g, b, 0, st, __VA_ARGS__);                        \
    else return false;                                                                                 \
  } while (0)

bool launch_twohot_nll_fwd(const float* logits, const float* y, const float* bins, float* loss, int R, int K,
                           hipStream_t st) {
  TH_DISPATCH(twohot_nll_fwd_kernel, logits, y, bins, loss, R, K);
  return true;
}
bool launch_twohot_nll_bwd(const float* logits, const float* y, const float* bins, const float* gl, float* dlogits, int R,
                           int K, hipStream_t st) {
  TH_DISPATCH(twohot_nll_bwd_kernel, logits, y, bins, gl, dlogits, R, K);
  return true;
}
bool launch_value_loss2(const float* logits, const float* y1, const float* y2, const float* w, const float* bins,
                        float* dlogits, float* partial, float* loss, int R, int K, hipStream_t st) {
  const float scale = 1.f / (float)R;
  TH_DISPATCH(value_loss2_kernel, logits, y1, y2, w, bins, dlogits, partial, R, K, scale);
  hipLaunchKernelGGL(value_loss_final, dim3(1), dim3(256), 0, st, partial, cdiv(R, 4), scale, loss);
  return true;
}
bool launch_twohot_mean_fwd(const float* logits, const float* bins, float* out, float* s, int R, int K, hipStream_t st) {
  TH_DISPATCH(twohot_mean_fwd_kernel, logits, bins, out, s, R, K);
  return true;
}
bool launch_twohot_mean_bwd(const float* logits, const float* bins, const float* s, const float* gout, float* dlogits,
                            int R, int K, hipStream_t st) {
  TH_DISPATCH(twohot_mean_bwd_kernel, logits, bins, s, gout, dlogits, R, K);
  return true;
}

bool launch_kl_fwd(const float* a, const float* b, float* kl, float* loss, float* ent_a, float* ent_b, int R, int G, int C,
                   float dyn, float rep, float free_nats, hipStream_t st) {
  if (C > 64) return false;
  hipLaunchKernelGGL(kl_fwd_kernel, dim3(R), dim3(256), 0, st, a, b, kl, loss, ent_a, ent_b, R, G, C, next_pow2(C), dyn,
                     rep, free_nats);
  return true;
}
bool launch_kl_bwd(const float* a, const float* b, const float* kl, const float* gl, float* da, float* db, int R, int G,
                   int C, float dyn, float rep, float free_nats, hipStream_t st) {
  if (C > 64) return false;
  hipLaunchKernelGGL(kl_bwd_kernel, dim3(R), dim3(256), 0, st, a, b, kl, gl, da, db, R, G, C, next_pow2(C), dyn, rep,
                     free_nats);
  return true;
}
