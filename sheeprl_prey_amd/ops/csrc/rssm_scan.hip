// DreamerV3 posterior scan in FOUR launches per step forward and FOUR per step backward
// (reference loop: dreamer_v3.py:122-129 over RSSM.dynamic, agent.py:350-437).
//
// The scan is latency-bound: every GEMM has M = per-rank batch (16) rows, so each step is a chain
// of weight-streaming GEMMs whose LayerNorm / GRU / unimix work is all-to-all over a row.  Instead
// of one launch per op (9 + 9 per step, ops/rssm.py RSSMScanFn), every launch here is
//
//     prologue  : every workgroup rebuilds the WHOLE 16-row A operand in LDS from the previous
//                 launch's raw output (LN+act, LN-GRU cell, is_first masking, LN backward, GRU
//                 backward) - redundant but cheap (16 x K elements), and it removes the seam;
//                 each workgroup also publishes its own disjoint slice of the step's saved tensors
//     GEMM      : a 16 x (16*NT) output tile on v_mfma_f32_16x16x4_f32 (exact fp32), K split
//                 over the 16 waves, weights streamed as float4 (one 16 B fragment feeds 4 MFMAs)
//
// Workgroups are 1024 threads (16 waves, 4 per SIMD): the LDS footprint (the whole A operand,
// up to ~150 KiB) allows one workgroup per CU, so the prologue's LDS/VALU chains get their
// latency hiding from waves inside the workgroup; row reductions use one wave per row.
//     epilogue  : bias/residual, and for the categorical layers (32-column tiles = whole
//                 categorical groups) the unimix + straight-through sample (fwd) or its adjoint
//                 (bwd) on the tile itself.
//
// Forward step t:  F1 zm = mask(z_{t-1}); xr = zm Wz^T + a_proj[t]
//                  F2 A = [mask(h_{t-1}), act(LN1(xr))];  gx = A Wg^T
//                  F3 A = h_t = LNGRU(gx, h_{t-1});       u = h_t [Wt1; Wr1]^T + P[t]
//                  F4 A = act(LN2_g(u_g));  logits_g = A W2_g^T + b2_g; unimix; sample
// Backward step t: G1 dv_g = dlog_g W2_g
//                  G2 A = du = LN2_bwd(dv);              DH[t] += du W1
//                  G3 A = dgx = LNGRU_bwd(DH[t]);        dcat = dgx Wg
//                  G4 A = dx = LN1_bwd(dcat[:, H:]);     dz = dx Wz; dlog_post[t-1] = unimix_bwd(...)
// Weight gradients are NOT formed per step: the caller does one GEMM per weight over all T*B rows.
// LayerNorm parameter gradients are written as per-step column partials [T, N] (summed over rows
// in-kernel, no atomics) and reduced over T by the caller.
#include "common.h"
#include "scan_dev.h"
#include "scan4.h"

#include <algorithm>

namespace srl {
namespace scan4 {

using namespace scandev;

#define STAMP(id, k)                                                                        \
  do {                                                                                      \
    if (p.prof && blockIdx.x == 0 && threadIdx.x == 0) p.prof[(id) * 16 + (k)] = clock64(); \
  } while (0)


// ------------------------------------------------------------------------------------------ F1
__global__ void __launch_bounds__(NTH) f1_kernel(SP p, int t) {
  STAMP(0, 0);
  extern __shared__ float sm[];
  const int K = p.S, lda = K + 4, B = p.B, S = p.S, H = p.H, HD = p.H + p.D;
  const int n0 = blockIdx.x * 16;
  WTile<1, 4> wt;
  wload<1, 4>(wt, p.Wz + (size_t)n0 * K, K, K, threadIdx.x >> 6);
  float* As = sm;
  float* red = As + 16 * lda;
  float* ct = red + 4096;
  const float* first = p.first + (size_t)t * B;
  const float* zprev = t > 0 ? p.samples + ((size_t)p.T + t - 1) * B * S : nullptr;  // samples[1][t-1]
  {
    const int c4 = K >> 2, n = 16 * c4;
    constexpr int U = 4;
    for (int base = 0; base < n; base += NTH * U) {
      f4 z[U], z0[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int idx = base + q * NTH + threadIdx.x;
        const int i = idx / c4, k = (idx - i * c4) << 2;
        const bool ok = idx < n && i < B;
        z[q] = (ok && zprev) ? *(const f4*)(zprev + (size_t)i * S + k) : f4{0.f, 0.f, 0.f, 0.f};
        z0[q] = ok ? *(const f4*)(p.z0 + k) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int idx = base + q * NTH + threadIdx.x;
        const int i = idx / c4, k = (idx - i * c4) << 2;
        if (idx < n) {
          const float f = i < B ? first[i] : 0.f;
          *(f4*)(As + i * lda + k) = (1.f - f) * z[q] + f * z0[q];
        }
      }
    }
  }
  int lo, hi;
  chunk(B * H, lo, hi);
  float* cat = p.cat + (size_t)t * B * HD;
  const float* hprev = t > 0 ? p.hs + (size_t)(t - 1) * B * H : nullptr;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) {
    const int b = e / H, j = e - b * H;
    cat[(size_t)b * HD + j] = hprev ? (1.f - first[b]) * hprev[e] : 0.f;
  }
  __syncthreads();
  STAMP(0, 1);
  chunk(B * S, lo, hi);
  float* zm = p.zm + (size_t)t * B * S;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) zm[e] = As[(e / S) * lda + e % S];
  STAMP(0, 2);
  gemm16<1, 4>(wt, As, lda, p.Wz + (size_t)n0 * K, K, K, red, ct);
  STAMP(0, 3);
  if (threadIdx.x < 256) {
    const float* ap = p.a_proj + (size_t)t * B * p.D;
    float* xr = p.xr + (size_t)t * B * p.D;
    const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
    if (b < B) xr[(size_t)b * p.D + n0 + c] = ct[threadIdx.x] + ap[(size_t)b * p.D + n0 + c];
  }
  STAMP(0, 4);
}

// ------------------------------------------------------------------------------------------ F2
__global__ void __launch_bounds__(NTH) f2_kernel(SP p, int t) {
  STAMP(1, 0);
  extern __shared__ float sm[];
  const int H = p.H, D = p.D, HD = H + D, K = HD, lda = K + 4, B = p.B;
  const int n0 = blockIdx.x * 16, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WTile<1, 4> wt;
  wload<1, 4>(wt, p.Wg + (size_t)n0 * K, K, K, w);
  float* As = sm;
  float* lw = As + 16 * lda;  // ln1 gamma, beta
  float* lb = lw + D;
  float* red = lb + D;
  float* ct = red + 4096;
  float* cat = p.cat + (size_t)t * B * HD;
  stage(As, lda, cat, HD, B, H);
  stage(As + H, lda, p.xr + (size_t)t * B * D, D, B, D);
  stage_vec(lw, p.ln1w, D);
  stage_vec(lb, p.ln1b, D);
  __syncthreads();
  STAMP(1, 1);
  if (w < B) {
    float* r = As + w * lda + H;
    float mu, rs;
    wave_row_stats(r, D, p.eps1, mu, rs);
    for (int k = lane; k < D; k += 64) r[k] = f_act((r[k] - mu) * rs * lw[k] + lb[k], p.act1);
    if (blockIdx.x == 0 && lane == 0) {
      p.m1[(size_t)t * B + w] = mu;
      p.r1[(size_t)t * B + w] = rs;
    }
  }
  __syncthreads();
  STAMP(1, 2);
  int lo, hi;
  chunk(B * D, lo, hi);
  for (int e = lo + threadIdx.x; e < hi; e += NTH) {
    const int b = e / D, k = e - b * D;
    cat[(size_t)b * HD + H + k] = As[b * lda + H + k];
  }
  STAMP(1, 3);
  gemm16<1, 4>(wt, As, lda, p.Wg + (size_t)n0 * K, K, K, red, ct);
  STAMP(1, 4);
  if (threadIdx.x < 256) {
    float* gx = p.gx + (size_t)t * B * 3 * H;
    const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
    if (b < B) gx[(size_t)b * 3 * H + n0 + c] = ct[threadIdx.x];
  }
  STAMP(1, 5);
}

// ------------------------------------------------------------------------------------------ F3
__global__ void __launch_bounds__(NTH) f3_kernel(SP p, int t) {
  STAMP(2, 0);
  extern __shared__ float sm[];
  const int H = p.H, HD = H + p.D, K = H, lda = K + 4, B = p.B, N3 = 3 * H, NU = 2 * p.hid, ldr = N3 + 4;
  const int n0 = blockIdx.x * 16, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WTile<1, 4> wt;
  wload<1, 4>(wt, p.W1 + (size_t)n0 * K, K, K, w);
  float* As = sm;
  float* R = As + 16 * lda;
  float* gw = R + 16 * ldr;  // LN-GRU gamma, beta [3H]
  float* gb = gw + N3;
  float* red = gb + N3;
  float* ct = red + 4096;
  stage(As, lda, p.cat + (size_t)t * B * HD, HD, B, H);  // masked h_{t-1}
  stage(R, ldr, p.gx + (size_t)t * B * N3, N3, B, N3);
  stage_vec(gw, p.lngw, N3);
  stage_vec(gb, p.lngb, N3);
  __syncthreads();
  STAMP(2, 1);
  if (w < B) {
    const float* x = R + w * ldr;
    float mu, rs;
    wave_row_stats(x, N3, p.epsg, mu, rs);
    float* a = As + w * lda;
    for (int j = lane; j < H; j += 64) {
      const float zr = (x[j] - mu) * rs * gw[j] + gb[j];
      const float zc = (x[H + j] - mu) * rs * gw[H + j] + gb[H + j];
      const float zu = (x[2 * H + j] - mu) * rs * gw[2 * H + j] + gb[2 * H + j];
      const float r = fsig(zr);
      const float c = ftanh(r * zc);
      const float uu = fsig(zu - 1.f);
      a[j] = uu * c + (1.f - uu) * a[j];
    }
    if (blockIdx.x == 0 && lane == 0) {
      p.mg[(size_t)t * B + w] = mu;
      p.rg[(size_t)t * B + w] = rs;
    }
  }
  __syncthreads();
  STAMP(2, 2);
  int lo, hi;
  chunk(B * H, lo, hi);
  float* hs = p.hs + (size_t)t * B * H;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) hs[e] = As[(e / H) * lda + e % H];
  if (t + 1 < p.T) {
    // step t+1's F1 work that does not need the posterior sample: the masked h half of its GRU input (its
    // recurrent input xr[t+1] is formed by FX of step t+1 from F4's selected rows)
    const float* first1 = p.first + (size_t)(t + 1) * B;
    float* cat1 = p.cat + (size_t)(t + 1) * B * HD;
    for (int e = lo + threadIdx.x; e < hi; e += NTH) {
      const int b = e / H, j = e - b * H;
      cat1[(size_t)b * HD + j] = (1.f - first1[b]) * As[b * lda + j];
    }
  }
  STAMP(2, 3);
  gemm16<1, 4>(wt, As, lda, p.W1 + (size_t)n0 * K, K, K, red, ct);
  STAMP(2, 4);
  if (threadIdx.x < 256) {
    const float* P = p.P + (size_t)t * B * NU;
    float* u = p.u + (size_t)t * B * NU;
    const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
    if (b < B) u[(size_t)b * NU + n0 + c] = ct[threadIdx.x] + P[(size_t)b * NU + n0 + c];
  }
  STAMP(2, 5);
}

// ------------------------------------------------------------------------------------------ F4
__global__ void __launch_bounds__(NTH) f4_kernel(SP p, int t) {
  STAMP(3, 0);
  extern __shared__ float sm[];
  const int hid = p.hid, K = hid, lda = K + 4, B = p.B, S = p.S, NU = 2 * hid, C = p.C, T = p.T;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col0 = blockIdx.x * 32;
  const int g = col0 / S, n0 = col0 - g * S;
  WTile<2, 4> wt;
  wload<2, 4>(wt, p.W2 + ((size_t)g * S + n0) * hid, hid, K, w);
  float* As = sm;
  float* lw = As + 16 * lda;
  float* lb = lw + hid;
  float* red = lb + hid;
  float* ct = red + 8192;
  stage(As, lda, p.u + (size_t)t * B * NU + (size_t)g * hid, NU, B, hid);
  stage_vec(lw, p.ln2w + (size_t)g * hid, hid);
  stage_vec(lb, p.ln2b + (size_t)g * hid, hid);
  __syncthreads();
  STAMP(3, 1);
  if (w < B) {
    float* r = As + w * lda;
    float mu, rs;
    wave_row_stats(r, hid, p.eps2, mu, rs);
    for (int k = lane; k < hid; k += 64) r[k] = f_act((r[k] - mu) * rs * lw[k] + lb[k], p.act2);
    if (n0 == 0 && lane == 0) {
      p.m2[(size_t)t * 2 * B + w * 2 + g] = mu;
      p.r2[(size_t)t * 2 * B + w * 2 + g] = rs;
    }
  }
  __syncthreads();
  STAMP(3, 2);
  {  // v[g][t] slice: the S/32 workgroups of group g split it
    const int Q = S / 32, q = n0 / 32, total = B * hid, per = (total + Q - 1) / Q;
    const int lo = q * per, hi = min(total, lo + per);
    float* v = p.v + ((size_t)g * T + t) * B * hid;
    for (int e = lo + threadIdx.x; e < hi; e += NTH) v[e] = As[(e / hid) * lda + e % hid];
  }
  STAMP(3, 3);
  gemm16<2, 4>(wt, As, lda, p.W2 + ((size_t)g * S + n0) * hid, hid, K, red, ct);
  STAMP(3, 4);
  // epilogue: bias, unimix + straight-through sample; a wave covers 2 rows x 32 columns
  if (threadIdx.x < 512) {
    const size_t base = ((size_t)g * T + t) * B * S;
    const int nseg = S / C;
    const float* uni = p.uni + (size_t)t * 2 * B * nseg;
    const int idx = threadIdx.x;
    const int b = idx >> 5, c = idx & 31, k = c % C;
    const bool valid = b < B;
    const float l = ct[idx] + p.b2[(size_t)g * S + n0 + c];
    float m = l;
    if (p.alpha > 0.f) {
      const float mx = seg_max(l, C);
      const float e = __expf(l - mx);
      const float q = e / seg_sum(e, C);
      float pm = (1.f - p.alpha) * q + p.alpha / C;
      pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
      m = logf(pm);
    }
    const float mx2 = seg_max(m, C);
    const float e2 = __expf(m - mx2);
    const float pr = e2 / seg_sum(e2, C);
    float cdf = pr;  // inclusive prefix sum inside the segment
    for (int o = 1; o < C; o <<= 1) {
      const float tt = __shfl_up(cdf, o, C);
      if (k >= o) cdf += tt;
    }
    const int r = (g * B + (valid ? b : 0)) * nseg + (n0 + c) / C;
    const float uu = valid ? uni[r] : 0.f;
    const float below = cdf < uu * seg_max(cdf, C) ? 1.f : 0.f;
    int pick = (int)seg_sum(below, C);
    if (pick > C - 1) pick = C - 1;
    if (valid) {
      const size_t o = base + (size_t)b * S + n0 + c;
      p.logits[o] = l;
      p.mixed[o] = m;
      p.samples[o] = (k == pick) ? 1.f : 0.f;
    }
    if (g == 1 && t + 1 < T) {
      // posterior z_t feeds step t+1: masked copy zm[t+1], and its selected rows go to the LDS list
      const float f1 = valid ? p.first[(size_t)(t + 1) * B + b] : 1.f;
      if (valid) {
        const size_t o = ((size_t)(t + 1) * B + b) * S + n0 + c;
        p.zm[o] = (1.f - f1) * (k == pick ? 1.f : 0.f) + f1 * p.z0[n0 + c];
      }
      // [t+1][16 rows][S / C categoricals]: selected WzT row, -1 = reset row (is_first is binary) / padding row;
      // FX of step t+1 sums the rows (no atomics: one thread per output element)
      if (k == 0) p.sel[((size_t)(t + 1) * 16 + b) * (S / C) + (n0 + c) / C] = (valid && f1 == 0.f) ? n0 + (c - k) + pick : -1;
    }
  }
  STAMP(3, 5);
}

// ------------------------------------------------------------------------------------------ FX
// xr[t][b][:] = a_proj[t][b][:] + first[t][b] z0 Wz^T + sum over categoricals of WzT[sel[t][b][g]][:] (t >= 1): the
// posterior one-hot of step t-1 as row gathers.  Grid D / 64 workgroups; thread (b, quad) owns 4 columns of row b,
// every gathered row load unconditional (a clamped row 0, weighted 0 for -1).
__global__ void __launch_bounds__(NTH) fx_kernel(SP p, int t) {
  const int B = p.B, D = p.D, nseg = p.S / p.C;
  const int b = threadIdx.x >> 4, j = blockIdx.x * 64 + 4 * (threadIdx.x & 15);
  if (b >= B || j >= D) return;
  const int* sl = p.sel + ((size_t)t * 16 + b) * nseg;
  const size_t o = ((size_t)t * B + b) * D + j;
  const float f = p.first[(size_t)t * B + b];
  float4 x = *reinterpret_cast<const float4*>(p.a_proj + o);
  const float4 c = *reinterpret_cast<const float4*>(p.c0 + j);
  x.x += f * c.x;
  x.y += f * c.y;
  x.z += f * c.z;
  x.w += f * c.w;
  // batches of 8 categoricals: the 8 indices, then the 8 row loads in flight together (4 round trips at 32
  // categoricals instead of 32)
  for (int g0 = 0; g0 < nseg; g0 += 8) {
    int row[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int gi = g0 + u < nseg ? g0 + u : nseg - 1;
      const int r = sl[gi];
      row[u] = g0 + u < nseg ? r : -1;
    }
    float4 rv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) rv[u] = *reinterpret_cast<const float4*>(p.WzT + (size_t)(row[u] >= 0 ? row[u] : 0) * D + j);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float w = row[u] >= 0 ? 1.f : 0.f;
      x.x += w * rv[u].x;
      x.y += w * rv[u].y;
      x.z += w * rv[u].z;
      x.w += w * rv[u].w;
    }
  }
  *reinterpret_cast<float4*>(p.xr + o) = x;
}

// ------------------------------------------------------------------------------------------ G1
__global__ void __launch_bounds__(NTH) g1_kernel(SP p, int t) {
  STAMP(4, 0);
  extern __shared__ float sm[];
  const int S = p.S, K = S, lda = K + 4, B = p.B, hid = p.hid, T = p.T;
  const int tiles = hid / 16;
  const int g = blockIdx.x / tiles, n0 = (blockIdx.x - g * tiles) * 16;
  WTile<1, 4> wt;
  wload<1, 4>(wt, p.W2T + ((size_t)g * hid + n0) * S, S, K, threadIdx.x >> 6);
  float* As = sm;
  float* red = As + 16 * lda;
  float* ct = red + 4096;
  stage(As, lda, p.dlog + ((size_t)g * T + t) * B * S, S, B, S);
  __syncthreads();
  STAMP(4, 1);
  gemm16<1, 4>(wt, As, lda, p.W2T + ((size_t)g * hid + n0) * S, S, K, red, ct);
  STAMP(4, 2);
  if (threadIdx.x < 256) {
    float* dv = p.dv + ((size_t)g * T + t) * B * hid;
    const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
    if (b < B) dv[(size_t)b * hid + n0 + c] = ct[threadIdx.x];
  }
  STAMP(4, 3);
}

// ------------------------------------------------------------------------------------------ G2
__global__ void __launch_bounds__(NTH) g2_kernel(SP p, int t) {
  STAMP(5, 0);
  extern __shared__ float sm[];
  const int hid = p.hid, NU = 2 * hid, K = NU, lda = K + 4, B = p.B, T = p.T, H = p.H;
  const int n0 = blockIdx.x * 16, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WTile<1, 4> wt;
  wload<1, 4>(wt, p.W1T + (size_t)n0 * NU, NU, K, w);
  float* As = sm;            // raw u -> xh -> du
  float* R = As + 16 * lda;  // dv -> dz (both groups side by side)
  float* st = R + 16 * lda;  // s1[16][2], s2[16][2], rs[16][2]
  float* lw = st + 96;       // ln2 gamma, beta [2 * hid]
  float* lb = lw + NU;
  float* red = lb + NU;
  float* ct = red + 4096;
  stage_vec(lw, p.ln2w, NU);
  stage_vec(lb, p.ln2b, NU);
  stage(As, lda, p.u + (size_t)t * B * NU, NU, B, NU);
  stage(R, lda, p.dv + (size_t)t * B * hid, hid, B, hid);
  stage(R + hid, lda, p.dv + ((size_t)T + t) * B * hid, hid, B, hid);
  __syncthreads();
  STAMP(5, 1);
  if (w < B) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const float mu = p.m2[(size_t)t * 2 * B + w * 2 + g], rs = p.r2[(size_t)t * 2 * B + w * 2 + g];
      float s1, s2;
      wave_ln_bwd_prep(As + w * lda + g * hid, R + w * lda + g * hid, lw + g * hid, lb + g * hid, hid, p.act2, mu, rs, s1,
                       s2);
      if (lane == 0) {
        st[w * 2 + g] = s1;
        st[32 + w * 2 + g] = s2;
        st[64 + w * 2 + g] = rs;
      }
    }
  }
  __syncthreads();
  STAMP(5, 2);
  int lo, hi;
  chunk(NU, lo, hi);
  ln_param_partials(As, lda, R, lda, B, lo, hi, p.p2g + (size_t)t * NU, p.p2b + (size_t)t * NU);
  __syncthreads();
  if (w < B) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const float s1 = st[w * 2 + g], s2 = st[32 + w * 2 + g], rs = st[64 + w * 2 + g];
      float* x = As + w * lda + g * hid;
      const float* dz = R + w * lda + g * hid;
      const float* gm = lw + g * hid;
      for (int k = lane; k < hid; k += 64) x[k] = rs * (dz[k] * gm[k] - s1 - x[k] * s2);
    }
  }
  __syncthreads();
  STAMP(5, 3);
  chunk(B * NU, lo, hi);
  float* du = p.du + (size_t)t * B * NU;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) du[e] = As[(e / NU) * lda + e % NU];
  STAMP(5, 4);
  gemm16<1, 4>(wt, As, lda, p.W1T + (size_t)n0 * NU, NU, K, red, ct);
  STAMP(5, 5);
  if (threadIdx.x < 256) {
    float* DH = p.DH + (size_t)t * B * H;
    const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
    if (b < B) DH[(size_t)b * H + n0 + c] += ct[threadIdx.x];
  }
  STAMP(5, 6);
}

// ------------------------------------------------------------------------------------------ G3
// Wave i owns row i; lane s owns j = s + 64 m (m < G3_MAXM): h_{t-1}, DH[t] and the normalised
// gate inputs stay in registers between the passes.  Requires H <= 64 * G3_MAXM.
#define G3_MAXM 8
__global__ void __launch_bounds__(NTH) g3_kernel(SP p, int t) {
  STAMP(6, 0);
  extern __shared__ float sm[];
  const int H = p.H, HD = H + p.D, N3 = 3 * H, K = N3, lda = K + 4, B = p.B;
  const int n0 = blockIdx.x * 16, i = threadIdx.x >> 6, s = threadIdx.x & 63;
  WTile<1, 6> wt;
  wload<1, 6>(wt, p.WgT + (size_t)n0 * N3, N3, K, i);
  float* As = sm;             // raw gx -> dz*gamma -> dgx (in place)
  float* gw = As + 16 * lda;  // LN-GRU gamma, beta [3H]
  float* gb = gw + N3;
  float* red = gb + N3;
  float* ct = red + 4096;
  float* sc = ct + 256;       // column partial scratch [2][chunk][16]
  const bool row_ok = i < B;
  float hpv[G3_MAXM], dhv[G3_MAXM];
  {
    const float* cat = p.cat + ((size_t)t * B + (row_ok ? i : 0)) * HD;
    const float* DH = p.DH + ((size_t)t * B + (row_ok ? i : 0)) * H;
#pragma unroll
    for (int m = 0; m < G3_MAXM; ++m) {
      const int j = s + 64 * m;
      const bool ok = row_ok && j < H;
      hpv[m] = ok ? cat[j] : 0.f;
      dhv[m] = ok ? DH[j] : 0.f;
    }
  }
  stage(As, lda, p.gx + (size_t)t * B * N3, N3, B, N3);
  stage_vec(gw, p.lngw, N3);
  stage_vec(gb, p.lngb, N3);
  __syncthreads();
  STAMP(6, 1);
  int clo, chi;
  chunk(N3, clo, chi);
  const int nch = chi - clo;
  int hlo, hhi;
  chunk(B * H, hlo, hhi);
  if (row_ok) {
    const float mu = p.mg[(size_t)t * B + i], rs = p.rg[(size_t)t * B + i];
    float* x = As + i * lda;
    float xh0[G3_MAXM], xh1[G3_MAXM], xh2[G3_MAXM];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int m = 0; m < G3_MAXM; ++m) {  // pass 1: gate adjoints, stored as dz*gamma in place
      const int j = s + 64 * m;
      if (j < H) {
        const float a0 = (x[j] - mu) * rs, a1 = (x[H + j] - mu) * rs, a2 = (x[2 * H + j] - mu) * rs;
        const float zr = a0 * gw[j] + gb[j];
        const float zc = a1 * gw[H + j] + gb[H + j];
        const float zu = a2 * gw[2 * H + j] + gb[2 * H + j];
        const float r = fsig(zr), c = ftanh(r * zc), u = fsig(zu - 1.f);
        const float go = dhv[m];
        const float dua = go * (c - hpv[m]);
        const float da = go * u * (1.f - c * c);
        const float dz2 = dua * u * (1.f - u);
        const float dz1 = da * r;
        const float dz0 = da * zc * r * (1.f - r);
        const float d0 = dz0 * gw[j], d1 = dz1 * gw[H + j], d2 = dz2 * gw[2 * H + j];
        x[j] = d0;
        x[H + j] = d1;
        x[2 * H + j] = d2;
        xh0[m] = a0;
        xh1[m] = a1;
        xh2[m] = a2;
        s1 += d0 + d1 + d2;
        s2 += d0 * a0 + d1 * a1 + d2 * a2;
        if (j >= clo && j < chi) {
          sc[(j - clo) * 16 + i] = dz0 * a0;
          sc[(nch + j - clo) * 16 + i] = dz0;
        }
        if (H + j >= clo && H + j < chi) {
          sc[(H + j - clo) * 16 + i] = dz1 * a1;
          sc[(nch + H + j - clo) * 16 + i] = dz1;
        }
        if (2 * H + j >= clo && 2 * H + j < chi) {
          sc[(2 * H + j - clo) * 16 + i] = dz2 * a2;
          sc[(nch + 2 * H + j - clo) * 16 + i] = dz2;
        }
        const int e = i * H + j;
        if (e >= hlo && e < hhi) p.dhp[e] = go * (1.f - u);
      }
    }
    const float m1 = wave_sum(s1) / N3, m2 = wave_sum(s2) / N3;
#pragma unroll
    for (int m = 0; m < G3_MAXM; ++m) {  // pass 2: dgx (the wave owns its row: no barrier needed)
      const int j = s + 64 * m;
      if (j < H) {
        x[j] = rs * (x[j] - m1 - xh0[m] * m2);
        x[H + j] = rs * (x[H + j] - m1 - xh1[m] * m2);
        x[2 * H + j] = rs * (x[2 * H + j] - m1 - xh2[m] * m2);
      }
    }
  }
  __syncthreads();
  STAMP(6, 2);
  for (int col = threadIdx.x; col < nch; col += NTH) {
    float ag = 0.f, ab = 0.f;
    for (int b = 0; b < B; ++b) {
      ag += sc[col * 16 + b];
      ab += sc[(nch + col) * 16 + b];
    }
    p.pgg[(size_t)t * N3 + clo + col] = ag;
    p.pgb[(size_t)t * N3 + clo + col] = ab;
  }
  int lo, hi;
  chunk(B * N3, lo, hi);
  float* dgx = p.dgx + (size_t)t * B * N3;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) dgx[e] = As[(e / N3) * lda + e % N3];
  STAMP(6, 3);
  gemm16<1, 6>(wt, As, lda, p.WgT + (size_t)n0 * N3, N3, K, red, ct);
  STAMP(6, 4);
  if (threadIdx.x < 256) {
    const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
    if (b < B) p.dcat[(size_t)b * HD + n0 + c] = ct[threadIdx.x];
  }
  STAMP(6, 5);
}

// ------------------------------------------------------------------------------------------ G4
constexpr int G4_RED = 8192 + 512;  // red + ct of gemm16<2, .>

__global__ void __launch_bounds__(NTH) g4_kernel(SP p, int t) {
  STAMP(7, 0);
  extern __shared__ float sm[];
  const int H = p.H, D = p.D, HD = H + D, K = D, lda = K + 4, B = p.B, S = p.S, C = p.C, T = p.T;
  const int n0 = blockIdx.x * 32, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WTile<2, 4> wt;
  if (t > 0) wload<2, 4>(wt, p.WzT + (size_t)n0 * D, D, K, w);
  float* As = sm;             // raw xr -> xh -> dx
  float* R = As + 16 * lda;   // dcat[:, H:] -> dz
  float* st = R + 16 * lda;   // s1[16], s2[16], rs[16]
  float* lw = st + 48;        // ln1 gamma, beta
  float* lb = lw + D;
  // the GEMM's cross-wave reduction scratch (8192 + 512 floats) reuses R once R is dead (after the LN backward)
  // when R is large enough (D >= 540: the prey preset's dense 1024 then fits the 160 KB of LDS)
  float* red = 16 * lda >= G4_RED ? R : lb + D;
  float* ct = red + 8192;
  stage_vec(lw, p.ln1w, D);
  stage_vec(lb, p.ln1b, D);
  stage(As, lda, p.xr + (size_t)t * B * D, D, B, D);
  stage(R, lda, p.dcat + H, HD, B, D);
  __syncthreads();
  STAMP(7, 1);
  if (w < B) {
    const float mu = p.m1[(size_t)t * B + w], rs = p.r1[(size_t)t * B + w];
    float s1, s2;
    wave_ln_bwd_prep(As + w * lda, R + w * lda, lw, lb, D, p.act1, mu, rs, s1, s2);
    if (lane == 0) {
      st[w] = s1;
      st[16 + w] = s2;
      st[32 + w] = rs;
    }
  }
  __syncthreads();
  STAMP(7, 2);
  int lo, hi;
  chunk(D, lo, hi);
  ln_param_partials(As, lda, R, lda, B, lo, hi, p.p1g + (size_t)t * D, p.p1b + (size_t)t * D);
  __syncthreads();
  if (w < B) {
    const float s1 = st[w], s2 = st[16 + w], rs = st[32 + w];
    float* x = As + w * lda;
    const float* dz = R + w * lda;
    for (int k = lane; k < D; k += 64) x[k] = rs * (dz[k] * lw[k] - s1 - x[k] * s2);
  }
  __syncthreads();
  STAMP(7, 3);
  chunk(B * D, lo, hi);
  float* dx = p.dx + (size_t)t * B * D;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) dx[e] = As[(e / D) * lda + e % D];
  if (t == 0) return;  // uniform: no h_{-1} / z_{-1} to propagate into
  const float* first = p.first + (size_t)t * B;
  chunk(B * H, lo, hi);
  float* DHp = p.DH + (size_t)(t - 1) * B * H;
  for (int e = lo + threadIdx.x; e < hi; e += NTH) {
    const int b = e / H, j = e - b * H;
    DHp[e] += (1.f - first[b]) * (p.dhp[e] + p.dcat[(size_t)b * HD + j]);
  }
  STAMP(7, 4);
  gemm16<2, 4>(wt, As, lda, p.WzT + (size_t)n0 * D, D, K, red, ct);
  STAMP(7, 5);
  // epilogue: d(sample) of step t-1 posterior, then the unimix / straight-through adjoint
  if (threadIdx.x < 512) {
    const size_t base = ((size_t)T + t - 1) * B * S;  // [1][t-1]
    const float* dpost = p.dpost ? p.dpost + (size_t)(t - 1) * B * S : nullptr;
    const int idx = threadIdx.x;
    const int b = idx >> 5, c = idx & 31;
    const bool valid = b < B;
    const int bb = valid ? b : 0;
    const size_t o = base + (size_t)bb * S + n0 + c;
    const float ds = (dpost ? dpost[(size_t)bb * S + n0 + c] : 0.f) + (1.f - first[bb]) * ct[idx];
    const float l = p.logits[o];
    float q = 0.f, pm = 0.f, m = l;
    bool clamped = false;
    if (p.alpha > 0.f) {
      const float mx = seg_max(l, C);
      const float e = __expf(l - mx);
      q = e / seg_sum(e, C);
      pm = (1.f - p.alpha) * q + p.alpha / C;
      clamped = pm <= FEPS || pm >= 1.f - FEPS;
      m = logf(fminf(fmaxf(pm, FEPS), 1.f - FEPS));
    }
    float gm = p.dmixed[o];
    const float mx2 = seg_max(m, C);
    const float e2 = __expf(m - mx2);
    const float pr = e2 / seg_sum(e2, C);
    const float dot = seg_sum(pr * ds, C);
    gm += pr * (ds - dot);
    float dl;
    if (p.alpha > 0.f) {
      const float wv = clamped ? 0.f : (1.f - p.alpha) * gm / pm;
      dl = q * (wv - seg_sum(q * wv, C));
    } else {
      dl = gm;
    }
    if (valid) p.dlog[o] = dl;
  }
  STAMP(7, 6);
}

void set_lds(const void* fn, int bytes) { (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes); }

}  // namespace scan4
}  // namespace srl

using namespace srl;
using namespace srl::scan4;

bool launch_unimix_sample_bwd(const float* logits, const float* g_mixed, const float* g_sample, float* dl, int R, int C,
                              float alpha, hipStream_t st);

// Dynamic LDS bytes of each kernel; mirrors the carving at the top of every kernel.
struct Lds {
  int f1, f2, f3, f4, g1, g2, g3, g4;
};

static Lds scan4_lds_sizes(int S, int D, int H, int hid) {
  const int HD = H + D, N3 = 3 * H;
  const int g3_grid = HD / 16, g3_nch = (N3 + g3_grid - 1) / g3_grid;
  Lds l;
  const int r1 = 4096 + 256, r2 = 8192 + 512;  // red + ct for NT = 1 / 2
  l.f1 = 16 * (S + 4) + r1;
  l.f2 = 16 * (HD + 4) + 2 * D + r1;
  l.f3 = 16 * (H + 4) + 16 * (N3 + 4) + 2 * N3 + r1;
  l.f4 = 16 * (hid + 4) + 2 * hid + r2;
  l.g1 = 16 * (S + 4) + r1;
  l.g2 = 2 * 16 * (2 * hid + 4) + 96 + 4 * hid + r1;
  l.g3 = 16 * (N3 + 4) + 2 * N3 + r1 + 2 * 16 * g3_nch;
  l.g4 = 2 * 16 * (D + 4) + 48 + 2 * D + (16 * (D + 4) >= G4_RED ? 0 : r2);  // red aliases the dead dz tile
  int* v = &l.f1;
  for (int k = 0; k < 8; ++k) v[k] *= 4;
  return l;
}

// Max dynamic LDS a single workgroup may take (bytes); the host checks shapes against it.
int scan4_max_lds() { return 160 * 1024; }

int scan4_fwd_lds(int S, int D, int H, int hid) {
  const Lds l = scan4_lds_sizes(S, D, H, hid);
  return std::max(std::max(l.f1, l.f2), std::max(l.f3, l.f4));
}

int scan4_bwd_lds(int S, int D, int H, int hid) {
  const Lds l = scan4_lds_sizes(S, D, H, hid);
  return std::max(std::max(l.g1, l.g2), std::max(l.g3, l.g4));
}

void launch_scan4_fwd(const SP& p, hipStream_t st) {
  static bool init = false;
  if (!init) {
    const int mx = scan4_max_lds();
    set_lds((const void*)f1_kernel, mx);
    set_lds((const void*)f2_kernel, mx);
    set_lds((const void*)f3_kernel, mx);
    set_lds((const void*)f4_kernel, mx);
    init = true;
  }
  const Lds l = scan4_lds_sizes(p.S, p.D, p.H, p.hid);
  for (int t = 0; t < p.T; ++t) {
    // F1 only starts the scan: later steps get masked z / masked h from F3 and F4 of step t-1, xr from FX
    if (t == 0)
      hipLaunchKernelGGL(f1_kernel, dim3(p.D / 16), dim3(NTH), l.f1, st, p, t);
    else
      hipLaunchKernelGGL(fx_kernel, dim3((p.D + 63) / 64), dim3(NTH), 0, st, p, t);
    hipLaunchKernelGGL(f2_kernel, dim3(3 * p.H / 16), dim3(NTH), l.f2, st, p, t);
    hipLaunchKernelGGL(f3_kernel, dim3(2 * p.hid / 16), dim3(NTH), l.f3, st, p, t);
    hipLaunchKernelGGL(f4_kernel, dim3(2 * p.S / 32), dim3(NTH), l.f4, st, p, t);
  }
}

void launch_scan4_bwd(const SP& p, hipStream_t st) {
  static bool init = false;
  if (!init) {
    const int mx = scan4_max_lds();
    set_lds((const void*)g1_kernel, mx);
    set_lds((const void*)g2_kernel, mx);
    set_lds((const void*)g3_kernel, mx);
    set_lds((const void*)g4_kernel, mx);
    init = true;
  }
  const int T = p.T, B = p.B, S = p.S, HD = p.H + p.D;
  const Lds l = scan4_lds_sizes(p.S, p.D, p.H, p.hid);
  // prior half: no recurrent gradient, one launch for all steps
  launch_unimix_sample_bwd(p.logits, p.dmixed, nullptr, p.dlog, T * B * S / p.C, p.C, p.alpha, st);
  // posterior of the last step: only the external gradients
  const size_t last = ((size_t)T + T - 1) * B * S;
  launch_unimix_sample_bwd(p.logits + last, p.dmixed + last, p.dpost ? p.dpost + (size_t)(T - 1) * B * S : nullptr,
                           p.dlog + last, B * S / p.C, p.C, p.alpha, st);
  for (int t = T - 1; t >= 0; --t) {
    hipLaunchKernelGGL(g1_kernel, dim3(2 * p.hid / 16), dim3(NTH), l.g1, st, p, t);
    hipLaunchKernelGGL(g2_kernel, dim3(p.H / 16), dim3(NTH), l.g2, st, p, t);
    hipLaunchKernelGGL(g3_kernel, dim3(HD / 16), dim3(NTH), l.g3, st, p, t);
    hipLaunchKernelGGL(g4_kernel, dim3(S / 32), dim3(NTH), l.g4, st, p, t);
  }
}
