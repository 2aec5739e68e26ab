// DreamerV3 posterior scan as ONE persistent launch forward and ONE backward (reference loop:
// dreamer_v3.py:122-129 over RSSM.dynamic, agent.py:350-437; the 4+4-launch predecessor is
// rssm_scan.hip).
//
// Why persistent: per step the scan is a chain of 16-row GEMMs (M = per-rank batch) whose weights
// (~9.4 MB fp32 on the posterior path at the Atari-100k shapes) were re-staged from L2/HBM by every
// launch, 7 launches per step.  Here every workgroup loads its weight tiles ONCE into registers
// (float4 MFMA B fragments, K split over the 16 waves) and keeps them for all T steps; the steps'
// GEMM -> LayerNorm seams become in-launch hand-offs between workgroups.
//
// Only the posterior path is sequential.  The prior (transition) logits depend on h_t alone, so the
// caller computes them after the forward scan as batched GEMMs over all T*B rows, and their
// gradient reaches h_t through d_hs before the backward scan starts.
//
// Forward, step t (three hand-offs):
//   A  (3H/16 tiles) A = [(1-first) h_{t-1}, act(LN1(xr_t))]; gx tile = A Wg^T; per-row (mean, M2)
//                    partials of the tile published with it
//   B  (hid/16)      LN-GRU: row statistics from the partials (Chan combine), gates straight from
//                    gx in global memory -> h_t (A operand, redundantly per workgroup);
//                    u tile = h_t Wr1^T + P_t
//   C  (S/32)        A = act(LN2(u_t)); logits tile = A W2^T + b2 (whole categorical groups);
//                    unimix + straight-through sample; the one-hot posterior enters xr_{t+1} as
//                    row gathers of Wz^T added with device-scope atomics
// Backward, step t (four hand-offs):
//   G1 (hid/16)  dv = dlog_t W2                   G2 (H/16)  du = LN2'(dv); DH_t += du Wr1
//   G3 ((H+D)/16) dgx = LNGRU'(DH_t); dcat = dgx Wg; DH_{t-1} += (1-first)(dh_direct + dcat_h)
//   G4 (S/32)    dx = LN1'(dcat_x); dz = dx Wz; dlog_{t-1} = unimix'(d_post + (1-first) dz)
//
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, write-through form): every word a
// workgroup hands to another inside the launch is stored sc1 (write-through) or by a device-scope
// atomic, every storing wave drains (s_waitcnt vmcnt(0)), the workgroup barrier follows, then ONE
// lane adds to the phase's arrival counter (8 shards on separate 128-B lines, shard = block % 8).
// Consumers poll the shards with sc1 loads from one wave, then read every handed-off word with sc1
// loads (bypassing the CU's L1, which other CUs' stores never refresh).  Counters are monotonic
// within a launch (round r expects r x producers) and zeroed by a kernel before every launch.  Every
// spin is bounded: on timeout the waiter writes its code to the error word and the workgroup leaves;
// every other waiter sees the error word and leaves too, so the grid always drains.
#include "common.h"
#include "scan_dev.h"
#include "scanp.h"

#include <algorithm>

namespace srl {
namespace scanp {

using namespace scandev;

typedef unsigned int u32;
typedef unsigned long long u64;

constexpr int NSH = 8;                // shards per arrival counter
constexpr int SHW = 32;               // u32 words between shards (128 B)
constexpr int NCTR = 4;               // counters per direction
constexpr int ERRW = NCTR * NSH * SHW;  // index of the error word
constexpr u32 SPIN_MAX = 1u << 20;

// Register tile caps per phase (K chunks of 16 per wave): host gate mirrors them.
constexpr int UA = 4, UB = 2, UC = 2;           // K = H+D <= 1024, H <= 512, hid <= 512
constexpr int U1 = 4, U2 = 2, U3 = 6, U4 = 2;   // K = S <= 1024, hid <= 512, 3H <= 1536, D <= 512
constexpr int GRU_M = 8;                        // H <= 64 * GRU_M

// ------------------------------------------------------------------ write-through accesses
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_wt2(const float* p) {
  const u64 x = __hip_atomic_load(reinterpret_cast<u64*>(const_cast<float*>(p)), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(float2, x);
}
__device__ __forceinline__ void st_wt2(float* p, float a, float b) {
  __hip_atomic_store(reinterpret_cast<u64*>(p), __builtin_bit_cast(u64, make_float2(a, b)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// 16 x cols tile (cols % 4 == 0) from global (row stride ls) into LDS (row stride ld); rows >= nvalid
// are zero; rows are optionally scaled by (1 - first[row]).  Every load is a 16-B sc1 buffer load.
__device__ __forceinline__ void stage_wt(float* dst, int ld, const float* src, int ls, int nvalid, int cols,
                                         const float* first = nullptr) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, nvalid * ls * 4, 0x00020000);
  const int c4 = cols >> 2, n = 16 * c4;
  constexpr int U = 4;
  for (int base = 0; base < n; base += NTH * U) {
    f4 r[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int idx = base + q * NTH + threadIdx.x;
      const int i = idx / c4, k = (idx - i * c4) << 2;
      r[q] = (idx < n && i < nvalid)
                 ? __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (i * ls + k) * 4, 0, 16))
                 : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int idx = base + q * NTH + threadIdx.x;
      const int i = idx / c4, k = (idx - i * c4) << 2;
      if (idx < n) {
        const float s = (first && i < nvalid) ? 1.f - first[i] : 1.f;
        *(f4*)(dst + i * ld + k) = s * r[q];
      }
    }
  }
}

// ------------------------------------------------------------------ arrival counters
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Every wave has issued its hand-off stores: drain them, join, one lane arrives.
__device__ __forceinline__ void arrive(u32* ctr) {
  drain();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(ctr + (blockIdx.x & (NSH - 1)) * SHW, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane s < NSH: how many producers in [p0, p0 + np) arrive on shard s per round.
__device__ __forceinline__ u32 shard_count(int p0, int np) {
  const int s = threadIdx.x & 63;
  u32 c = 0;
  if (s < NSH)
    for (int q = p0; q < p0 + np; ++q) c += (u32)((q & (NSH - 1)) == s);
  return c;
}

// Wave 0 polls until every shard holds rounds x its producer count; the workgroup then joins.
// Returns false (uniformly) when the launch is aborting.
__device__ __forceinline__ bool wait_ctr(u32* sync, int ctr, u32 cnt, u32 rounds, int code, int* flag) {
  if (threadIdx.x < 64) {
    const int s = threadIdx.x;
    const u32 need = cnt * rounds;
    u32* w = sync + ctr * NSH * SHW + s * SHW;
    u32* err = sync + ERRW;
    int bad = 0;
    for (u32 spins = 0;; ++spins) {
      const u32 v = s < NSH ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const u32 e = s == NSH ? __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      if (__any(e != 0u)) {
        bad = 1;
        break;
      }
      if (__all(s >= NSH || v >= need)) break;
      if (spins >= SPIN_MAX) {
        bad = 2;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (s == 0) {
      if (bad == 2) __hip_atomic_store(err, (u32)code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = bad;
    }
  }
  __syncthreads();
  const bool ok = *flag == 0;
  __syncthreads();
  return ok;
}

// Contiguous part `part` of [0, total) split into `parts`.
__device__ __forceinline__ void part_range(int total, int part, int parts, int& lo, int& hi) {
  const int per = (total + parts - 1) / parts;
  lo = part * per;
  hi = min(total, lo + per);
  if (lo > hi) lo = hi;
}

// ------------------------------------------------------------------ register-resident GEMM
// C[16][16*NT] (LDS ct) = A[16][K] (LDS) x Wtile^T, the whole K in the wave's register tile.
template <int NT, int U>
__device__ __forceinline__ void gemm_reg(const WTile<NT, U>& wt, const float* As, int lda, int K, float* red, float* ct) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  const int nch = K >> 4;
  const float* arow = As + i * lda + 4 * g;
  f4 a[U];
#pragma unroll
  for (int q = 0; q < U; ++q) {
    const int c = w + NWV * q;
    if (c < nch) a[q] = *(const f4*)(arow + (c << 4));
  }
#pragma unroll
  for (int q = 0; q < U; ++q) {
    const int c = w + NWV * q;
    if (c < nch) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][0], wt.b[q][t][0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][1], wt.b[q][t][1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][2], wt.b[q][t][2], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][3], wt.b[q][t][3], acc[t], 0, 0, 0);
      }
    }
  }
  constexpr int NC = 16 * NT;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(w * 16 + 4 * g + r) * NC + 16 * t + i] = acc[t][r];
  __syncthreads();
  if (threadIdx.x < 16 * NC) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) v += red[ww * 16 * NC + threadIdx.x];
    ct[threadIdx.x] = v;
  }
  __syncthreads();
}

// ======================================================================= LDS layouts
// One role per workgroup; each role carves the dynamic LDS its own way (floats).
__host__ __device__ inline int lds_A(int D, int H) { return 16 * (H + D + 4) + 2 * D + 4096 + 256 + 16; }
__host__ __device__ inline int lds_B(int H) { return 16 * (H + 4) + 6 * H + 4096 + 256 + 16; }
__host__ __device__ inline int lds_C(int hid) { return 16 * (hid + 4) + 2 * hid + 8192 + 512 + 16 + 512; }
__host__ __device__ inline int g3_parts(int H, int D) { return (H + D) / 16; }
__host__ __device__ inline int g3_nch(int H, int D) { return (3 * H + g3_parts(H, D) - 1) / g3_parts(H, D); }
__host__ __device__ inline int lds_G1(int S) { return 16 * (S + 4) + 4096 + 256 + 16; }
__host__ __device__ inline int lds_G2(int hid) { return 32 * (hid + 4) + 2 * hid + 48 + 4096 + 256 + 16; }
__host__ __device__ inline int lds_G3(int H, int D) { return 16 * (3 * H + 4) + 6 * H + 4096 + 256 + 256 + 32 * g3_nch(H, D) + 16; }
__host__ __device__ inline int lds_G4(int D) { return 32 * (D + 4) + 2 * D + 48 + 8192 + 512 + 16; }

// ======================================================================= forward roles
// Block ids: A = [0, nA), B = [nA, nA + nB), C = [nA + nB, nA + nB + nC).  Counters: 0 = A, 1 = B, 2 = C.

// A: gx tile = [(1-first) h_{t-1}, act(LN1(xr_t))] Wg^T, plus per-row (mean, M2) of the tile.
__device__ __forceinline__ void fwd_A(const PP& p, int a, float* sm) {
  const int B = p.B, D = p.D, H = p.H, HD = H + D, N3 = 3 * H, T = p.T;
  const int nA = N3 / 16, nB = p.hid / 16, nC = p.S / 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = HD + 4;
  float* As = sm;
  float* l1w = As + 16 * lda;
  float* l1b = l1w + D;
  float* red = l1b + D;
  float* ct = red + 4096;
  int* flag = (int*)(ct + 256);
  WTile<1, UA> wt;
  wload<1, UA>(wt, p.Wg + (size_t)a * 16 * HD, HD, HD, w);
  stage_vec(l1w, p.ln1w, D);
  stage_vec(l1b, p.ln1b, D);
  const u32 eB = shard_count(nA, nB), eC = shard_count(nA + nB, nC);
  for (int e = threadIdx.x; e < 16 * H; e += NTH) As[(e / H) * lda + e % H] = 0.f;  // h_{-1} = 0
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    if (t > 0) {
      // h_{t-1} is published by B(t-1) before C(t-1) runs: load it while C finishes
      if (!wait_ctr(p.sync, 1, eB, t, 1, flag)) return;
      stage_wt(As, lda, p.hs + (size_t)(t - 1) * B * H, H, B, H, p.first + (size_t)t * B);
      if (!wait_ctr(p.sync, 2, eC, t, 2, flag)) return;
    }
    stage_wt(As + H, lda, p.xr + (size_t)t * B * D, D, B, D);
    __syncthreads();
    if (w < B) {
      float* r = As + w * lda + H;
      float mu, rs;
      wave_row_stats(r, D, p.eps1, mu, rs);
      for (int k = lane; k < D; k += 64) r[k] = f_act((r[k] - mu) * rs * l1w[k] + l1b[k], p.act1);
      if (a == 0 && lane == 0) {
        p.m1[(size_t)t * B + w] = mu;
        p.r1[(size_t)t * B + w] = rs;
      }
    }
    __syncthreads();
    {
      int lo, hi;
      part_range(B * HD, a, nA, lo, hi);
      float* cat = p.cat + (size_t)t * B * HD;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) cat[e] = As[(e / HD) * lda + e % HD];
    }
    gemm_reg<1, UA>(wt, As, lda, HD, red, ct);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      const float x = ct[threadIdx.x];
      const float m = seg_sum(x, 16) * (1.f / 16.f);
      const float q = seg_sum((x - m) * (x - m), 16);
      if (b < B) {
        st_wt(p.gx + ((size_t)t * B + b) * N3 + a * 16 + c, x);
        if (c == 0) st_wt2(p.gst + (((size_t)t * nA + a) * 16 + b) * 2, m, q);
      }
    }
    arrive(p.sync + 0 * NSH * SHW);
  }
}

// B: h_t = LNGRU(gx_t, (1-first) h_{t-1}) (row statistics from A's partials, gates straight from gx);
// u tile = h_t Wr1^T + P_t.  h stays in this workgroup's LDS from one step to the next.
__device__ __forceinline__ void fwd_B(const PP& p, int bI, float* sm) {
  const int B = p.B, H = p.H, N3 = 3 * H, T = p.T, hid = p.hid;
  const int nA = N3 / 16, nB = hid / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = H + 4;
  float* As = sm;
  float* lgw = As + 16 * lda;
  float* lgb = lgw + N3;
  float* red = lgb + N3;
  float* ct = red + 4096;
  int* flag = (int*)(ct + 256);
  WTile<1, UB> wt;
  wload<1, UB>(wt, p.W1 + (size_t)bI * 16 * H, H, H, w);
  stage_vec(lgw, p.lngw, N3);
  stage_vec(lgb, p.lngb, N3);
  const u32 eA = shard_count(0, nA);
  for (int e = threadIdx.x; e < 16 * H; e += NTH) As[(e / H) * lda + e % H] = 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    if (!wait_ctr(p.sync, 0, eA, t + 1, 3, flag)) return;
    if (w < B) {
      // row statistics of gx from the nA tile partials (16 columns each): Chan's parallel combine
      float sm1 = 0.f;
      float2 pr[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = lane + 64 * k;
        pr[k] = i < nA ? ld_wt2(p.gst + (((size_t)t * nA + i) * 16 + w) * 2) : make_float2(0.f, 0.f);
        sm1 += pr[k].x;
      }
      const float mu = wave_sum(sm1) / nA;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = lane + 64 * k;
        if (i < nA) q += pr[k].y + 16.f * (pr[k].x - mu) * (pr[k].x - mu);
      }
      const float rs = rsqrtf(wave_sum(q) / N3 + p.epsg);
      const float keep = 1.f - p.first[(size_t)t * B + w];
      const float* gxr = p.gx + ((size_t)t * B + w) * N3;
      float x0[GRU_M], x1[GRU_M], x2[GRU_M];
#pragma unroll
      for (int m = 0; m < GRU_M; ++m) {
        const int j = lane + 64 * m;
        if (j < H) {
          x0[m] = ld_wt(gxr + j);
          x1[m] = ld_wt(gxr + H + j);
          x2[m] = ld_wt(gxr + 2 * H + j);
        }
      }
      float* hr = As + w * lda;
#pragma unroll
      for (int m = 0; m < GRU_M; ++m) {
        const int j = lane + 64 * m;
        if (j < H) {
          const float zr = (x0[m] - mu) * rs * lgw[j] + lgb[j];
          const float zc = (x1[m] - mu) * rs * lgw[H + j] + lgb[H + j];
          const float zu = (x2[m] - mu) * rs * lgw[2 * H + j] + lgb[2 * H + j];
          const float r = fsig(zr);
          const float c = ftanh(r * zc);
          const float uu = fsig(zu - 1.f);
          hr[j] = uu * c + (1.f - uu) * (keep * hr[j]);
        }
      }
      if (bI == 0 && lane == 0) {
        p.mg[(size_t)t * B + w] = mu;
        p.rg[(size_t)t * B + w] = rs;
      }
    }
    __syncthreads();
    {
      int lo, hi;
      part_range(B * H, bI, nB, lo, hi);
      float* hs = p.hs + (size_t)t * B * H;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) st_wt(hs + e, As[(e / H) * lda + e % H]);
    }
    gemm_reg<1, UB>(wt, As, lda, H, red, ct);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (b < B) {
        const size_t o = ((size_t)t * B + b) * hid + bI * 16 + c;
        st_wt(p.u + o, ct[threadIdx.x] + p.P[o]);
      }
    }
    arrive(p.sync + 1 * NSH * SHW);
  }
}

// C: logits tile = act(LN2(u_t)) W2^T + b2 over whole categorical groups; unimix + straight-through
// sample; the sampled one-hot rows of Wz^T are added into xr_{t+1} (device-scope atomics).
__device__ __forceinline__ void fwd_C(const PP& p, int cI, float* sm) {
  const int B = p.B, S = p.S, D = p.D, H = p.H, hid = p.hid, C = p.C, T = p.T;
  const int nA = 3 * H / 16, nB = hid / 16, nC = S / 32, nseg = S / C;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = hid + 4, n0 = cI * 32;
  float* As = sm;
  float* l2w = As + 16 * lda;
  float* l2b = l2w + hid;
  float* red = l2b + hid;
  float* ct = red + 8192;
  int* flag = (int*)(ct + 512);
  int* sel = flag + 16;  // [16 rows][32 / C groups]
  WTile<2, UC> wt;
  wload<2, UC>(wt, p.W2 + (size_t)n0 * hid, hid, hid, w);
  stage_vec(l2w, p.ln2w, hid);
  stage_vec(l2b, p.ln2b, hid);
  const u32 eB = shard_count(nA, nB);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    if (!wait_ctr(p.sync, 1, eB, t + 1, 4, flag)) return;
    stage_wt(As, lda, p.u + (size_t)t * B * hid, hid, B, hid);
    __syncthreads();
    if (w < B) {
      float* r = As + w * lda;
      float mu, rs;
      wave_row_stats(r, hid, p.eps2, mu, rs);
      for (int k = lane; k < hid; k += 64) r[k] = f_act((r[k] - mu) * rs * l2w[k] + l2b[k], p.act2);
      if (cI == 0 && lane == 0) {
        p.m2[(size_t)t * B + w] = mu;
        p.r2[(size_t)t * B + w] = rs;
      }
    }
    __syncthreads();
    {
      int lo, hi;
      part_range(B * hid, cI, nC, lo, hi);
      float* v = p.v + (size_t)t * B * hid;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) v[e] = As[(e / hid) * lda + e % hid];
    }
    gemm_reg<2, UC>(wt, As, lda, hid, red, ct);
    if (threadIdx.x < 512) {
      const size_t base = (size_t)t * B * S;
      const float* uni = p.uni + (size_t)t * B * nseg;
      const int idx = threadIdx.x;
      const int b = idx >> 5, c = idx & 31, k = c % C;
      const bool valid = b < B;
      const float l = ct[idx] + p.b2[n0 + c];
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
      const float uu = valid ? uni[b * nseg + (n0 + c) / C] : 0.f;
      const float below = cdf < uu * seg_max(cdf, C) ? 1.f : 0.f;
      int pick = (int)seg_sum(below, C);
      if (pick > C - 1) pick = C - 1;
      if (valid) {
        const size_t o = base + (size_t)b * S + n0 + c;
        p.logits[o] = l;
        p.mixed[o] = m;
        p.samples[o] = (k == pick) ? 1.f : 0.f;
      }
      if (t + 1 < T) {
        const float f1 = valid ? p.first[(size_t)(t + 1) * B + b] : 1.f;
        if (valid) p.zm[((size_t)(t + 1) * B + b) * S + n0 + c] = (1.f - f1) * (k == pick ? 1.f : 0.f) + f1 * p.z0[n0 + c];
        // selected Wz^T row per (row, group); -1: reset row (its z0 Wz^T is already in xr) or padding
        if (k == 0) sel[b * (32 / C) + c / C] = (valid && f1 == 0.f) ? n0 + c + pick : -1;
      }
    }
    if (t + 1 < T) {
      __syncthreads();
      const int npair = 16 * (32 / C);
      float* xr1 = p.xr + (size_t)(t + 1) * B * D;
      for (int e = threadIdx.x; e < npair * D; e += NTH) {
        const int pr = e / D, j = e - pr * D;
        const int row = sel[pr];
        if (row >= 0) atomicAdd(xr1 + (size_t)(pr / (32 / C)) * D + j, p.WzT[(size_t)row * D + j]);
      }
    }
    arrive(p.sync + 2 * NSH * SHW);
  }
}

__global__ void __launch_bounds__(NTH) fwd_kernel(PP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nA = 3 * p.H / 16, nB = p.hid / 16;
  const int bid = blockIdx.x;
  if (bid < nA)
    fwd_A(p, bid, sm);
  else if (bid < nA + nB)
    fwd_B(p, bid - nA, sm);
  else
    fwd_C(p, bid - nA - nB, sm);
}

// ======================================================================= backward roles
// Block ids: G1 = [0, n1), G2 = [n1, +n2), G3 = [n1 + n2, +n3), G4 = [n1 + n2 + n3, +n4).
// Counters: 0 = G1, 1 = G2, 2 = G3, 3 = G4.  Inputs the forward saved are staged BEFORE each wait.

// G1: dv_t = dlog_t W2 (K = S).
__device__ __forceinline__ void bwd_G1(const PP& p, int i, float* sm) {
  const int B = p.B, S = p.S, hid = p.hid, T = p.T, H = p.H, D = p.D;
  const int n1 = hid / 16, n2 = H / 16, n3 = (H + D) / 16, n4 = S / 32;
  const int w = threadIdx.x >> 6, lda = S + 4;
  float* As = sm;
  float* red = As + 16 * lda;
  float* ct = red + 4096;
  int* flag = (int*)(ct + 256);
  WTile<1, U1> wt;
  wload<1, U1>(wt, p.W2T + (size_t)i * 16 * S, S, S, w);
  const u32 e4 = shard_count(n1 + n2 + n3, n4);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    if (t < T - 1 && !wait_ctr(p.sync, 3, e4, T - 1 - t, 11, flag)) return;
    stage_wt(As, lda, p.dlog + (size_t)t * B * S, S, B, S);
    __syncthreads();
    gemm_reg<1, U1>(wt, As, lda, S, red, ct);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (b < B) st_wt(p.dv + ((size_t)t * B + b) * hid + i * 16 + c, ct[threadIdx.x]);
    }
    arrive(p.sync + 0 * NSH * SHW);
  }
}

// G2: du_t = LN2'(dv_t) (+ LN2 parameter partials); DH_t += du_t Wr1 (K = hid).
__device__ __forceinline__ void bwd_G2(const PP& p, int i, float* sm) {
  const int B = p.B, H = p.H, hid = p.hid, T = p.T;
  const int n1 = hid / 16, n2 = H / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = hid + 4;
  float* As = sm;
  float* R = As + 16 * lda;
  float* l2w = R + 16 * lda;
  float* l2b = l2w + hid;
  float* st = l2b + hid;
  float* red = st + 48;
  float* ct = red + 4096;
  int* flag = (int*)(ct + 256);
  WTile<1, U2> wt;
  wload<1, U2>(wt, p.W1T + (size_t)i * 16 * hid, hid, hid, w);
  stage_vec(l2w, p.ln2w, hid);
  stage_vec(l2b, p.ln2b, hid);
  const u32 e1 = shard_count(0, n1);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    stage(As, lda, p.u + (size_t)t * B * hid, hid, B, hid);
    if (!wait_ctr(p.sync, 0, e1, T - t, 12, flag)) return;
    stage_wt(R, lda, p.dv + (size_t)t * B * hid, hid, B, hid);
    __syncthreads();
    if (w < B) {
      const float mu = p.m2[(size_t)t * B + w], rs = p.r2[(size_t)t * B + w];
      float s1, s2;
      wave_ln_bwd_prep(As + w * lda, R + w * lda, l2w, l2b, hid, p.act2, mu, rs, s1, s2);
      if (lane == 0) {
        st[w] = s1;
        st[16 + w] = s2;
        st[32 + w] = rs;
      }
    }
    __syncthreads();
    int lo, hi;
    part_range(hid, i, n2, lo, hi);
    ln_param_partials(As, lda, R, lda, B, lo, hi, p.p2g + (size_t)t * hid, p.p2b + (size_t)t * hid);
    __syncthreads();
    if (w < B) {
      const float s1 = st[w], s2 = st[16 + w], rs = st[32 + w];
      float* x = As + w * lda;
      const float* dz = R + w * lda;
      for (int k = lane; k < hid; k += 64) x[k] = rs * (dz[k] * l2w[k] - s1 - x[k] * s2);
    }
    __syncthreads();
    part_range(B * hid, i, n2, lo, hi);
    float* du = p.du + (size_t)t * B * hid;
    for (int e = lo + threadIdx.x; e < hi; e += NTH) du[e] = As[(e / hid) * lda + e % hid];
    gemm_reg<1, U2>(wt, As, lda, hid, red, ct);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (b < B) {
        float* d = p.DH + ((size_t)t * B + b) * H + i * 16 + c;
        st_wt(d, ld_wt(d) + ct[threadIdx.x]);
      }
    }
    arrive(p.sync + 1 * NSH * SHW);
  }
}

// G3: dgx_t = LNGRU'(DH_t) (+ LN-GRU parameter partials); dcat tile = dgx_t Wg (K = 3H); h columns of
// the tile go straight into DH_{t-1} with the gate's direct path, feature columns are handed to G4.
__device__ __forceinline__ void bwd_G3(const PP& p, int i3, float* sm) {
  const int B = p.B, H = p.H, D = p.D, HD = H + D, N3 = 3 * H, T = p.T;
  const int n2 = H / 16, n3 = HD / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = N3 + 4, n0 = i3 * 16;
  const int nch = g3_nch(H, D);
  float* As = sm;
  float* lgw = As + 16 * lda;
  float* lgb = lgw + N3;
  float* red = lgb + N3;
  float* ct = red + 4096;
  float* dhpL = ct + 256;  // [16][16]: direct h gradient of this tile's columns
  float* sc = dhpL + 256;  // [2][nch][16] column partial scratch
  int* flag = (int*)(sc + 32 * nch);
  WTile<1, U3> wt;
  wload<1, U3>(wt, p.WgT + (size_t)n0 * N3, N3, N3, w);
  stage_vec(lgw, p.lngw, N3);
  stage_vec(lgb, p.lngb, N3);
  const u32 e2 = shard_count(p.hid / 16, n2);
  int clo, chi;
  part_range(N3, i3, n3, clo, chi);
  const int ncol = chi - clo;
  const int i = w;
  const bool row_ok = i < B;
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    stage(As, lda, p.gx + (size_t)t * B * N3, N3, B, N3);
    if (!wait_ctr(p.sync, 1, e2, T - t, 13, flag)) return;
    if (row_ok) {
      const float mu = p.mg[(size_t)t * B + i], rs = p.rg[(size_t)t * B + i];
      const float* DHr = p.DH + ((size_t)t * B + i) * H;
      const float* catr = p.cat + ((size_t)t * B + i) * HD;  // (1 - first) h_{t-1}
      float* x = As + i * lda;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll 2
      for (int m = 0; m < GRU_M; ++m) {  // pass 1: gate adjoints, stored as dz*gamma in place
        const int j = lane + 64 * m;
        if (j < H) {
          const float a0 = (x[j] - mu) * rs, a1 = (x[H + j] - mu) * rs, a2 = (x[2 * H + j] - mu) * rs;
          const float zr = a0 * lgw[j] + lgb[j];
          const float zc = a1 * lgw[H + j] + lgb[H + j];
          const float zu = a2 * lgw[2 * H + j] + lgb[2 * H + j];
          const float r = fsig(zr), c = ftanh(r * zc), u = fsig(zu - 1.f);
          const float go = ld_wt(DHr + j);
          const float dua = go * (c - catr[j]);
          const float da = go * u * (1.f - c * c);
          const float dz2 = dua * u * (1.f - u);
          const float dz1 = da * r;
          const float dz0 = da * zc * r * (1.f - r);
          const float d0 = dz0 * lgw[j], d1 = dz1 * lgw[H + j], d2 = dz2 * lgw[2 * H + j];
          x[j] = d0;
          x[H + j] = d1;
          x[2 * H + j] = d2;
          s1 += d0 + d1 + d2;
          s2 += d0 * a0 + d1 * a1 + d2 * a2;
          if (j >= clo && j < chi) {
            sc[(j - clo) * 16 + i] = dz0 * a0;
            sc[(ncol + j - clo) * 16 + i] = dz0;
          }
          if (H + j >= clo && H + j < chi) {
            sc[(H + j - clo) * 16 + i] = dz1 * a1;
            sc[(ncol + H + j - clo) * 16 + i] = dz1;
          }
          if (2 * H + j >= clo && 2 * H + j < chi) {
            sc[(2 * H + j - clo) * 16 + i] = dz2 * a2;
            sc[(ncol + 2 * H + j - clo) * 16 + i] = dz2;
          }
          if (j >= n0 && j < n0 + 16) dhpL[i * 16 + j - n0] = go * (1.f - u);
        }
      }
      const float m1 = wave_sum(s1) / N3, m2 = wave_sum(s2) / N3;
      // pass 2: dgx (the wave owns its row); the normalised inputs are re-read from gx (just staged,
      // cache-resident) instead of being held in 3 x GRU_M registers across the row reduction
      const float* gxr = p.gx + ((size_t)t * B + i) * N3;
#pragma unroll
      for (int m = 0; m < GRU_M; ++m) {
        const int j = lane + 64 * m;
        if (j < H) {
          x[j] = rs * (x[j] - m1 - (gxr[j] - mu) * rs * m2);
          x[H + j] = rs * (x[H + j] - m1 - (gxr[H + j] - mu) * rs * m2);
          x[2 * H + j] = rs * (x[2 * H + j] - m1 - (gxr[2 * H + j] - mu) * rs * m2);
        }
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < ncol; col += NTH) {
      float ag = 0.f, ab = 0.f;
      for (int b = 0; b < B; ++b) {
        ag += sc[col * 16 + b];
        ab += sc[(ncol + col) * 16 + b];
      }
      p.pgg[(size_t)t * N3 + clo + col] = ag;
      p.pgb[(size_t)t * N3 + clo + col] = ab;
    }
    {
      int lo, hi;
      part_range(B * N3, i3, n3, lo, hi);
      float* dgx = p.dgx + (size_t)t * B * N3;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) dgx[e] = As[(e / N3) * lda + e % N3];
    }
    gemm_reg<1, U3>(wt, As, lda, N3, red, ct);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (b < B) {
        const float v = ct[threadIdx.x];
        if (n0 >= H) {
          st_wt(p.dcat + ((size_t)t * B + b) * HD + n0 + c, v);
        } else if (t > 0) {
          float* d = p.DH + ((size_t)(t - 1) * B + b) * H + n0 + c;
          st_wt(d, ld_wt(d) + (1.f - p.first[(size_t)t * B + b]) * (dhpL[b * 16 + c] + v));
        }
      }
    }
    arrive(p.sync + 2 * NSH * SHW);
  }
}

// G4: dx_t = LN1'(dcat_x) (+ LN1 parameter partials); dz = dx_t Wz (K = D);
// dlog_{t-1} = unimix_ST'(logits_{t-1}; dmixed, d_post + (1-first_t) dz).
__device__ __forceinline__ void bwd_G4(const PP& p, int i4, float* sm) {
  const int B = p.B, S = p.S, D = p.D, H = p.H, HD = H + D, C = p.C, T = p.T;
  const int n3 = HD / 16, n4 = S / 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = D + 4, n0 = i4 * 32;
  float* As = sm;
  float* R = As + 16 * lda;
  float* l1w = R + 16 * lda;
  float* l1b = l1w + D;
  float* st = l1b + D;
  float* red = st + 48;
  float* ct = red + 8192;
  int* flag = (int*)(ct + 512);
  WTile<2, U4> wt;
  wload<2, U4>(wt, p.WzT + (size_t)n0 * D, D, D, w);
  stage_vec(l1w, p.ln1w, D);
  stage_vec(l1b, p.ln1b, D);
  const u32 e3 = shard_count(p.hid / 16 + H / 16, n3);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    stage(As, lda, p.xr + (size_t)t * B * D, D, B, D);
    if (!wait_ctr(p.sync, 2, e3, T - t, 14, flag)) return;
    stage_wt(R, lda, p.dcat + (size_t)t * B * HD + H, HD, B, D);
    __syncthreads();
    if (w < B) {
      const float mu = p.m1[(size_t)t * B + w], rs = p.r1[(size_t)t * B + w];
      float s1, s2;
      wave_ln_bwd_prep(As + w * lda, R + w * lda, l1w, l1b, D, p.act1, mu, rs, s1, s2);
      if (lane == 0) {
        st[w] = s1;
        st[16 + w] = s2;
        st[32 + w] = rs;
      }
    }
    __syncthreads();
    int lo, hi;
    part_range(D, i4, n4, lo, hi);
    ln_param_partials(As, lda, R, lda, B, lo, hi, p.p1g + (size_t)t * D, p.p1b + (size_t)t * D);
    __syncthreads();
    if (w < B) {
      const float s1 = st[w], s2 = st[16 + w], rs = st[32 + w];
      float* x = As + w * lda;
      const float* dz = R + w * lda;
      for (int k = lane; k < D; k += 64) x[k] = rs * (dz[k] * l1w[k] - s1 - x[k] * s2);
    }
    __syncthreads();
    part_range(B * D, i4, n4, lo, hi);
    float* dx = p.dx + (size_t)t * B * D;
    for (int e = lo + threadIdx.x; e < hi; e += NTH) dx[e] = As[(e / D) * lda + e % D];
    if (t == 0) break;  // no z_{-1} to propagate into
    gemm_reg<2, U4>(wt, As, lda, D, red, ct);
    if (threadIdx.x < 512) {
      const float* first = p.first + (size_t)t * B;
      const size_t base = (size_t)(t - 1) * B * S;
      const int idx = threadIdx.x;
      const int b = idx >> 5, c = idx & 31;
      const bool valid = b < B;
      const int bb = valid ? b : 0;
      const size_t o = base + (size_t)bb * S + n0 + c;
      const float ds = (p.dpost ? p.dpost[o] : 0.f) + (1.f - first[bb]) * ct[idx];
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
      if (valid) st_wt(p.dlog + o, dl);
    }
    arrive(p.sync + 3 * NSH * SHW);
  }
}

__global__ void __launch_bounds__(NTH) bwd_kernel(PP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n1 = p.hid / 16, n2 = p.H / 16, n3 = (p.H + p.D) / 16;
  const int bid = blockIdx.x;
  if (bid < n1)
    bwd_G1(p, bid, sm);
  else if (bid < n1 + n2)
    bwd_G2(p, bid - n1, sm);
  else if (bid < n1 + n2 + n3)
    bwd_G3(p, bid - n1 - n2, sm);
  else
    bwd_G4(p, bid - n1 - n2 - n3, sm);
}

__global__ void zero_kernel(u32* w, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) w[i] = 0u;
}

void set_lds(const void* fn, int bytes) { (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes); }

}  // namespace scanp
}  // namespace srl

using namespace srl;
using namespace srl::scanp;

// Words of the hand-off counter block (counters + error word, padded).
int scanp_sync_words() { return ERRW + SHW; }

int scanp_fwd_grid(int S, int H, int hid) { return 3 * H / 16 + hid / 16 + S / 32; }
int scanp_bwd_grid(int S, int D, int H, int hid) { return hid / 16 + H / 16 + (H + D) / 16 + S / 32; }

int scanp_fwd_lds(int S, int D, int H, int hid) {
  (void)S;
  return 4 * std::max(std::max(lds_A(D, H), lds_B(H)), lds_C(hid));
}

int scanp_bwd_lds(int S, int D, int H, int hid) {
  return 4 * std::max(std::max(lds_G1(S), lds_G2(hid)), std::max(lds_G3(H, D), lds_G4(D)));
}

// Shape gate (register tile caps, LDS, residency of every workgroup): mirrors the kernels.
bool scanp_supported(int B, int S, int D, int H, int hid, int C) {
  if (B < 1 || B > 16 || C < 1 || C > 32 || (32 % C) != 0 || S % 32 || D % 16 || H % 16 || hid % 16) return false;
  if (H + D > 16 * 16 * UA || H > 16 * 16 * UB || hid > 16 * 16 * UC) return false;
  if (S > 16 * 16 * U1 || hid > 16 * 16 * U2 || 3 * H > 16 * 16 * U3 || D > 16 * 16 * U4 || H > 64 * GRU_M) return false;
  if (3 * H / 16 > 128) return false;  // Chan combine: two partials per lane
  const int mx = 160 * 1024;
  if (scanp_fwd_lds(S, D, H, hid) > mx || scanp_bwd_lds(S, D, H, hid) > mx) return false;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return scanp_fwd_grid(S, H, hid) <= cus && scanp_bwd_grid(S, D, H, hid) <= cus;
}

void launch_scanp_fwd(const PP& p, hipStream_t st) {
  static bool init = false;
  if (!init) {
    set_lds((const void*)fwd_kernel, 160 * 1024);
    init = true;
  }
  hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, st, p.sync, scanp_sync_words());
  hipLaunchKernelGGL(fwd_kernel, dim3(scanp_fwd_grid(p.S, p.H, p.hid)), dim3(NTH), scanp_fwd_lds(p.S, p.D, p.H, p.hid), st,
                     p);
}

void launch_scanp_bwd(const PP& p, hipStream_t st) {
  static bool init = false;
  if (!init) {
    set_lds((const void*)bwd_kernel, 160 * 1024);
    init = true;
  }
  hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, st, p.sync, scanp_sync_words());
  hipLaunchKernelGGL(bwd_kernel, dim3(scanp_bwd_grid(p.S, p.D, p.H, p.hid)), dim3(NTH), scanp_bwd_lds(p.S, p.D, p.H, p.hid),
                     st, p);
}
