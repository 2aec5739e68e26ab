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

// Phase timestamps (s_memrealtime, 100 MHz): 0 step start, 1 hand-off in, 2 operand ready, 3 GEMM done, 4 published.
// The read is an asm statement with a memory clobber so the compiler can neither move it across the
// phase's memory operations nor merge it with a neighbour.
__device__ __forceinline__ long long prof_clock() {
  long long c;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  return c;
}
#define PROF(role, k)                                                                                 \
  do {                                                                                                \
    if (p.prof && first_wg && threadIdx.x == 0) p.prof[((role) * p.T + t) * 8 + (k)] = prof_clock(); \
  } while (0)

// Register tile caps per phase (K chunks of 16 per wave): host gate mirrors them.
constexpr int UA = 4, UB = 2, UC = 2;           // K = H+D <= 1024, H <= 512, hid <= 512
constexpr int U1 = 4, U2 = 2, U3 = 6, U4 = 2;   // K = S <= 1024, hid <= 512, 3H <= 1536, D <= 512
constexpr int GRU_M = 8;                        // H <= 64 * GRU_M
// "big" form for a wide recurrent input (exp=dreamer_v3_prey: dense 1024, deter / hidden 256): the A tile takes
// K = H + D <= 1280, its LN1 row up to 1024 wide, and G4 (dz = dx Wz, K = D <= 1024) keeps its LN1 adjoint in LDS
// (two passes) with the GEMM reduction aliased onto the dead xh tile (bwd_G4_big)
constexpr int UA_BIG = 5, LN_BIG = 16, U4_BIG = 4;
constexpr int LN_M = 8;                         // D, hid <= 64 * LN_M (row LayerNorms in registers)

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
template <int U = 4>
__device__ __forceinline__ void stage_wt(float* dst, int ld, const float* src, int ls, int nvalid, int cols,
                                         const float* first = nullptr) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, nvalid * ls * 4, 0x00020000);
  const int c4 = cols >> 2, n = 16 * c4;
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
__device__ __forceinline__ bool wait_ctr(const PP& p, int ctr, u32 cnt, u32 rounds, int code, int* flag) {
  u32* sync = p.sync;
  const u32 spin_max = p.spin_max ? p.spin_max : SPIN_MAX;
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
      if (spins >= spin_max) {
        bad = 2;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (s == 0) {
      if (bad == 2) {
        __hip_atomic_store(err, (u32)code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p.health) __hip_atomic_fetch_or(p.health, 1u << (code & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
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
__host__ __device__ inline int lds_A(int D, int H) { return 16 * (H + D + 4) + 2 * D + 4096 + 256 + 32 + 16; }
__host__ __device__ inline int lds_B(int H) { return 16 * (H + 4) + 6 * H + 4096 + 256 + 32 + 16; }
__host__ __device__ inline int lds_C_base(int hid, int S, int C) { return 16 * (hid + 4) + 2 * hid + 8192 + 512 + 16 + 16 * (S / C) + 32 + 1024 + 512; }
// C also keeps its Wz^T column tiles (S rows x 16 columns each, ceil(D/16 / nC) of them) in LDS when they fit:
// the per-step posterior gather then reads LDS instead of L2
__host__ __device__ inline int wz_tiles(int D, int S) { return (D / 16 + S / 32 - 1) / (S / 32); }
__host__ __device__ inline bool wz_in_lds(int hid, int S, int C, int D) {
  return 4 * (lds_C_base(hid, S, C) + wz_tiles(D, S) * S * 16) <= 160 * 1024;
}
__host__ __device__ inline int lds_C(int hid, int S, int C, int D) {
  return lds_C_base(hid, S, C) + (wz_in_lds(hid, S, C, D) ? wz_tiles(D, S) * S * 16 : 0);
}
__host__ __device__ inline int lds_G1(int S) { return 16 * (S + 4) + 4096 + 256 + 16; }
__host__ __device__ inline int lds_G2(int hid) { return 48 * (hid + 4) + 2 * hid + 48 + 4096 + 256 + 1536 + 1792 + 16; }
__host__ __device__ inline int lds_G3(int H) { return 16 * (3 * H + 4) + 64 + 4096 + 256 + 16; }
__host__ __device__ inline int lds_G4(int D) { return 48 * (D + 4) + 2 * D + 48 + 8192 + 512 + 16 + 7 * 512 + 32; }

// ======================================================================= forward roles
// Block ids: A = [0, nA), B = [nA, nA + nB), C = [nA + nB, nA + nB + nC).  Counters: 0 = A, 1 = B, 2 = C.

// A: gx tile = [(1-first) h_{t-1}, act(LN1(xr_t))] Wg^T, plus per-row (mean, M2) of the tile.
template <int UA_, int LNA_>
__device__ __forceinline__ void fwd_A(const PP& p, int a, float* sm) {
  const bool first_wg = a == 0;
  const int B = p.B, D = p.D, H = p.H, HD = H + D, N3 = 3 * H, T = p.T;
  const int nA = N3 / 16, nB = p.hid / 16, nC = p.S / 32;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = HD + 4;
  float* As = sm;
  float* l1w = As + 16 * lda;
  float* l1b = l1w + D;
  float* red = l1b + D;
  float* ct = red + 4096;         // [256] GEMM tile + [32] this step's LN1 row statistics (workgroup 0)
  int* flag = (int*)(ct + 256 + 32);
  WTile<1, UA_> wt;
  wload<1, UA_>(wt, p.Wg + (size_t)a * 16 * HD, HD, HD, w);
  stage_vec(l1w, p.ln1w, D);
  stage_vec(l1b, p.ln1b, D);
  const u32 eB = shard_count(nA, nB), eC = shard_count(nA + nB, nC);
  for (int e = threadIdx.x; e < 16 * H; e += NTH) As[(e / H) * lda + e % H] = 0.f;  // h_{-1} = 0
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    PROF(0, 0);
    if (t > 0) {
      // h_{t-1} is published by B(t-1) before C(t-1) runs: load it while C finishes
      if (!wait_ctr(p, 1, eB, t, 1, flag)) return;
      stage_wt(As, lda, p.hs + (size_t)(t - 1) * B * H, H, B, H, p.first + (size_t)t * B);
      if (!wait_ctr(p, 2, eC, t, 2, flag)) return;
    }
    PROF(0, 1);
    stage_wt(As + H, lda, p.xr + (size_t)t * B * D, D, B, D);
    __syncthreads();
    PROF(0, 5);
    if (w < B) {
      float mu, rs;
      wave_ln_act_row<LNA_>(As + w * lda + H, D, p.eps1, l1w, l1b, p.act1, mu, rs);
      if (a == 0 && lane == 0) {  // stored after the hand-off: a global store before a barrier would be drained there
        ct[256 + w] = mu;
        ct[272 + w] = rs;
      }
    }
    __syncthreads();
    PROF(0, 2);
    gemm_reg<1, UA_>(wt, As, lda, HD, red, ct);
    PROF(0, 3);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      const float x = ct[threadIdx.x];
      const float m = row16_sum(x) * (1.f / 16.f);
      const float q = row16_sum((x - m) * (x - m));
      if (b < B) {
        st_wt(p.gx + ((size_t)t * B + b) * N3 + a * 16 + c, x);
        if (c == 0) st_wt2(p.gst + (((size_t)t * nA + a) * 16 + b) * 2, m, q);
      }
    }
    arrive(p.sync + 0 * NSH * SHW);
    PROF(0, 4);
    if (a == 0 && threadIdx.x < B) {
      p.m1[(size_t)t * B + threadIdx.x] = ct[256 + threadIdx.x];
      p.r1[(size_t)t * B + threadIdx.x] = ct[272 + threadIdx.x];
    }
    {  // the GRU input of step t, read only by the backward: behind the hand-off
      int lo, hi;
      part_range(B * HD, a, nA, lo, hi);
      float* cat = p.cat + (size_t)t * B * HD;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) cat[e] = As[(e / HD) * lda + e % HD];
    }
  }
}

// B: h_t = LNGRU(gx_t, (1-first) h_{t-1}) (row statistics from A's partials, gates straight from gx);
// u tile = h_t Wr1^T + P_t.  h stays in this workgroup's LDS from one step to the next.
__device__ __forceinline__ void fwd_B(const PP& p, int bI, float* sm) {
  const bool first_wg = bI == 0;
  const int B = p.B, H = p.H, N3 = 3 * H, T = p.T, hid = p.hid;
  const int nA = N3 / 16, nB = hid / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = H + 4;
  float* As = sm;
  float* lgw = As + 16 * lda;
  float* lgb = lgw + N3;
  float* red = lgb + N3;
  float* ct = red + 4096;  // [256] GEMM tile + [32] LN-GRU row statistics (workgroup 0)
  int* flag = (int*)(ct + 256 + 32);
  WTile<1, UB> wt;
  wload<1, UB>(wt, p.W1 + (size_t)bI * 16 * H, H, H, w);
  stage_vec(lgw, p.lngw, N3);
  stage_vec(lgb, p.lngb, N3);
  const u32 eA = shard_count(0, nA);
  for (int e = threadIdx.x; e < 16 * H; e += NTH) As[(e / H) * lda + e % H] = 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    PROF(1, 0);
    const int eb = threadIdx.x >> 4, ec = threadIdx.x & 15;
    const size_t eo = ((size_t)t * B + eb) * hid + bI * 16 + ec;
    const float pre = (threadIdx.x < 256 && eb < B) ? p.P[eo] : 0.f;  // epilogue input, loaded behind the wait
    if (!wait_ctr(p, 0, eA, t + 1, 3, flag)) return;
    PROF(1, 1);
    if (w < B) {
      // gate inputs and the nA per-tile (mean, M2) partials, all loads issued before any use: 16-byte
      // write-through (sc1) buffer loads, lane l owning columns 4l..4l+3 (+256 m) of each gate
      const float* gxr = p.gx + ((size_t)t * B + w) * N3;
      const auto grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gxr), (short)0, N3 * 4, 0x00020000);
      constexpr int GV = GRU_M / 4;
      f4 x0[GV], x1[GV], x2[GV];
#pragma unroll
      for (int m = 0; m < GV; ++m) {
        const int j = 4 * lane + 256 * m;
        if (j < H) {
          x0[m] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(grs, j * 4, 0, 16));
          x1[m] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(grs, (H + j) * 4, 0, 16));
          x2[m] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(grs, (2 * H + j) * 4, 0, 16));
        }
      }
      float2 pr[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = lane + 64 * k;
        pr[k] = i < nA ? ld_wt2(p.gst + (((size_t)t * nA + i) * 16 + w) * 2) : make_float2(0.f, 0.f);
      }
      // row statistics of gx from the tile partials (16 columns each): Chan's parallel combine
      const float mu = wave_sum_dpp(pr[0].x + pr[1].x) / nA;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = lane + 64 * k;
        if (i < nA) q += pr[k].y + 16.f * (pr[k].x - mu) * (pr[k].x - mu);
      }
      const float rs = rsqrtf(wave_sum_dpp(q) / N3 + p.epsg);
      const float keep = 1.f - p.first[(size_t)t * B + w];
      float* hr = As + w * lda;
#pragma unroll
      for (int m = 0; m < GV; ++m) {
        const int j = 4 * lane + 256 * m;
        if (j < H) {
          const f4 zr = (x0[m] - mu) * rs * *(const f4*)(lgw + j) + *(const f4*)(lgb + j);
          const f4 zc = (x1[m] - mu) * rs * *(const f4*)(lgw + H + j) + *(const f4*)(lgb + H + j);
          const f4 zu = (x2[m] - mu) * rs * *(const f4*)(lgw + 2 * H + j) + *(const f4*)(lgb + 2 * H + j);
          f4 hv = *(f4*)(hr + j);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = fsig(zr[e]);
            const float c = ftanh(r * zc[e]);
            const float uu = fsig(zu[e] - 1.f);
            hv[e] = uu * c + (1.f - uu) * (keep * hv[e]);
          }
          *(f4*)(hr + j) = hv;
        }
      }
      if (bI == 0 && lane == 0) {  // stored after the hand-off (see fwd_A)
        ct[256 + w] = mu;
        ct[272 + w] = rs;
      }
    }
    __syncthreads();
    PROF(1, 5);
    {
      int lo, hi;
      part_range(B * H, bI, nB, lo, hi);
      float* hs = p.hs + (size_t)t * B * H;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) st_wt(hs + e, As[(e / H) * lda + e % H]);
    }
    PROF(1, 2);
    gemm_reg<1, UB>(wt, As, lda, H, red, ct);
    PROF(1, 3);
    if (threadIdx.x < 256 && eb < B) st_wt(p.u + eo, ct[threadIdx.x] + pre);
    arrive(p.sync + 1 * NSH * SHW);
    PROF(1, 4);
    if (bI == 0 && threadIdx.x < B) {
      p.mg[(size_t)t * B + threadIdx.x] = ct[256 + threadIdx.x];
      p.rg[(size_t)t * B + threadIdx.x] = ct[272 + threadIdx.x];
    }
  }
}

// C: logits tile = act(LN2(u_t)) W2^T + b2 over whole categorical groups; unimix + straight-through
// sample; the sampled one-hot rows of Wz^T are added into xr_{t+1} (device-scope atomics).
__device__ __forceinline__ void fwd_C(const PP& p, int cI, float* sm) {
  const bool first_wg = cI == 0;
  const int B = p.B, S = p.S, D = p.D, H = p.H, hid = p.hid, C = p.C, T = p.T;
  const int nA = 3 * H / 16, nB = hid / 16, nC = S / 32, nseg = S / C;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = hid + 4, n0 = cI * 32;
  float* As = sm;
  float* l2w = As + 16 * lda;
  float* l2b = l2w + hid;
  float* red = l2b + hid;
  float* ct = red + 8192;
  int* flag = (int*)(ct + 512);
  int* selL = flag + 16;  // [B][S / C] sampled rows of the step
  float* cst = (float*)(selL + 16 * nseg);  // [32]: this step's LN2 row statistics (workgroup 0), stored after the hand-off
  float* xr0s = cst + 32;                    // [NTH]: prefetched xr_{t+1} base values (gather threads)
  float* ef1s = xr0s + NTH;                  // [512]: prefetched first_{t+1} flags (epilogue threads)
  // this workgroup's Wz^T column tiles q = cI, cI + nC, ... ([S][16] each), resident for all T steps
  const bool wzl = wz_in_lds(hid, S, C, D);
  float* wzt = ef1s + 512;
  if (wzl) {
    int lt = 0;
    for (int q = cI; q < D / 16; q += nC, ++lt)
      for (int e = threadIdx.x; e < S * 4; e += NTH) {  // float4 per (row, quarter tile)
        const int row = e >> 2, c4 = (e & 3) * 4;
        *(f4*)(wzt + ((size_t)lt * S + row) * 16 + c4) = *(const f4*)(p.WzT + (size_t)row * D + q * 16 + c4);
      }
  }
  WTile<2, UC> wt;
  wload<2, UC>(wt, p.W2 + (size_t)n0 * hid, hid, hid, w);
  stage_vec(l2w, p.ln2w, hid);
  stage_vec(l2b, p.ln2b, hid);
  const u32 eB = shard_count(nA, nB), eC = shard_count(nA + nB, nC);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    PROF(2, 0);
    // epilogue inputs, loaded behind the wait: bias and the uniform of this lane's (row, categorical)
    const int eb = threadIdx.x >> 5, ec = threadIdx.x & 31;
    const bool evalid = threadIdx.x < 512 && eb < B;
    const float ebias = threadIdx.x < 512 ? p.b2[n0 + ec] : 0.f;
    const float euni = evalid ? p.uni[(size_t)t * B * nseg + eb * nseg + (n0 + ec) / C] : 0.f;
    // first_{t+1} and this workgroup's xr_{t+1} columns before the posterior rows are added (a_proj + z0
    // part, written by the host; only this workgroup adds into them): loaded here, off the critical path,
    // parked in LDS (each thread reads back its own entries)
    if (threadIdx.x < 512) ef1s[threadIdx.x] = (evalid && t + 1 < T) ? p.first[(size_t)(t + 1) * B + eb] : 0.f;
    {
      const int gb = threadIdx.x >> 6, gc = (threadIdx.x >> 2) & 15, gq = threadIdx.x & 3;
      xr0s[threadIdx.x] = (t + 1 < T && gb < B && gq == 0 && cI < D / 16) ? p.xr[((size_t)(t + 1) * B + gb) * D + cI * 16 + gc] : 0.f;
    }
    if (!wait_ctr(p, 1, eB, t + 1, 4, flag)) return;
    PROF(2, 1);
    stage_wt(As, lda, p.u + (size_t)t * B * hid, hid, B, hid);
    __syncthreads();
    if (w < B) {
      float mu, rs;
      wave_ln_act_row<LN_M>(As + w * lda, hid, p.eps2, l2w, l2b, p.act2, mu, rs);
      if (cI == 0 && lane == 0) {
        cst[w] = mu;
        cst[16 + w] = rs;
      }
    }
    __syncthreads();
    PROF(2, 2);
    gemm_reg<2, UC>(wt, As, lda, hid, red, ct);
    PROF(2, 3);
    float el = 0.f, em = 0.f, esamp = 0.f;
    if (threadIdx.x < 512) {
      const int k = ec % C;
      const float l = ct[threadIdx.x] + ebias;
      float m = l;
      if (p.alpha > 0.f) {
        const float mx = seg_max_f(l, C);
        const float e = __expf(l - mx);
        const float q = e / seg_sum_f(e, C);
        float pm = (1.f - p.alpha) * q + p.alpha / C;
        pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
        m = logf(pm);
      }
      const float mx2 = seg_max_f(m, C);
      const float e2 = __expf(m - mx2);
      const float pr = e2 / seg_sum_f(e2, C);
      float cdf = pr;  // inclusive prefix sum inside the segment
      if (C == 32) {
        cdf = seg32_scan(cdf);
      } else {
        for (int o = 1; o < C; o <<= 1) {
          const float tt = __shfl_up(cdf, o, C);
          if (k >= o) cdf += tt;
        }
      }
      const float below = cdf < euni * seg_max_f(cdf, C) ? 1.f : 0.f;
      int pick = (int)seg_sum_f(below, C);
      if (pick > C - 1) pick = C - 1;
      el = l;
      em = m;
      esamp = k == pick ? 1.f : 0.f;
      // sampled row of Wz^T per (row, categorical) of step t+1's input; -1: reset row (z0 Wz^T is in xr)
      if (t + 1 < T && k == 0 && evalid) {
        __hip_atomic_store(p.sel + ((size_t)(t + 1) * B + eb) * nseg + (n0 + ec) / C, ef1s[threadIdx.x] == 0.f ? n0 + ec + pick : -1,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    PROF(2, 5);
    if (t + 1 < T) {
      // every C workgroup's samples of step t -> xr_{t+1} column tiles (16 columns of D) gathered from Wz^T:
      // xr = a_proj + first z0 Wz^T (host) + sum over categoricals of the sampled rows.  All 1024 threads
      // gather (row, column, quarter of the categoricals) so every load of a thread is in flight at once.
      arrive(p.sync + 3 * NSH * SHW);
      if (!wait_ctr(p, 3, eC, t + 1, 5, flag)) return;
      PROF(2, 6);
      for (int e = threadIdx.x; e < B * nseg; e += NTH)
        selL[e] = __hip_atomic_load(p.sel + (size_t)(t + 1) * B * nseg + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      float* xr1 = p.xr + (size_t)(t + 1) * B * D;
      const int gb = threadIdx.x >> 6, gc = (threadIdx.x >> 2) & 15, gq = threadIdx.x & 3;
      const int per = (nseg + 3) >> 2;
      for (int q = cI, lt = 0; q < D / 16; q += nC, ++lt) {
        const int col = q * 16 + gc;
        float x = 0.f;
        if (gb < B) {
          const int* sr = selL + gb * nseg;
          if (wzl) {
            const float* tile = wzt + (size_t)lt * S * 16 + gc;
#pragma unroll 8
            for (int g = gq * per; g < min(nseg, gq * per + per); ++g) {
              const int row = sr[g];
              if (row >= 0) x += tile[row * 16];
            }
          } else {
#pragma unroll 8
            for (int g = gq * per; g < min(nseg, gq * per + per); ++g) {
              const int row = sr[g];
              if (row >= 0) x += p.WzT[(size_t)row * D + col];
            }
          }
        }
        x += dpp_f<0xB1>(x);  // quad sum (quad_perm [1,0,3,2], [2,3,0,1])
        x += dpp_f<0x4E>(x);
        if (gb < B && gq == 0) {
          float* d = xr1 + (size_t)gb * D + col;
          st_wt(d, (lt == 0 ? xr0s[threadIdx.x] : *d) + x);
        }
      }
      PROF(2, 7);
    }
    arrive(p.sync + 2 * NSH * SHW);
    PROF(2, 4);
    if (cI == 0 && threadIdx.x < B) {
      p.m2[(size_t)t * B + threadIdx.x] = cst[threadIdx.x];
      p.r2[(size_t)t * B + threadIdx.x] = cst[16 + threadIdx.x];
    }
    // outputs read only after the launch: issued behind the hand-off
    if (evalid) {
      const size_t o = (size_t)t * B * S + (size_t)eb * S + n0 + ec;
      p.logits[o] = el;
      p.mixed[o] = em;
      p.samples[o] = esamp;
      if (t + 1 < T) {
        const float f1 = ef1s[threadIdx.x];
        p.zm[o + (size_t)B * S] = (1.f - f1) * esamp + f1 * p.z0[n0 + ec];
      }
    }
    {
      int lo, hi;
      part_range(B * hid, cI, nC, lo, hi);
      float* v = p.v + (size_t)t * B * hid;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) v[e] = As[(e / hid) * lda + e % hid];
    }
  }
}

template <int UA_, int LNA_>
__device__ __forceinline__ void fwd_body(const PP& p, float* sm) {
  const int bid = blockIdx.x;
  const int nA = 3 * p.H / 16, nB = p.hid / 16;
  if (bid < nA)
    fwd_A<UA_, LNA_>(p, bid, sm);
  else if (bid < nA + nB)
    fwd_B(p, bid - nA, sm);
  else
    fwd_C(p, bid - nA - nB, sm);
}

__global__ void __launch_bounds__(NTH) fwd_kernel(PP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  fwd_body<UA, LN_M>(p, sm);
}

__global__ void __launch_bounds__(NTH) fwd_kernel_big(PP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  fwd_body<UA_BIG, LN_BIG>(p, sm);
}

// ======================================================================= backward roles
// Block ids: G1 = [0, n1), G2 = [n1, +n2), G3 = [n1 + n2, +n3), G4 = [n1 + n2 + n3, +n4).
// Counters: 0 = G1, 1 = G2, 2 = G3, 3 = G4.  Inputs the forward saved are staged BEFORE each wait.

// G1: dv_t = dlog_t W2 (K = S).
__device__ __forceinline__ void bwd_G1(const PP& p, int i, float* sm) {
  const bool first_wg = i == 0;
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
    PROF(3, 0);
    if (t < T - 1 && !wait_ctr(p, 3, e4, T - 1 - t, 11, flag)) return;
    PROF(3, 1);
    stage_wt(As, lda, p.dlog + (size_t)t * B * S, S, B, S);
    __syncthreads();
    PROF(3, 2);
    gemm_reg<1, U1>(wt, As, lda, S, red, ct);
    PROF(3, 3);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (b < B) st_wt(p.dv + ((size_t)t * B + b) * hid + i * 16 + c, ct[threadIdx.x]);
    }
    arrive(p.sync + 0 * NSH * SHW);
    PROF(3, 4);
  }
}

// G2: du_t = LN2'(dv_t) (+ LN2 parameter partials); DH_t tile = DH_t + du_t Wr1 (K = hid) is final for
// this workgroup's 16 h columns, so the LN-GRU adjoint of those columns is formed here: dz * gamma of
// the three gates (handed to G3 with the row partial sums the LayerNorm adjoint needs), the LN-GRU
// parameter partials, and the gate's direct path into DH_{t-1}.
__device__ __forceinline__ void bwd_G2(const PP& p, int i, float* sm) {
  const bool first_wg = i == 0;
  const int B = p.B, H = p.H, hid = p.hid, T = p.T, N3 = 3 * H, HD = H + p.D;
  const int n1 = hid / 16, n2 = H / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = hid + 4;
  float* As = sm;
  float* R = As + 16 * lda;
  float* l2w = R + 16 * lda;
  float* l2b = l2w + hid;
  float* st = l2b + hid;
  float* red = st + 48;
  float* ct = red + 4096;
  float* gsc = ct + 256;  // [16 rows][6][16 columns]: LN-GRU parameter partial terms
  float* pre = gsc + 1536;  // [7][256]: forward values of this thread's GRU adjoint element
  int* flag = (int*)(pre + 1792);
  float* X2 = (float*)(flag + 16);  // [16][hid + 4]: du (As keeps xh for the LN2 parameter partials)
  WTile<1, U2> wt;
  wload<1, U2>(wt, p.W1T + (size_t)i * 16 * hid, hid, hid, w);
  stage_vec(l2w, p.ln2w, hid);
  stage_vec(l2b, p.ln2b, hid);
  const u32 e1 = shard_count(0, n1);
  // thread -> (row eb, h column j) of the GRU adjoint; gate parameters fixed per thread
  const int eb = threadIdx.x >> 4, ec = threadIdx.x & 15, j = i * 16 + ec;
  const bool eok = threadIdx.x < 256;
  float gw0 = 0.f, gw1 = 0.f, gw2 = 0.f, gb0 = 0.f, gb1 = 0.f, gb2 = 0.f;
  if (eok) {
    gw0 = p.lngw[j], gw1 = p.lngw[H + j], gw2 = p.lngw[2 * H + j];
    gb0 = p.lngb[j], gb1 = p.lngb[H + j], gb2 = p.lngb[2 * H + j];
  }
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    PROF(4, 0);
    stage(As, lda, p.u + (size_t)t * B * hid, hid, B, hid);
    // forward values of the GRU adjoint: loaded behind the wait
    const bool rv = eok && eb < B;
    if (eok) {  // parked in LDS, not registers: they are consumed after the LN2 adjoint and the GEMM
      const size_t gr = ((size_t)t * B + (rv ? eb : 0)) * N3;
      pre[threadIdx.x] = rv ? p.gx[gr + j] : 0.f;
      pre[256 + threadIdx.x] = rv ? p.gx[gr + H + j] : 0.f;
      pre[512 + threadIdx.x] = rv ? p.gx[gr + 2 * H + j] : 0.f;
      pre[768 + threadIdx.x] = rv ? p.cat[((size_t)t * B + eb) * HD + j] : 0.f;
      pre[1024 + threadIdx.x] = rv ? p.mg[(size_t)t * B + eb] : 0.f;
      pre[1280 + threadIdx.x] = rv ? p.rg[(size_t)t * B + eb] : 0.f;
      pre[1536 + threadIdx.x] = (rv && t > 0) ? 1.f - p.first[(size_t)t * B + eb] : 0.f;
    }
    if (threadIdx.x < B) {  // LN2 row statistics of the forward (read after the wait from LDS)
      st[threadIdx.x] = p.m2[(size_t)t * B + threadIdx.x];
      st[16 + threadIdx.x] = p.r2[(size_t)t * B + threadIdx.x];
    }
    if (!wait_ctr(p, 0, e1, T - t, 12, flag)) return;
    PROF(4, 1);
    stage_wt(R, lda, p.dv + (size_t)t * B * hid, hid, B, hid);
    __syncthreads();
    PROF(4, 5);
    float xh[LN_M], dzr[LN_M], s1 = 0.f, s2 = 0.f, rsw = 0.f;
    if (w < B) {
      const float m2 = st[w];
      rsw = st[16 + w];
      wave_ln_bwd_regs<LN_M>(As + w * lda, R + w * lda, l2w, l2b, hid, p.act2, m2, rsw, xh, dzr, s1, s2);
    }
    PROF(4, 6);
    // du into X2 (As keeps xh, R keeps dz): the LN2 parameter partials and the du stores (weight-gradient
    // inputs only) run after this step's hand-off
    if (w < B) wave_ln_bwd_finish<LN_M>(X2 + w * lda, l2w, hid, rsw, s1, s2, xh, dzr);
    __syncthreads();
    PROF(4, 7);
    PROF(4, 2);
    gemm_reg<1, U2>(wt, X2, lda, hid, red, ct);
    PROF(4, 3);
    if (eok) {
      const float go = rv ? ld_wt(p.DH + ((size_t)t * B + eb) * H + j) + ct[threadIdx.x] : 0.f;
      const float x0 = pre[threadIdx.x], x1 = pre[256 + threadIdx.x], x2 = pre[512 + threadIdx.x];
      const float hp = pre[768 + threadIdx.x], mu = pre[1024 + threadIdx.x], rsg = pre[1280 + threadIdx.x];
      const float keep = pre[1536 + threadIdx.x];
      const float a0 = (x0 - mu) * rsg, a1 = (x1 - mu) * rsg, a2 = (x2 - mu) * rsg;
      const float r = fsig(a0 * gw0 + gb0), zc = a1 * gw1 + gb1, c = ftanh(r * zc), u = fsig(a2 * gw2 + gb2 - 1.f);
      const float dua = go * (c - hp);
      const float da = go * u * (1.f - c * c);
      const float dz2 = dua * u * (1.f - u);
      const float dz1 = da * r;
      const float dz0 = da * zc * r * (1.f - r);
      const float d0 = dz0 * gw0, d1 = dz1 * gw1, d2 = dz2 * gw2;
      const float s1p = row16_sum(d0 + d1 + d2), s2p = row16_sum(d0 * a0 + d1 * a1 + d2 * a2);
      float* g = gsc + eb * 96 + ec;
      g[0] = dz0 * a0;
      g[16] = dz0;
      g[32] = dz1 * a1;
      g[48] = dz1;
      g[64] = dz2 * a2;
      g[80] = dz2;
      if (rv) {
        float* dZ = p.dZ + ((size_t)t * B + eb) * N3;
        st_wt(dZ + j, d0);
        st_wt(dZ + H + j, d1);
        st_wt(dZ + 2 * H + j, d2);
        if (ec == 0) st_wt2(p.sst + (((size_t)t * n2 + i) * 16 + eb) * 2, s1p, s2p);
        if (t > 0) {  // direct path h_{t-1} -> h_t through the update gate
          float* d = p.DH + ((size_t)(t - 1) * B + eb) * H + j;
          st_wt(d, ld_wt(d) + keep * go * (1.f - u));
        }
      }
    }
    arrive(p.sync + 1 * NSH * SHW);  // (its barrier also orders the gsc writes before the reads below)
    PROF(4, 4);
    if (threadIdx.x < 96) {  // LN-GRU parameter partials of this workgroup's 3 x 16 gate columns
      const int k = threadIdx.x >> 4, c = threadIdx.x & 15;
      float a = 0.f;
      for (int b = 0; b < B; ++b) a += gsc[b * 96 + k * 16 + c];
      const int col = (k >> 1) * H + i * 16 + c;
      (k & 1 ? p.pgb : p.pgg)[(size_t)t * p.ldp + col] = a;
    }
    {  // behind the hand-off: LN2 parameter partials and du (weight-gradient inputs)
      int lo, hi;
      part_range(hid, i, n2, lo, hi);
      ln_param_partials(As, lda, R, lda, B, lo, hi, p.p2g + (size_t)t * p.ldp, p.p2b + (size_t)t * p.ldp);
      part_range(B * hid, i, n2, lo, hi);
      float* du = p.du + (size_t)t * B * hid;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) du[e] = X2[(e / hid) * lda + e % hid];
      __syncthreads();  // As / R / X2 are rewritten by the next step
    }
  }
}

// G3: dgx_t = rs (dz*gamma - mean(dz*gamma) - xh mean(dz*gamma*xh)) from G2's pieces; dcat tile =
// dgx_t Wg (K = 3H); h columns of the tile go straight into DH_{t-1}, feature columns to G4.
__device__ __forceinline__ void bwd_G3(const PP& p, int i3, float* sm) {
  const bool first_wg = i3 == 0;
  const int B = p.B, H = p.H, D = p.D, HD = H + D, N3 = 3 * H, T = p.T;
  const int n2 = H / 16, n3 = HD / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lda = N3 + 4, n0 = i3 * 16;
  float* As = sm;
  float* rowst = As + 16 * lda;  // [16][4]: mu, rs, mean(dz*g), mean(dz*g*xh)
  float* red = rowst + 64;
  float* ct = red + 4096;
  int* flag = (int*)(ct + 256);
  WTile<1, U3> wt;
  wload<1, U3>(wt, p.WgT + (size_t)n0 * N3, N3, N3, w);
  const u32 e2 = shard_count(p.hid / 16, n2);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    PROF(5, 0);
    stage(As, lda, p.gx + (size_t)t * B * N3, N3, B, N3);
    if (threadIdx.x < B) {
      rowst[threadIdx.x * 4] = p.mg[(size_t)t * B + threadIdx.x];
      rowst[threadIdx.x * 4 + 1] = p.rg[(size_t)t * B + threadIdx.x];
    }
    if (!wait_ctr(p, 1, e2, T - t, 13, flag)) return;
    PROF(5, 1);
    if (w < B) {
      const float2 sp = lane < n2 ? ld_wt2(p.sst + (((size_t)t * n2 + lane) * 16 + w) * 2) : make_float2(0.f, 0.f);
      const float m1 = wave_sum_dpp(sp.x) / N3, m2 = wave_sum_dpp(sp.y) / N3;
      if (lane == 0) {
        rowst[w * 4 + 2] = m1;
        rowst[w * 4 + 3] = m2;
      }
    }
    __syncthreads();
    PROF(5, 5);
    {
      const int c4 = N3 >> 2, n = B * c4;
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.dZ + (size_t)t * B * N3, (short)0, B * N3 * 4, 0x00020000);
      for (int e = threadIdx.x; e < n; e += NTH) {
        const int r = e / c4, k = (e - r * c4) << 2;
        const f4 d = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (r * N3 + k) * 4, 0, 16));
        const float mu = rowst[r * 4], rg = rowst[r * 4 + 1], m1 = rowst[r * 4 + 2], m2 = rowst[r * 4 + 3];
        f4* x = (f4*)(As + r * lda + k);
        *x = rg * (d - m1 - (*x - mu) * (rg * m2));
      }
    }
    __syncthreads();
    PROF(5, 6);
    PROF(5, 2);
    gemm_reg<1, U3>(wt, As, lda, N3, red, ct);
    PROF(5, 3);
    if (threadIdx.x < 256) {
      const int b = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (b < B) {
        const float v = ct[threadIdx.x];
        if (n0 >= H) {
          st_wt(p.dcat + ((size_t)t * B + b) * HD + n0 + c, v);
        } else if (t > 0) {
          float* d = p.DH + ((size_t)(t - 1) * B + b) * H + n0 + c;
          st_wt(d, ld_wt(d) + (1.f - p.first[(size_t)t * B + b]) * v);
        }
      }
    }
    arrive(p.sync + 2 * NSH * SHW);
    PROF(5, 4);
    {  // behind the hand-off: dgx (weight-gradient input)
      int lo, hi;
      part_range(B * N3, i3, n3, lo, hi);
      float* dgx = p.dgx + (size_t)t * B * N3;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) dgx[e] = As[(e / N3) * lda + e % N3];
      __syncthreads();  // As is restaged by the next step
    }
  }
}

// G4: dx_t = LN1'(dcat_x) (+ LN1 parameter partials); dz = dx_t Wz (K = D);
// dlog_{t-1} = unimix_ST'(logits_{t-1}; dmixed, d_post + (1-first_t) dz).
__device__ __forceinline__ void bwd_G4(const PP& p, int i4, float* sm) {
  const bool first_wg = i4 == 0;
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
  // [7][512]: the unimix adjoint's forward-only terms q, pm, pr, clamped and its epilogue inputs dmixed,
  // d_post, keep (parked in LDS: the kernel is at the 128-VGPR cap); [32]: LN1 row statistics
  float* fpre = (float*)(flag + 16);
  float* X2 = fpre + 7 * 512 + 32;     // [16][D + 4]: dx (As keeps xh for the LN1 parameter partials)
  WTile<2, U4> wt;
  wload<2, U4>(wt, p.WzT + (size_t)n0 * D, D, D, w);
  stage_vec(l1w, p.ln1w, D);
  stage_vec(l1b, p.ln1b, D);
  const u32 e3 = shard_count(p.hid / 16 + H / 16, n3);
  // LN1 row statistics of the forward, one step ahead (loaded at the end of the previous step, into LDS)
  if (threadIdx.x < B) {
    fpre[3584 + threadIdx.x] = p.m1[(size_t)(T - 1) * B + threadIdx.x];
    fpre[3600 + threadIdx.x] = p.r1[(size_t)(T - 1) * B + threadIdx.x];
  }
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    PROF(6, 0);
    stage(As, lda, p.xr + (size_t)t * B * D, D, B, D);
    // epilogue inputs (forward values / external gradients of step t-1): loaded behind the wait
    const int eb = threadIdx.x >> 5, ec = threadIdx.x & 31, ebb = eb < B ? eb : 0;
    const size_t eo = (size_t)(t > 0 ? t - 1 : 0) * B * S + (size_t)ebb * S + n0 + ec;
    const bool eok = threadIdx.x < 512 && t > 0;
    const float el = eok ? p.logits[eo] : 0.f;
    if (threadIdx.x < 512) {
      fpre[2048 + threadIdx.x] = eok ? p.dmixed[eo] : 0.f;
      fpre[2560 + threadIdx.x] = (eok && p.dpost) ? p.dpost[eo] : 0.f;
      fpre[3072 + threadIdx.x] = eok ? 1.f - p.first[(size_t)t * B + ebb] : 0.f;
    }
    if (threadIdx.x < 512 && t > 0) {
      // the unimix / straight-through adjoint's terms that depend on the forward logits only, computed
      // before the wait (off the G3 -> G4 -> G1 critical path) and parked in LDS
      float q = 0.f, pm = 0.f, m = el, cl = 0.f;
      if (p.alpha > 0.f) {
        const float mx = seg_max_f(el, C);
        const float e = __expf(el - mx);
        q = e / seg_sum_f(e, C);
        pm = (1.f - p.alpha) * q + p.alpha / C;
        cl = (pm <= FEPS || pm >= 1.f - FEPS) ? 1.f : 0.f;
        m = logf(fminf(fmaxf(pm, FEPS), 1.f - FEPS));
      }
      const float mx2 = seg_max_f(m, C);
      const float e2 = __expf(m - mx2);
      fpre[threadIdx.x] = q;
      fpre[512 + threadIdx.x] = pm;
      fpre[1024 + threadIdx.x] = e2 / seg_sum_f(e2, C);
      fpre[1536 + threadIdx.x] = cl;
    }
    if (!wait_ctr(p, 2, e3, T - t, 14, flag)) return;
    PROF(6, 1);
    stage_wt(R, lda, p.dcat + (size_t)t * B * HD + H, HD, B, D);
    __syncthreads();
    PROF(6, 5);
    float xh[LN_M], dzr[LN_M], s1 = 0.f, s2 = 0.f, rsw = 0.f;
    if (w < B) {
      const float mu = fpre[3584 + w];
      rsw = fpre[3600 + w];
      wave_ln_bwd_regs<LN_M>(As + w * lda, R + w * lda, l1w, l1b, D, p.act1, mu, rsw, xh, dzr, s1, s2);
    }
    PROF(6, 6);
    // dx into X2 (As keeps xh, R keeps dz): the LN1 parameter partials and the dx stores (weight-gradient
    // inputs only) run after this step's hand-off
    if (w < B) wave_ln_bwd_finish<LN_M>(X2 + w * lda, l1w, D, rsw, s1, s2, xh, dzr);
    __syncthreads();
    auto tail = [&]() {
      int lo, hi;
      part_range(D, i4, n4, lo, hi);
      ln_param_partials(As, lda, R, lda, B, lo, hi, p.p1g + (size_t)t * p.ldp, p.p1b + (size_t)t * p.ldp);
      part_range(B * D, i4, n4, lo, hi);
      float* dx = p.dx + (size_t)t * B * D;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) dx[e] = X2[(e / D) * lda + e % D];
      __syncthreads();  // As / R / X2 are rewritten by the next step
    };
    if (t == 0) {  // no z_{-1} to propagate into
      tail();
      break;
    }
    PROF(6, 2);
    gemm_reg<2, U4>(wt, X2, lda, D, red, ct);
    PROF(6, 3);
    if (threadIdx.x < 512) {
      const float ds = fpre[2560 + threadIdx.x] + fpre[3072 + threadIdx.x] * ct[threadIdx.x];
      const float q = fpre[threadIdx.x], pm = fpre[512 + threadIdx.x], pr = fpre[1024 + threadIdx.x];
      const bool clamped = fpre[1536 + threadIdx.x] != 0.f;
      float gm = fpre[2048 + threadIdx.x];
      const float dot = seg_sum_f(pr * ds, C);
      gm += pr * (ds - dot);
      float dl;
      if (p.alpha > 0.f) {
        const float wv = clamped ? 0.f : (1.f - p.alpha) * gm / pm;
        dl = q * (wv - seg_sum_f(q * wv, C));
      } else {
        dl = gm;
      }
      if (eb < B) st_wt(p.dlog + eo, dl);
    }
    PROF(6, 7);
    arrive(p.sync + 3 * NSH * SHW);
    PROF(6, 4);
    tail();
    if (threadIdx.x < B) {  // the next (earlier) step's LN1 row statistics
      fpre[3584 + threadIdx.x] = p.m1[(size_t)(t - 1) * B + threadIdx.x];
      fpre[3600 + threadIdx.x] = p.r1[(size_t)(t - 1) * B + threadIdx.x];
    }
  }
}

// G4 for a wide recurrent input (D <= 1024): the same adjoint as bwd_G4, laid out for 160 KB of LDS -
//   LN1' in two LDS passes (wave_ln_bwd_prep: x <- xh, dy <- dz in place) instead of registers, the LN1 parameter
//   partials taken before the GEMM, dx written over dz in R (the GEMM's A operand and, behind the hand-off, the
//   stored weight-gradient input), the GEMM's cross-wave reduction in the then-dead xh tile As.
// LDS (floats): As [16][D+4] | R [16][D+4] | l1w [D] | l1b [D] | st 48 | ct 512 | flag 16 | fpre 7 * 512 + 32.
__host__ __device__ inline int lds_G4_big(int D) { return 32 * (D + 4) + 2 * D + 48 + 512 + 16 + 7 * 512 + 32; }

__device__ __forceinline__ void bwd_G4_big(const PP& p, int i4, float* sm) {
  const bool first_wg = i4 == 0;
  const int B = p.B, S = p.S, D = p.D, H = p.H, HD = H + D, C = p.C, T = p.T;
  const int n3 = HD / 16, n4 = S / 32;
  const int w = threadIdx.x >> 6, lda = D + 4, n0 = i4 * 32;
  float* As = sm;
  float* R = As + 16 * lda;
  float* l1w = R + 16 * lda;
  float* l1b = l1w + D;
  float* st = l1b + D;
  float* ct = st + 48;
  int* flag = (int*)(ct + 512);
  float* fpre = (float*)(flag + 16);  // as bwd_G4: [7][512] unimix-adjoint terms, [32] LN1 row statistics
  float* red = As;                    // [16 waves][16][32]: 8192 floats <= 16 (D + 4)
  WTile<2, U4_BIG> wt;
  wload<2, U4_BIG>(wt, p.WzT + (size_t)n0 * D, D, D, w);
  stage_vec(l1w, p.ln1w, D);
  stage_vec(l1b, p.ln1b, D);
  const u32 e3 = shard_count(p.hid / 16 + H / 16, n3);
  if (threadIdx.x < B) {
    fpre[3584 + threadIdx.x] = p.m1[(size_t)(T - 1) * B + threadIdx.x];
    fpre[3600 + threadIdx.x] = p.r1[(size_t)(T - 1) * B + threadIdx.x];
  }
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    PROF(6, 0);
    stage(As, lda, p.xr + (size_t)t * B * D, D, B, D);
    const int eb = threadIdx.x >> 5, ec = threadIdx.x & 31, ebb = eb < B ? eb : 0;
    const size_t eo = (size_t)(t > 0 ? t - 1 : 0) * B * S + (size_t)ebb * S + n0 + ec;
    const bool eok = threadIdx.x < 512 && t > 0;
    const float el = eok ? p.logits[eo] : 0.f;
    if (threadIdx.x < 512) {
      fpre[2048 + threadIdx.x] = eok ? p.dmixed[eo] : 0.f;
      fpre[2560 + threadIdx.x] = (eok && p.dpost) ? p.dpost[eo] : 0.f;
      fpre[3072 + threadIdx.x] = eok ? 1.f - p.first[(size_t)t * B + ebb] : 0.f;
    }
    if (threadIdx.x < 512 && t > 0) {
      float q = 0.f, pm = 0.f, m = el, cl = 0.f;
      if (p.alpha > 0.f) {
        const float mx = seg_max_f(el, C);
        const float e = __expf(el - mx);
        q = e / seg_sum_f(e, C);
        pm = (1.f - p.alpha) * q + p.alpha / C;
        cl = (pm <= FEPS || pm >= 1.f - FEPS) ? 1.f : 0.f;
        m = logf(fminf(fmaxf(pm, FEPS), 1.f - FEPS));
      }
      const float mx2 = seg_max_f(m, C);
      const float e2 = __expf(m - mx2);
      fpre[threadIdx.x] = q;
      fpre[512 + threadIdx.x] = pm;
      fpre[1024 + threadIdx.x] = e2 / seg_sum_f(e2, C);
      fpre[1536 + threadIdx.x] = cl;
    }
    if (!wait_ctr(p, 2, e3, T - t, 14, flag)) return;
    PROF(6, 1);
    stage_wt(R, lda, p.dcat + (size_t)t * B * HD + H, HD, B, D);
    __syncthreads();
    PROF(6, 5);
    float s1 = 0.f, s2 = 0.f, rsw = 0.f;
    if (w < B) {
      rsw = fpre[3600 + w];
      wave_ln_bwd_prep(As + w * lda, R + w * lda, l1w, l1b, D, p.act1, fpre[3584 + w], rsw, s1, s2);
    }
    __syncthreads();
    {  // LN1 parameter partials of this workgroup's column range (xh in As, dz in R), then dx over dz
      int lo, hi;
      part_range(D, i4, n4, lo, hi);
      ln_param_partials(As, lda, R, lda, B, lo, hi, p.p1g + (size_t)t * p.ldp, p.p1b + (size_t)t * p.ldp);
    }
    __syncthreads();
    if (w < B) {
      const int s = threadIdx.x & 63;
      float* xr = As + w * lda;
      float* dr = R + w * lda;
      for (int k = s; k < D; k += 64) dr[k] = rsw * (dr[k] * l1w[k] - s1 - xr[k] * s2);
    }
    __syncthreads();
    PROF(6, 6);
    auto tail = [&]() {  // dx (weight-gradient input) behind the hand-off
      int lo, hi;
      part_range(B * D, i4, n4, lo, hi);
      float* dx = p.dx + (size_t)t * B * D;
      for (int e = lo + threadIdx.x; e < hi; e += NTH) dx[e] = R[(e / D) * lda + e % D];
      __syncthreads();  // As / R are rewritten by the next step
    };
    if (t == 0) {
      tail();
      break;
    }
    PROF(6, 2);
    gemm_reg<2, U4_BIG>(wt, R, lda, D, red, ct);
    PROF(6, 3);
    if (threadIdx.x < 512) {
      const float ds = fpre[2560 + threadIdx.x] + fpre[3072 + threadIdx.x] * ct[threadIdx.x];
      const float q = fpre[threadIdx.x], pm = fpre[512 + threadIdx.x], pr = fpre[1024 + threadIdx.x];
      const bool clamped = fpre[1536 + threadIdx.x] != 0.f;
      float gm = fpre[2048 + threadIdx.x];
      const float dot = seg_sum_f(pr * ds, C);
      gm += pr * (ds - dot);
      float dl;
      if (p.alpha > 0.f) {
        const float wv = clamped ? 0.f : (1.f - p.alpha) * gm / pm;
        dl = q * (wv - seg_sum_f(q * wv, C));
      } else {
        dl = gm;
      }
      if (eb < B) st_wt(p.dlog + eo, dl);
    }
    PROF(6, 7);
    arrive(p.sync + 3 * NSH * SHW);
    PROF(6, 4);
    tail();
    if (threadIdx.x < B) {
      fpre[3584 + threadIdx.x] = p.m1[(size_t)(t - 1) * B + threadIdx.x];
      fpre[3600 + threadIdx.x] = p.r1[(size_t)(t - 1) * B + threadIdx.x];
    }
  }
}

template <bool BIG>
__device__ __forceinline__ void bwd_body(const PP& p, float* sm) {
  const int n1 = p.hid / 16, n2 = p.H / 16, n3 = (p.H + p.D) / 16;
  const int bid = blockIdx.x;
  if (bid < n1)
    bwd_G1(p, bid, sm);
  else if (bid < n1 + n2)
    bwd_G2(p, bid - n1, sm);
  else if (bid < n1 + n2 + n3)
    bwd_G3(p, bid - n1 - n2, sm);
  else if constexpr (BIG)
    bwd_G4_big(p, bid - n1 - n2 - n3, sm);
  else
    bwd_G4(p, bid - n1 - n2 - n3, sm);
}

__global__ void __launch_bounds__(NTH) bwd_kernel(PP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  bwd_body<false>(p, sm);
}

__global__ void __launch_bounds__(NTH) bwd_kernel_big(PP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  bwd_body<true>(p, sm);
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

// Form of a shape: 0 = the register-tile form (D <= 512), 1 = the wide-input form (fwd_kernel_big / bwd_kernel_big,
// H + D <= 1280, D <= 1024), -1 = not covered.
static bool scanp_caps(int B, int S, int D, int H, int hid, int C, bool big) {
  if (B < 1 || B > 16 || C < 1 || C > 32 || (32 % C) != 0 || S % 32 || D % 16 || H % 16 || hid % 16) return false;
  if (H > 16 * 16 * UB || hid > 16 * 16 * UC) return false;
  if (S > 16 * 16 * U1 || hid > 16 * 16 * U2 || 3 * H > 16 * 16 * U3 || H > 64 * GRU_M) return false;
  if (hid > 64 * LN_M) return false;
  if (3 * H / 16 > 128) return false;  // Chan combine: two partials per lane
  if (!big) return H + D <= 16 * 16 * UA && D <= 16 * 16 * U4 && D <= 64 * LN_M;
  return H + D <= 16 * 16 * UA_BIG && D <= 16 * 16 * U4_BIG && D <= 64 * LN_BIG && 16 * (D + 4) >= 8192;
}

int scanp_fwd_lds(int S, int D, int H, int hid, int C) {
  return 4 * std::max(std::max(lds_A(D, H), lds_B(H)), lds_C(hid, S, C, D));
}

static int scanp_bwd_lds_form(int S, int D, int H, int hid, bool big) {
  return 4 * std::max(std::max(lds_G1(S), lds_G2(hid)), std::max(lds_G3(H), big ? lds_G4_big(D) : lds_G4(D)));
}

int scanp_bwd_lds(int S, int D, int H, int hid) {
  return scanp_bwd_lds_form(S, D, H, hid, !scanp_caps(1, S, D, H, hid, 1, false));
}

static bool scanp_resident(int S, int D, int H, int hid, int C, bool big) {
  const int mx = 160 * 1024;
  if (scanp_fwd_lds(S, D, H, hid, C) > mx || scanp_bwd_lds_form(S, D, H, hid, big) > mx) return false;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // co-residency: every workgroup must be resident at once (they hand off to each other), so the grid
  // must fit the occupancy the compiler/runtime report for these kernels at their LDS size - not just
  // the CU count.  Another process or stream sharing the CUs can still starve a wave: the bounded
  // waits + the sticky health word (check_scan_health on the host) catch that at run time.
  const void* fk = big ? (const void*)fwd_kernel_big : (const void*)fwd_kernel;
  const void* bk = big ? (const void*)bwd_kernel_big : (const void*)bwd_kernel;
  set_lds(fk, 160 * 1024);
  set_lds(bk, 160 * 1024);
  int occ_f = 0, occ_b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_f, fk, NTH, scanp_fwd_lds(S, D, H, hid, C)) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_b, bk, NTH, scanp_bwd_lds_form(S, D, H, hid, big)) != hipSuccess)
    return false;
  return scanp_fwd_grid(S, H, hid) <= cus * occ_f && scanp_bwd_grid(S, D, H, hid) <= cus * occ_b;
}

int scanp_form(int B, int S, int D, int H, int hid, int C) {
  // memo of the last shapes asked (every launch asks; the residency query is a host API round trip)
  struct Q { int key[7]; int form; };
  static Q memo[8];
  static int nmemo = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const int key[7] = {B, S, D, H, hid, C, dev};
  for (int i = 0; i < nmemo; ++i)
    if (std::equal(key, key + 7, memo[i].key)) return memo[i].form;
  int form = -1;
  for (int f = 0; f < 2 && form < 0; ++f)
    if (scanp_caps(B, S, D, H, hid, C, f == 1) && scanp_resident(S, D, H, hid, C, f == 1)) form = f;
  Q& q = memo[nmemo < 8 ? nmemo++ : 7];
  std::copy(key, key + 7, q.key);
  q.form = form;
  return form;
}

// Shape gate (register tile caps, LDS, residency of every workgroup): mirrors the kernels.
bool scanp_supported(int B, int S, int D, int H, int hid, int C) { return scanp_form(B, S, D, H, hid, C) >= 0; }

void launch_scanp_fwd(const PP& p, hipStream_t st) {
  const bool big = scanp_form(p.B, p.S, p.D, p.H, p.hid, p.C) == 1;
  hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, st, p.sync, scanp_sync_words());
  hipLaunchKernelGGL(big ? fwd_kernel_big : fwd_kernel, dim3(scanp_fwd_grid(p.S, p.H, p.hid)), dim3(NTH),
                     scanp_fwd_lds(p.S, p.D, p.H, p.hid, p.C), st, p);
}

void launch_scanp_bwd(const PP& p, hipStream_t st) {
  const bool big = scanp_form(p.B, p.S, p.D, p.H, p.hid, p.C) == 1;
  hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, st, p.sync, scanp_sync_words());
  hipLaunchKernelGGL(big ? bwd_kernel_big : bwd_kernel, dim3(scanp_bwd_grid(p.S, p.D, p.H, p.hid)), dim3(NTH),
                     scanp_bwd_lds_form(p.S, p.D, p.H, p.hid, big), st, p);
}
