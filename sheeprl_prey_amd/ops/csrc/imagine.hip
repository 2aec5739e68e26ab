// DreamerV3 imagination rollout (discrete actors) as ONE persistent launch.
//
// Reference loop: dreamer_v3.py:235-257 over RSSM.imagination (agent.py:439-455) and Actor.forward
// (agent.py:682-739): per imagined step the actor MLP + heads sample an action, the recurrent model
// (Linear -> LN -> act -> LayerNormGRUCell) advances h, and the transition MLP samples the next prior.
// The discrete objective back-propagates only through log-probs of detached actions, so the rollout
// needs no autograd graph: it is a pure forward over M = B*T independent rows.
//
// Rows never interact, so the grid is a set of 64-row blocks, each owned by NB workgroups that split
// every layer's output columns (weights of one column slice stay hot in the L2 of one XCD: block id =
// slot * NB + n puts every row block's slice n on XCD n % 8).  The NB workgroups of a row block meet
// only at their own arrival counter; row blocks never wait for each other.
//
// Per step t, workgroup n of a row block (all MFMA work is v_mfma_f32_16x16x4_f32, exact fp32):
//   actor l     y_l slice = act(LN_{l-1}(y_{l-1})) Wa_l^T        (l = 0: h_t Wa_0[:, S:]^T + one-hot
//                                                                prior gathered from Wa_0[:, :S]^T)
//   head        logits = act(LN(y_La)) Wh^T + bh, every workgroup redundantly; unimix sample per head
//   recurrent   x slice = gather of Wr^T rows picked by (prior, action) one-hots (no GEMM at all)
//   GRU         gx slice = [h_t, act(LN_r(x))] Wg^T for the three gates of h columns [n*ch, (n+1)*ch),
//               row statistics over 3Hd from the NB partials, h_{t+1} slice from the gates
//   transition  u slice = h_{t+1} Wt1^T;  logits slice = act(LN_t(u)) Wt2^T + bt2 over whole
//               categoricals; unimix + sample -> prior_{t+1} one-hot and class index
// LayerNorms never need a pass of their own: producers publish per-row (mean, M2) partials of their
// column slice, consumers combine them (Chan) and normalise while staging the A operand.
//
// Hand-offs follow the write-through protocol of rssm_persist.hip: every handed-off word is stored
// device-coherent (agent-scope atomic store / sc1 buffer store), stores drain, the workgroup joins,
// one lane bumps the slot's arrival counter; consumers poll it and read handed-off words with sc1
// loads.  A buffer published at arrival k is read only between wait(k) and arrive(k + 1), so two
// parities of every hand-off buffer suffice.  Spins are bounded; a timeout sets the error word and
// every waiter leaves, so the grid always drains.
#include "common.h"
#include "imag.h"

#include <algorithm>

namespace srl {
namespace imag {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32;
typedef unsigned long long u64;

constexpr int NTH = 256;      // 4 waves; wave w owns rows 16w .. 16w + 15 of the 64-row block
constexpr int ROWS = 64;
constexpr int KC = 64;        // k per staged chunk
constexpr int ALD = KC + 4;   // LDS row stride of staged chunks
constexpr int NTMAX = 6;      // 16-column MFMA tiles per workgroup slice
constexpr int CLD = 16 * NTMAX + 4;
constexpr int SLOTW = 32;     // u32 words between slot counters (128 B)
constexpr u32 SPIN_MAX = 1u << 22;

// LDS carving (floats)
constexpr int L_AS = 0;
constexpr int L_WS = L_AS + 2 * ROWS * ALD;
constexpr int L_CT = L_WS + 2 * 16 * NTMAX * ALD;
constexpr int L_MU = L_CT + ROWS * CLD;
constexpr int L_RS = L_MU + ROWS;
constexpr int L_AIDX = L_RS + ROWS;               // int [64][MAXH]
constexpr int L_PIDX = L_AIDX + ROWS * MAXH;      // uint8 [64][64]
constexpr int L_U = L_PIDX + ROWS * 64 / 4;      // this step's uniforms: heads [64][MAXH], prior [64][gpw]
constexpr int L_HT = L_U + ROWS * 64;            // h_t of this workgroup's GRU columns [64][ch <= 32]
constexpr int L_HOFF = L_HT + ROWS * 32;         // int [MAXH]
constexpr int L_FLAG = L_HOFF + MAXH;
constexpr int L_TOTAL = L_FLAG + 4;

// The dynamic LDS block, addressed directly in every helper so the compiler keeps LDS instructions.
#define SMEM extern __shared__ float sm[]

// ------------------------------------------------------------------ device-coherent accesses
// Buffer resource of a wave-uniform base: the pointer is made scalar explicitly (values that reach a
// device function through its arguments live in VGPRs, and a VGPR base would make the compiler wrap
// every buffer load in a waterfall loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* b = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, 0x7fffffff, 0x00020000);
}
// 16-B load / store with sc1 (device scope: misses the CU's L1, which other CUs' stores never refresh)
__device__ __forceinline__ f4 ld4_wt(const float* base, int off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), off * 4, 0, 16));
}
__device__ __forceinline__ void st4_wt(float* base, int off, f4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc(base), off * 4, 0, 16);
}
// plain (cached) 16-B buffer load: read-only operands (weights, LayerNorm parameters)
__device__ __forceinline__ f4 ld4(const float* base, int off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), off * 4, 0, 0));
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ldi_wt(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sti_wt(int* p, int v) {
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

// ------------------------------------------------------------------ arrival counters
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ long long prof_clock() {
  long long c;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  return c;
}

struct Sync {
  long long* prof;  // block 0 only (s_memrealtime, 100 MHz): [arrival][0] work done, [1] wait done
  u32* ctr;   // this slot's counter
  u32* err;   // error word (shared)
  int NB;
  u32 ph;     // arrivals so far in this slot (per workgroup)
  int* flag;  // LDS
};

// Sub-phase stamp j (< 4) of the current arrival, block 0 only: prof[4096 + 4 * arrival + j].
__device__ __forceinline__ void mark(const Sync& s, int j) {
  if (s.prof && threadIdx.x == 0) s.prof[4096 + 4 * s.ph + j] = prof_clock();
}

// Every wave's hand-off stores drain, the workgroup joins, one lane arrives; then wait for the NB
// workgroups of the row block.  Returns false (uniformly) when the launch is aborting.
__device__ __forceinline__ bool handoff(Sync& s) {
  drain();
  __syncthreads();
  if (s.prof && threadIdx.x == 0) s.prof[2 * s.ph] = prof_clock();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(s.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ++s.ph;
  if (threadIdx.x == 0) {
    const u32 need = s.ph * (u32)s.NB;
    int bad = 0;
    for (u32 spins = 0;; ++spins) {
      if (__hip_atomic_load(s.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) break;
      if (__hip_atomic_load(s.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        bad = 1;
        break;
      }
      if (spins >= SPIN_MAX) {
        __hip_atomic_store(s.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad = 2;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *s.flag = bad;
    if (s.prof) s.prof[2 * s.ph - 1] = prof_clock();
  }
  __syncthreads();
  const bool ok = *s.flag == 0;
  __syncthreads();
  return ok;
}

// ------------------------------------------------------------------ fast math (as the scan kernels)
__device__ __forceinline__ float f_act(float z, int act) {
  switch (act) {
    case ACT_SILU: return z * __builtin_amdgcn_rcpf(1.f + __expf(-z));
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_TANH: return tanhf(z);
    default: return z;
  }
}

// ------------------------------------------------------------------ categorical sampling
#define FEPS 1.1920928955078125e-07f

__device__ __forceinline__ float seg_prefix(float v, int width, int k) {
  for (int o = 1; o < width; o <<= 1) {
    const float t = __shfl_up(v, o, width);
    if (k >= o) v += t;
  }
  return v;
}

// Unimix + inverse-CDF sample of one categorical held by an aligned segment of W lanes (lane k of
// the segment holds class k; k >= C or !valid lanes hold nothing).  Same operation order as
// dist.hip unimix_sample_fwd_kernel, so both pick the same class from the same logits and uniform.
__device__ __forceinline__ int seg_pick(float l, bool valid, int k, int W, int C, float alpha, float u) {
  float m = l;
  if (alpha > 0.f) {
    const float mx = seg_max(l, W);
    const float e = valid ? __expf(l - mx) : 0.f;
    const float s = seg_sum(e, W);
    const float q = e / s;
    float pm = (1.f - alpha) * q + alpha / C;
    pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
    m = valid ? logf(pm) : -INFINITY;
  }
  const float mx2 = seg_max(m, W);
  const float e2 = valid ? __expf(m - mx2) : 0.f;
  const float s2 = seg_sum(e2, W);
  const float p = e2 / s2;
  const float cdf = seg_prefix(p, W, k);
  const float below = (valid && cdf < u * seg_max(cdf, W)) ? 1.f : 0.f;
  int pick = (int)seg_sum(below, W);
  return pick > C - 1 ? C - 1 : pick;
}

// One categorical per LANE, classes in registers (W = power of two >= C): the operations of the W-lane
// segment form above in the same order - sums as the xor-butterfly tree, the CDF as the Hillis-Steele
// scan - without ~60 dependent cross-lane steps per categorical; divisions are reciprocal-multiplies
// and the log is v_log (ulp-level differences: a sample flips only when a uniform lands within a few
// ulp of a CDF boundary).
template <int W>
__device__ __forceinline__ float tree_sum(const float (&v)[W]) {
  float t[W];
#pragma unroll
  for (int k = 0; k < W; ++k) t[k] = v[k];
#pragma unroll
  for (int o = W >> 1; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < o; ++k) t[k] = t[k] + t[k + o];
  return t[0];
}

// In place on one register array (plus the tree's temporary): the main kernel keeps a lot live, and
// five W-arrays spilled to scratch.
template <int W>
__device__ __forceinline__ int lane_pick(const float* l, int C, float alpha, float u) {
  float x[W];
#pragma unroll
  for (int k = 0; k < W; ++k) x[k] = k < C ? l[k] : -INFINITY;
  if (alpha > 0.f) {
    float mx = x[0];
#pragma unroll
    for (int k = 1; k < W; ++k) mx = fmaxf(mx, x[k]);
#pragma unroll
    for (int k = 0; k < W; ++k) x[k] = k < C ? __expf(x[k] - mx) : 0.f;
    const float inv = __builtin_amdgcn_rcpf(tree_sum<W>(x)), mix = alpha / C;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      float pm = (1.f - alpha) * (x[k] * inv) + mix;
      pm = fminf(fmaxf(pm, FEPS), 1.f - FEPS);
      x[k] = k < C ? __logf(pm) : -INFINITY;
    }
  }
  float mx2 = x[0];
#pragma unroll
  for (int k = 1; k < W; ++k) mx2 = fmaxf(mx2, x[k]);
#pragma unroll
  for (int k = 0; k < W; ++k) x[k] = k < C ? __expf(x[k] - mx2) : 0.f;
  const float inv2 = __builtin_amdgcn_rcpf(tree_sum<W>(x));
#pragma unroll
  for (int k = 0; k < W; ++k) x[k] *= inv2;
#pragma unroll
  for (int o = 1; o < W; o <<= 1)
#pragma unroll
    for (int k = W - 1; k >= o; --k) x[k] += x[k - o];
  float cm = x[0];
#pragma unroll
  for (int k = 1; k < W; ++k) cm = fmaxf(cm, x[k]);
  const float thr = u * cm;
  int pick = 0;
#pragma unroll
  for (int k = 0; k < W; ++k) pick += (k < C && x[k] < thr) ? 1 : 0;
  return pick > C - 1 ? C - 1 : pick;
}

__device__ __forceinline__ int lane_pick_any(int W, const float* l, int C, float alpha, float u) {
  switch (W) {
    case 1: return 0;
    case 2: return lane_pick<2>(l, C, alpha, u);
    case 4: return lane_pick<4>(l, C, alpha, u);
    case 8: return lane_pick<8>(l, C, alpha, u);
    case 16: return lane_pick<16>(l, C, alpha, u);
    default: return lane_pick<32>(l, C, alpha, u);
  }
}

// ------------------------------------------------------------------ GEMM tile
// A operand segment: rows r0 .. r0 + 63 of a row-major source, columns [col, col + K); optionally
// LayerNorm'd (row statistics in LDS mu/rs) and activated while staged.
struct ASeg {
  const float* base;
  int ld, col, K;
  const float *gam, *bet;
  int act, ln;
};

// One staged K chunk in registers: 4 A float4s, up to NTMAX W float4s, and the chunk's LayerNorm
// parameters (a thread's k offset within the chunk is the same for its four A loads).
template <int NT>
struct Stage {
  f4 ra[4], rw[NT], gm, bt;
};

template <int ACT>
__device__ __forceinline__ float act_t(float z) {
  if constexpr (ACT == ACT_SILU) return z * __builtin_amdgcn_rcpf(1.f + __expf(-z));
  else if constexpr (ACT == ACT_ELU) return z > 0.f ? z : expm1f(z);
  else if constexpr (ACT == ACT_RELU) return z > 0.f ? z : 0.f;
  else if constexpr (ACT == ACT_TANH) return tanhf(z);
  else return z;
}

// LayerNorm + activation of a staged A chunk (4 float4 per thread) into LDS.
template <int ACT, int NT>
__device__ __forceinline__ void ln_stage(const Stage<NT>& st, float* Ab, const float* mu, const float* rs, int tid, int kq) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (q * NTH + tid) >> 4;
    const float m = mu[row], r = rs[row];
    f4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = act_t<ACT>((st.ra[q][j] - m) * r * st.gm[j] + st.bt[j]);
    *(f4*)(Ab + row * ALD + kq) = v;
  }
}

// Ct[64][16*nt] = A[64][K] W_slice^T (nt <= NTMAX, uniform).  W_slice row of local column c:
//   row0 + (c / segw) * segs + c % segw   (every one of the 16*nt rows exists: the head weights come
//   zero-padded to whole tiles, so no load is conditional)
// Chunks of KC columns go global -> registers -> LDS through a two-deep register ring (two chunks'
// loads in flight while the MFMAs of a third run) and two LDS buffers.  Tiles t >= nt are skipped by
// uniform branches, so one body serves every slice width.
template <int NT>
__device__ __noinline__ void gemm_nt(const ASeg s0_, const ASeg s1_, int r0, const float* __restrict__ W,
                                       int ldw, int wk0, int row0, int segw, int segs, int nrow) {
  SMEM;
  // arguments of a device function arrive in VGPRs: make the uniform ones scalar so branches on them
  // stay uniform (no exec masking) and addresses stay SGPR bases
#define SCAL(x) x = __builtin_amdgcn_readfirstlane(x)
  SCAL(r0); SCAL(ldw); SCAL(wk0); SCAL(row0); SCAL(segw); SCAL(segs); SCAL(nrow);
  ASeg s0 = s0_, s1 = s1_;
  SCAL(s0.ld); SCAL(s0.col); SCAL(s0.K); SCAL(s0.act); SCAL(s0.ln);
  SCAL(s1.ld); SCAL(s1.col); SCAL(s1.K); SCAL(s1.act); SCAL(s1.ln);
#undef SCAL
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15, g = lane >> 4;
  float* As = sm + L_AS;
  float* Ws = sm + L_WS;
  const float* mu = sm + L_MU;
  const float* rs = sm + L_RS;
  const int K = s0.K + s1.K, nch = K / KC;
  const int kq = (tid & 15) << 2;  // this thread's k offset in every chunk (A and W alike)
  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  // Per-thread byte offsets are fixed for the whole GEMM; a chunk only moves the scalar offset, so a
  // load is one buffer instruction with no per-lane address arithmetic.
  int wofs[NT], aofs0[4], aofs1[4];
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int wr = (q * NTH + tid) >> 4;
    wofs[q] = ((row0 + (wr / segw) * segs + (wr % segw)) * ldw + wk0 + kq) * 4;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = r0 + ((q * NTH + tid) >> 4);
    aofs0[q] = (row * s0.ld + s0.col + kq) * 4;
    aofs1[q] = (row * s1.ld + s1.col + kq) * 4;
  }
  const auto rA0 = rsrc(s0.base), rA1 = rsrc(s1.K ? s1.base : s0.base), rW = rsrc(W);
  const auto rG0 = rsrc(s0.gam), rB0 = rsrc(s0.bet);
  const auto rG1 = rsrc(s1.K ? s1.gam : s0.gam), rB1 = rsrc(s1.K ? s1.bet : s0.bet);

  // every load of a stage is unconditional (straight-line), so the compiler can wait for one stage
  // with a counted vmcnt while the next stage's loads stay in flight
  auto load = [&](Stage<NT>& st, int c) {
    const int k = c * KC;
    const bool first = k < s0.K;
    const int kb = (first ? k : k - s0.K) * 4;  // chunk offset within the segment (bytes, uniform)
    // segment choice by selects, not branches: a branch around loads defeats the counted waits
    const auto rA = first ? rA0 : rA1, rG = first ? rG0 : rG1, rB = first ? rB0 : rB1;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      st.ra[q] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rA, first ? aofs0[q] : aofs1[q], kb, 16));
    st.gm = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rG, kq * 4, kb, 0));
    st.bt = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rB, kq * 4, kb, 0));
#pragma unroll
    for (int q = 0; q < NT; ++q)
      st.rw[q] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rW, wofs[q], k * 4, 0));
  };
  auto store = [&](Stage<NT>& st, int c, int b) {
    const int k = c * KC;
    const bool first = k < s0.K;
    float* Ab = As + b * ROWS * ALD;
    float* Wb = Ws + b * 16 * NTMAX * ALD;
    if (first ? s0.ln : s1.ln) {
      ln_stage<ACT_SILU>(st, Ab, mu, rs, tid, kq);  // the host gate admits SiLU MLPs only
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) *(f4*)(Ab + ((q * NTH + tid) >> 4) * ALD + kq) = st.ra[q];
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) *(f4*)(Wb + ((q * NTH + tid) >> 4) * ALD + kq) = st.rw[q];
  };
  // All of a chunk's fragments are read up front (the MFMAs of k-step kk start as soon as its reads
  // land); with NT <= 2 the even / odd k-steps accumulate into separate registers so consecutive
  // MFMAs never wait on each other's accumulator.
  constexpr int NA = NT <= 2 ? 2 : 1;
  f4 acc2[NA - 1 > 0 ? NT : 1];
  if constexpr (NA == 2) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc2[t] = f4{0.f, 0.f, 0.f, 0.f};
  }
  auto compute = [&](int b) {
    const float* Ab = As + b * ROWS * ALD + (16 * w + i) * ALD + 4 * g;
    const float* Wb = Ws + b * 16 * NTMAX * ALD + i * ALD + 4 * g;
    f4 a[KC / 16], bv[KC / 16][NT];
#pragma unroll
    for (int kk = 0; kk < KC / 16; ++kk) {
      a[kk] = *(const f4*)(Ab + kk * 16);
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[kk][t] = *(const f4*)(Wb + 16 * t * ALD + kk * 16);
    }
#pragma unroll
    for (int kk = 0; kk < KC / 16; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if (NA == 2 && (kk & 1))
            acc2[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk][j], bv[kk][t][j], acc2[t], 0, 0, 0);
          else
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk][j], bv[kk][t][j], acc[t], 0, 0, 0);
        }
  };

  // nch is even (K % 128 == 0, host gate); the two loads past the end re-read the last chunk into a
  // stage nobody computes, which keeps every load unconditional
  Stage<NT> sa, sb;
  load(sa, 0);
  load(sb, 1);
  store(sa, 0, 0);
  __syncthreads();
  for (int c = 0; c < nch; c += 2) {
    load(sa, min(c + 2, nch - 1));
    compute(0);
    store(sb, c + 1, 1);
    __syncthreads();
    load(sb, min(c + 3, nch - 1));
    compute(1);
    store(sa, min(c + 2, nch - 1), 0);
    __syncthreads();
  }
  if constexpr (NA == 2) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] += acc2[t];
  }
  // C/D map of 16x16x4: col = lane & 15, row = 4 * (lane >> 4) + reg
  float* Ct = sm + L_CT;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) Ct[(16 * w + 4 * g + r) * CLD + 16 * t + i] = acc[t][r];
  __syncthreads();
}

__device__ __forceinline__ void gemm_tile(int nt, const ASeg s0, const ASeg s1, int r0, const float* W, int ldw, int wk0,
                                          int row0, int segw, int segs, int nrow) {
  switch (nt) {
    case 1: gemm_nt<1>(s0, s1, r0, W, ldw, wk0, row0, segw, segs, nrow); break;
    case 2: gemm_nt<2>(s0, s1, r0, W, ldw, wk0, row0, segw, segs, nrow); break;
    case 3: gemm_nt<3>(s0, s1, r0, W, ldw, wk0, row0, segw, segs, nrow); break;
    case 4: gemm_nt<4>(s0, s1, r0, W, ldw, wk0, row0, segw, segs, nrow); break;
    case 5: gemm_nt<5>(s0, s1, r0, W, ldw, wk0, row0, segw, segs, nrow); break;
    default: gemm_nt<6>(s0, s1, r0, W, ldw, wk0, row0, segw, segs, nrow); break;
  }
}

// ------------------------------------------------------------------ epilogue pieces
// Ct[.][c] += bias[row of local column c] for c < cw.
__device__ __forceinline__ void add_bias(const float* bias, int cw, int row0, int segw, int segs) {
  SMEM;
  if (!bias) return;
  float* Ct = sm + L_CT;
  // a thread keeps one column (one bias load, issued before any use), rows strided by NTH / cw
  const int rp = NTH / cw;
  if (threadIdx.x < rp * cw) {
    const int c = threadIdx.x % cw;
    const float b = bias[row0 + (c / segw) * segs + c % segw];
    for (int r = threadIdx.x / cw; r < ROWS; r += rp) Ct[r * CLD + c] += b;
  }
  __syncthreads();
}

// Ct[.][c] += sum over the one-hot inputs of WT[input row][col0 + c] (c < cw): the prior's G classes
// (pidx) and, with acts, the action heads' classes (aidx) at rows S + head offset.
__device__ __forceinline__ void gather_add(const float* __restrict__ WT, int ldT, int col0, int cw, int G, int disc,
                                           bool acts, int S, int nh) {
  SMEM;
  const int* hoff = (const int*)(sm + L_HOFF);
  float* Ct = sm + L_CT;
  const unsigned char* pidx = (const unsigned char*)(sm + L_PIDX);
  const int* aidx = (const int*)(sm + L_AIDX);
  const int c4n = cw >> 2;
  for (int e = threadIdx.x; e < ROWS * c4n; e += NTH) {
    const int r = e / c4n, c = (e - r * c4n) << 2;
    f4 a = *(const f4*)(Ct + r * CLD + c);
    const int cc = col0 + c;
    // sixteen independent row loads in flight; indices past the end are clamped (loaded, then dropped)
    for (int g0 = 0; g0 < G; g0 += 16) {
      f4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int gg = min(g0 + u, G - 1);
        v[u] = ld4(WT, (gg * disc + pidx[r * 64 + gg]) * ldT + cc);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (g0 + u < G) a += v[u];
    }
    if (acts) {
      f4 v[MAXH];
#pragma unroll
      for (int h = 0; h < MAXH; ++h) {
        const int hh = min(h, nh - 1);
        v[h] = ld4(WT, (S + hoff[hh] + aidx[r * MAXH + hh]) * ldT + cc);
      }
#pragma unroll
      for (int h = 0; h < MAXH; ++h)
        if (h < nh) a += v[h];
    }
    *(f4*)(Ct + r * CLD + c) = a;
  }
  __syncthreads();
}

// Publish Ct[64][cw] as columns [col0, col0 + cw) of Y (row stride ldy; rows r0 ..) and, unless
// cw == 0 rows... the per-row (mean, M2) partial of the slice at part[(r0 + row) * NB + n].
__device__ __forceinline__ void publish(float* Y, int ldy, int col0, int cw, int r0, float* part, int NB, int n) {
  SMEM;
  const float* Ct = sm + L_CT;
  if (Y) {
    const int c4n = cw >> 2;
    for (int e = threadIdx.x; e < ROWS * c4n; e += NTH) {
      const int r = e / c4n, c = (e - r * c4n) << 2;
      st4_wt(Y, (r0 + r) * ldy + col0 + c, *(const f4*)(Ct + r * CLD + c));
    }
  }
  // four lanes per row
  const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
  const int per = (cw + 3) >> 2, lo = q * per, hi = min(cw, lo + per);
  float s = 0.f;
  for (int c = lo; c < hi; ++c) s += Ct[r * CLD + c];
  const float mean = seg_sum(s, 4) / cw;
  float m2 = 0.f;
  for (int c = lo; c < hi; ++c) {
    const float d = Ct[r * CLD + c] - mean;
    m2 += d * d;
  }
  m2 = seg_sum(m2, 4);
  if (q == 0) st_wt2(part + ((size_t)(r0 + r) * NB + n) * 2, mean, m2);
}

// Row statistics (mean, 1/std) over N = NB * cw columns from the NB slice partials (Chan combine,
// two-pass over the partial means) into LDS mu / rs.
__device__ __forceinline__ void row_stats(const float* part, int NB, int cw, int r0, float eps) {
  SMEM;
  const int r = threadIdx.x >> 2, q = threadIdx.x & 3;
  float2 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = ld_wt2(part + ((size_t)(r0 + r) * NB + min(q + 4 * j, NB - 1)) * 2);  // NB <= 16
  float s = 0.f, m2 = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (q + 4 * j < NB) {
      s += v[j].x;
      m2 += v[j].y;
    }
  const float mean = seg_sum(s, 4) / NB;
  float d = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (q + 4 * j < NB) d += (v[j].x - mean) * (v[j].x - mean);
  const float M2 = seg_sum(m2, 4) + cw * seg_sum(d, 4);
  if (q == 0) {
    sm[L_MU + r] = mean;
    sm[L_RS + r] = rsqrtf(M2 / (float)(NB * cw) + eps);
  }
  __syncthreads();
}

// Prior class indices of the row block -> LDS (all loads issued before the first store).
__device__ __forceinline__ void load_pidx(const int* idx, int r0, int G) {
  SMEM;
  unsigned char* pidx = (unsigned char*)(sm + L_PIDX);
  constexpr int MAXE = ROWS * 64 / NTH;  // G <= 64
  int v[MAXE];
#pragma unroll
  for (int u = 0; u < MAXE; ++u) {
    const int e = min(threadIdx.x + u * NTH, ROWS * G - 1);
    v[u] = ldi_wt(idx + (size_t)r0 * G + e);
  }
#pragma unroll
  for (int u = 0; u < MAXE; ++u) {
    const int e = threadIdx.x + u * NTH;
    if (e < ROWS * G) pidx[(e / G) * 64 + e % G] = (unsigned char)v[u];
  }
  __syncthreads();
}

// ------------------------------------------------------------------ the kernel
__global__ void __launch_bounds__(NTH) imagine_kernel(const IP p) {
  SMEM;
  const int NB = p.NB, n = blockIdx.x % NB, slot = blockIdx.x / NB;
  const int M = p.M, S = p.S, Hd = p.Hd, A = p.A, G = p.G, disc = p.disc;
  const int LDB = A + S + Hd;
  const int YLD = max(p.Da, max(p.D, p.Ht));
  const int Ust = M * (p.nh + G);
  const int cwa = p.Da / NB, cwr = p.D / NB, ch = Hd / NB, cwt = p.Ht / NB, cws = S / NB;
  const int gpw = cws / disc;
  int* hoff = (int*)(sm + L_HOFF);
  int hmax = 1;
  {
    int o = 0;
    for (int h = 0; h < p.nh; ++h) {
      if (threadIdx.x == 0) hoff[h] = o;
      o += p.head[h];
      hmax = max(hmax, p.head[h]);
    }
  }
  int Wh = 1;
  while (Wh < hmax) Wh <<= 1;
  Sync sy{blockIdx.x == 0 ? p.prof : nullptr, p.sync + slot * SLOTW, p.sync + p.nslots * SLOTW, NB, 0u, (int*)(sm + L_FLAG)};
  unsigned char* pidx = (unsigned char*)(sm + L_PIDX);
  int* aidx = (int*)(sm + L_AIDX);
  const ASeg none{nullptr, 0, 0, 0, nullptr, nullptr, 0, 0};
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

  for (int rb = slot; rb < p.RB; rb += p.nslots) {
    const int r0 = rb * ROWS;
    load_pidx(p.idx, r0, G);
    for (int e = tid; e < ROWS * ch; e += NTH) {  // h_0 of this workgroup's GRU columns
      const int r = e / ch, j = e - r * ch;
      sm[L_HT + r * 32 + j] = p.buf[(size_t)(r0 + r) * LDB + A + S + n * ch + j];
    }
    __syncthreads();
    for (int t = 0; t <= p.horizon; ++t) {
      float* bt = p.buf + (size_t)t * M * LDB;
      float* bn = bt + (size_t)M * LDB;
      // ---------------- this step's uniforms -> LDS (read after the GEMMs, so their latency is paid once)
      {  // heads: 64 x nh (<= 512) values, prior: 64 x gpw; every load issued before the first store
        float* us = sm + L_U;
        float uh[2], up[4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = min(tid + u * NTH, ROWS * p.nh - 1), r = e / p.nh, h = e - r * p.nh;
          uh[u] = p.U[(size_t)t * Ust + (size_t)h * M + r0 + r];
        }
        const int np = t < p.horizon ? ROWS * gpw : 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = max(0, min(tid + u * NTH, np - 1)), r = e / gpw, gl = e - r * gpw;
          up[u] = p.U[(size_t)max(0, min(t, p.horizon - 1)) * Ust + (size_t)p.nh * M + (size_t)(r0 + r) * G + n * gpw + gl];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = tid + u * NTH;
          if (e < ROWS * p.nh) us[(e / p.nh) * MAXH + e % p.nh] = uh[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = tid + u * NTH;
          if (e < np) us[ROWS * MAXH + e] = up[u];
        }
        for (int e = tid + 4 * NTH; e < np; e += NTH)  // gpw > 16 (not the Atari shapes)
          us[ROWS * MAXH + e] = p.U[(size_t)t * Ust + (size_t)p.nh * M + (size_t)(r0 + e / gpw) * G + n * gpw + e % gpw];
      }
      // ---------------- actor MLP
      int ypar = 0;
      for (int l = 0; l < p.La; ++l) {
        const int par = sy.ph & 1;
        if (l == 0) {
          const ASeg a0{bt, LDB, A + S, Hd, p.lnaw[0], p.lnab[0], 0, 0};
          gemm_tile(cwa / 16, a0, none, r0, p.Wa[0], S + Hd, S, n * cwa, cwa, 0, cwa);
          gather_add(p.WaT, p.Da, n * cwa, cwa, G, disc, false, S, 0);
        } else {
          row_stats(p.part + (size_t)ypar * M * NB * 2, NB, cwa, r0, p.eps_a);
          const ASeg a0{p.Y + (size_t)ypar * M * YLD, YLD, 0, p.Da, p.lnaw[l - 1], p.lnab[l - 1], p.act_a, 1};
          gemm_tile(cwa / 16, a0, none, r0, p.Wa[l], p.Da, 0, n * cwa, cwa, 0, cwa);
        }
        add_bias(p.ba[l], cwa, n * cwa, cwa, 0);
        publish(p.Y + (size_t)par * M * YLD, YLD, n * cwa, cwa, r0, p.part + (size_t)par * M * NB * 2, NB, n);
        if (!handoff(sy)) return;
        ypar = par;
      }
      // ---------------- heads (every workgroup, redundantly) + action samples
      {
        row_stats(p.part + (size_t)ypar * M * NB * 2, NB, cwa, r0, p.eps_a);
        const ASeg a0{p.Y + (size_t)ypar * M * YLD, YLD, 0, p.Da, p.lnaw[p.La - 1], p.lnab[p.La - 1], p.act_a, 1};
        const int nth = (A + 15) / 16;
        mark(sy, 0);
        gemm_tile(nth, a0, none, r0, p.Wh, p.Da, 0, 0, 16 * nth, 0, A);
        mark(sy, 1);
        add_bias(p.bh, A, 0, 16 * nth, 0);
        const float* Ct = sm + L_CT;
        const int ncat = 16 * p.nh;  // categoricals of this wave: 16 rows x nh heads, one per lane
        for (int q = lane; q < ncat; q += 64) {
          const int r = 16 * w + q / p.nh, h = q % p.nh;
          const int C = p.head[h];
          const int pick = lane_pick_any(Wh, Ct + r * CLD + hoff[h], C, p.alpha_a, sm[L_U + r * MAXH + h]);
          aidx[r * MAXH + h] = pick;
        }
        __syncthreads();
        if (n == 0)  // action one-hots, written row-contiguously by the whole workgroup
          for (int e = tid; e < ROWS * A; e += NTH) {
            const int r = e / A, c = e - r * A;
            int h = 0;
            while (h + 1 < p.nh && c >= hoff[h + 1]) ++h;
            bt[(size_t)(r0 + r) * LDB + c] = c - hoff[h] == aidx[r * MAXH + h] ? 1.f : 0.f;
          }
      }
      if (t == p.horizon) break;
      // ---------------- recurrent input layer: one-hot gathers of Wr^T rows
      int par = sy.ph & 1;
      {
        float* Ct = sm + L_CT;
        for (int e = tid; e < ROWS * cwr; e += NTH) Ct[(e / cwr) * CLD + e % cwr] = 0.f;
        __syncthreads();
        add_bias(p.br, cwr, n * cwr, cwr, 0);
        mark(sy, 2);
        gather_add(p.WrT, p.D, n * cwr, cwr, G, disc, true, S, p.nh);
        mark(sy, 3);
        publish(p.Y + (size_t)par * M * YLD, YLD, n * cwr, cwr, r0, p.part + (size_t)par * M * NB * 2, NB, n);
        if (!handoff(sy)) return;
      }
      // ---------------- GRU projection for the three gates of h columns [n*ch, (n+1)*ch)
      {
        row_stats(p.part + (size_t)par * M * NB * 2, NB, cwr, r0, p.eps_r);
        const ASeg a0{bt, LDB, A + S, Hd, p.lngw, p.lngb, 0, 0};
        const ASeg a1{p.Y + (size_t)par * M * YLD, YLD, 0, p.D, p.lnrw, p.lnrb, p.act_r, 1};
        gemm_tile(3 * ch / 16, a0, a1, r0, p.Wg, Hd + p.D, 0, n * ch, ch, Hd, 3 * ch);
        add_bias(p.bg, 3 * ch, n * ch, ch, Hd);
        par = sy.ph & 1;
        publish(nullptr, 0, 0, 3 * ch, r0, p.part + (size_t)par * M * NB * 2, NB, n);
        if (!handoff(sy)) return;
        row_stats(p.part + (size_t)par * M * NB * 2, NB, 3 * ch, r0, p.eps_g);
        const float* Ct = sm + L_CT;
        {
          const int rp = NTH / ch;  // ch divides NTH (ch in 16, 32): a thread keeps one column
          const int j = tid % ch, col = n * ch + j;
          const float gr = p.lngw[col], br = p.lngb[col], gc = p.lngw[Hd + col], bc = p.lngb[Hd + col];
          const float gu = p.lngw[2 * Hd + col], bu = p.lngb[2 * Hd + col];
          for (int r = tid / ch; r < ROWS; r += rp) {
            const float m = sm[L_MU + r], rs = sm[L_RS + r];
            const float xr = (Ct[r * CLD + j] - m) * rs * gr + br;
            const float xc = (Ct[r * CLD + ch + j] - m) * rs * gc + bc;
            const float xu = (Ct[r * CLD + 2 * ch + j] - m) * rs * gu + bu;
            const float rg = sigmoidf_(xr);
            const float cd = tanhf(rg * xc);
            const float ug = sigmoidf_(xu - 1.f);
            const float hn = ug * cd + (1.f - ug) * sm[L_HT + r * 32 + j];
            sm[L_HT + r * 32 + j] = hn;  // this workgroup's columns of h_{t+1}: its h_prev next step
            st_wt(bn + (size_t)(r0 + r) * LDB + A + S + col, hn);
          }
        }
        if (!handoff(sy)) return;
      }
      // ---------------- transition hidden layer
      par = sy.ph & 1;
      {
        const ASeg a0{bn, LDB, A + S, Hd, p.lngw, p.lngb, 0, 0};
        gemm_tile(cwt / 16, a0, none, r0, p.Wt1, Hd, 0, n * cwt, cwt, 0, cwt);
        add_bias(p.bt1, cwt, n * cwt, cwt, 0);
        publish(p.Y + (size_t)par * M * YLD, YLD, n * cwt, cwt, r0, p.part + (size_t)par * M * NB * 2, NB, n);
        if (!handoff(sy)) return;
      }
      // ---------------- transition logits over whole categoricals + prior samples
      {
        row_stats(p.part + (size_t)par * M * NB * 2, NB, cwt, r0, p.eps_t);
        const ASeg a0{p.Y + (size_t)par * M * YLD, YLD, 0, p.Ht, p.lntw, p.lntb, p.act_t, 1};
        mark(sy, 0);
        gemm_tile(cws / 16, a0, none, r0, p.Wt2, p.Ht, 0, n * cws, cws, 0, cws);
        mark(sy, 1);
        add_bias(p.bt2, cws, n * cws, cws, 0);
        const float* Ct = sm + L_CT;
        int Wd = 1;
        while (Wd < disc) Wd <<= 1;
        const int ncat = 16 * gpw;  // this wave: 16 rows x gpw categoricals, one per lane
        for (int q = lane; q < ncat; q += 64) {
          const int r = 16 * w + q / gpw, gl = q % gpw, gg = n * gpw + gl;
          const int pick = lane_pick_any(Wd, Ct + r * CLD + gl * disc, disc, p.alpha_s, sm[L_U + ROWS * MAXH + r * gpw + gl]);
          sti_wt(p.idx + (size_t)(r0 + r) * G + gg, pick);
          ((int*)sm)[L_U + ROWS * MAXH + r * gpw + gl] = pick;  // the uniform's slot is free now
        }
        __syncthreads();
        {  // prior one-hots of this slice, row-contiguous
          const int* pk = (const int*)sm + L_U + ROWS * MAXH;
          for (int e = tid; e < ROWS * cws; e += NTH) {
            const int r = e / cws, c = e - r * cws, gl = c / disc;
            bn[(size_t)(r0 + r) * LDB + A + n * cws + c] = c - gl * disc == pk[r * gpw + gl] ? 1.f : 0.f;
          }
        }
        mark(sy, 2);
        if (!handoff(sy)) return;
        load_pidx(p.idx, r0, G);
      }
    }
  }
}

__global__ void zero_kernel(u32* w, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) w[i] = 0u;
}

}  // namespace imag
}  // namespace srl

using namespace srl;
using namespace srl::imag;

int imagine_sync_words(int nslots) { return (nslots + 1) * SLOTW; }

// Column split NB (power of two) and row-block slots for a shape; NB = 0: unsupported (the caller
// keeps the per-op rollout).
void imagine_plan(int M, int S, int Hd, int D, int Da, int Ht, int A, int nh, int disc, int La, int& NB, int& nslots) {
  NB = 0;
  nslots = 0;
  if (M <= 0 || M % ROWS || La < 1 || La > MAXL || nh < 1 || nh > MAXH || A > 64 || disc < 1 || disc > 32 || S % disc)
    return;
  if (S / disc > 64 || Hd % (2 * KC) || D % (2 * KC) || Da % (2 * KC) || Ht % (2 * KC)) return;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int RB = M / ROWS;
  for (int nb = 16; nb >= 1; nb >>= 1) {
    auto fits = [&](int N) { return N % (16 * nb) == 0 && N / nb <= 16 * NTMAX; };
    if (!fits(Da) || !fits(D) || !fits(Ht) || !fits(S)) continue;
    if (Hd % (16 * nb) || 3 * (Hd / nb) > 16 * NTMAX) continue;
    if ((S / nb) % disc || (S / nb / disc) * ROWS > ROWS * 64 - ROWS * MAXH) continue;
    if (nb > cus) continue;
    NB = nb;
    nslots = std::max(1, std::min(RB, cus / nb));
    return;
  }
}

int imagine_lds_bytes() { return L_TOTAL * 4; }

void launch_imagine(const IP& p, hipStream_t st) {
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute((const void*)imagine_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, L_TOTAL * 4);
    init = true;
  }
  hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(256), 0, st, p.sync, imagine_sync_words(p.nslots));
  hipLaunchKernelGGL(imagine_kernel, dim3(p.nslots * p.NB), dim3(NTH), L_TOTAL * 4, st, p);
}
