// Implicit-GEMM k4 s2 p1 convolutions for the Dreamer CNN encoder / decoder on CDNA4 MFMA
// (reference: dreamer_v3/agent.py:48-80 CNNEncoder, :160-206 CNNDecoder; LN channel-last
// utils/model.py:225-235).  fp32 in, fp32 accumulate: v_mfma_f32_32x32x2_f32 (exact fp32 products,
// 64 FLOP/clk/SIMD = the chip's fp32 peak).
//
// Activations are NHWC ("channels last"): the channel dim is the GEMM K (or N) dim, contiguous.
// A k4 s2 p1 conv links a LARGE spatial grid (2SH x 2SW) to a SMALL one (SH x SW).  Three GEMM forms
// cover every pass of both Conv2d and ConvTranspose2d:
//
//   DOWN  out[m=(n,p,q)][a]   = sum_{tap,b} Q[n, 2p-1+kh, 2q-1+kw, b] * W[a][b][kh][kw]
//         (Conv2d forward: Q=x, W=conv weight [co][ci];  ConvT data-grad: Q=dy, W=convT weight [ci][co])
//   UP    out[(n,y,x)][b]     = sum_{2x2 taps of y,x parity, a} P[n, p, q, a] * W[a][b][kh][kw]
//         (ConvT forward: P=x, W=[ci][co];  Conv2d data-grad: P=dy, W=[co][ci]); one parity class per
//         blockIdx.z, so each class is a dense GEMM with K = 4*Ca
//   WGRAD dW[a][tap][b]       = sum_{m=(n,p,q)} P[m][a] * Q[n, 2p-1+kh, 2q-1+kw, b]
//         split-K over pixels into partial slabs, reduced (and permuted to [a][b][kh][kw]) by a 2nd kernel
//
// Epilogues fuse the channel LayerNorm: the workgroup tile spans the whole channel row (N <= 256), so
//   LN_ACT : z = acc; y = act(LN(z)) (+ per-pixel mean/rstd)        (forward of conv -> LN -> act)
//   LN_BWD : acc = dy of the NEXT-lower layer's output; dz = LN/act backward, dgamma/dbeta as per-workgroup
//            column-sum rows reduced in a fixed order afterwards (deterministic; float atomics only without a buffer)
//   PLAIN  : out = acc + bias + c0, NHWC or NCHW (for the 3-channel image / the flat Linear seam)
// Spatial sizes are powers of two; channel counts are multiples of 32 up to 1024 (the 4-channel image
// side: a power of two below 32); all host-checked.
#include "common.h"
#include "conv.h"
#include <algorithm>
#include <cstdlib>
#include <string>


namespace srl {
namespace conv {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int BK = 32;        // K per LDS stage
constexpr int LDK = BK + 4;   // LDS row stride (floats): conflict-free float4 fragment reads

__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// Out-of-range (padding) taps read this zero vector instead of being skipped: the operand loads are then
// unconditional - an exec-masked load under a branch, or a select on the loaded value, made the wait-count
// pass put vmcnt(0) in front of the NEXT K stage's loads, so every stage paid a full memory latency before
// its MFMAs (the prefetch into registers did not overlap anything).
__device__ __attribute__((aligned(16))) float g_zero16[4];
__device__ __forceinline__ const float* zsrc(bool ok, const float* p) { return ok ? p : g_zero16; }
__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float cact(float z, int act) {
  switch (act) {
    case ACT_SILU: return z * fsig(z);
    case ACT_ELU: return z > 0.f ? z : __expf(z) - 1.f;
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_TANH: return 2.f * fsig(2.f * z) - 1.f;
    default: return z;
  }
}
__device__ __forceinline__ float cact_grad(float z, int act) {
  switch (act) {
    case ACT_SILU: {
      const float s = fsig(z);
      return s * (1.f + z * (1.f - s));
    }
    case ACT_ELU: return z > 0.f ? 1.f : __expf(z);
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_TANH: {
      const float t = 2.f * fsig(2.f * z) - 1.f;
      return 1.f - t * t;
    }
    default: return 1.f;
  }
}
// compile-time activation forms for the epilogue loops (common.h SRL_ACT_SPECIALIZE)
template <int ACTC>
__device__ __forceinline__ float cact_c(float z, int act) {
  if constexpr (ACTC == ACT_SILU) return z * fsig(z);
  else return cact(z, act);
}
template <int ACTC>
__device__ __forceinline__ float cact_grad_c(float z, int act) {
  if constexpr (ACTC == ACT_SILU) {
    const float s = fsig(z);
    return s * (1.f + z * (1.f - s));
  } else {
    return cact_grad(z, act);
  }
}

// ------------------------------------------------------------------------------------- loaders
// A loader fills a ROWS x BK tile (row-major, k contiguous, stride LDK) of LDS from one K stage.
// Each thread owns NV float4 slots; load() issues the global reads into registers (so the next
// stage's latency hides behind the current stage's MFMAs), store() writes them to LDS.

// DOWN gather: rows = small-grid pixels m=(n,p,q), k = tap*Cb + b; Q is NHWC on the large grid.
// Cb is either a multiple of 32 (every BK = 32 chunk of K lies inside one tap: the tap is a per-stage
// scalar) or a power of two below 32 (the 4-channel image input: taps change inside a chunk).
template <int ROWS, int NTH>
struct DownGather {
  static constexpr int NV = (ROWS * BK / 4 + NTH - 1) / NTH;  // a 32-row tile under 512 threads: half a slot
  static constexpr bool FULL = ROWS * BK / 4 % NTH == 0;
  const float* Q;
  int Cb, lCb, lSH, lSW, M;
  int pix[NV], py[NV], px[NV];  // per slot: n*LH*LW, 2p-1, 2q-1 (pix = -1: row out of range)
  __device__ void init(int m0, int) {
    const int LH = 2 << lSH, LW = 2 << lSW;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v, m = m0 + (idx >> 3);
      const int n = m >> (lSH + lSW), p = (m >> lSW) & ((1 << lSH) - 1), q = m & ((1 << lSW) - 1);
      pix[v] = (m < M && (FULL || idx < ROWS * BK / 4)) ? n * LH * LW : -1;
      py[v] = 2 * p - 1;
      px[v] = 2 * q - 1;
    }
  }
  __device__ void load(int k0, f4* r) const {
    const int LH = 2 << lSH, LW = 2 << lSW;
    if (Cb >= BK) {
      const int tap = k0 / Cb, b0 = k0 - tap * Cb, dy = tap >> 2, dx = tap & 3;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int b = b0 + 4 * ((threadIdx.x + NTH * v) & 7);
        const int iy = py[v] + dy, ix = px[v] + dx;
        const bool ok = pix[v] >= 0 && iy >= 0 && iy < LH && ix >= 0 && ix < LW;
        r[v] = *(const f4*)zsrc(ok, Q + ((pix[v] + iy * LW + ix) * Cb + b));  // < 2^31 (host-checked)
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int k = k0 + 4 * ((threadIdx.x + NTH * v) & 7);
      const int tap = k >> lCb, b = k & (Cb - 1);
      const int iy = py[v] + (tap >> 2), ix = px[v] + (tap & 3);
      const bool ok = pix[v] >= 0 && iy >= 0 && iy < LH && ix >= 0 && ix < LW;
      r[v] = *(const f4*)zsrc(ok, Q + ((size_t)(pix[v] + iy * LW + ix) << lCb) + b);
    }
  }
  __device__ void store(const f4* r, float* s) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      if (FULL || idx < ROWS * BK / 4) *(f4*)(s + (idx >> 3) * LDK + 4 * (idx & 7)) = r[v];
    }
  }
};

// UP gather: rows = large-grid pixels of parity class (cy,cx) (blockIdx.z), m=(n,u,v) -> (2u+cy, 2v+cx);
// k = t*Ca + a with t = (th,tw) in 2x2; source pixel (u+cy-th, v+cx-tw) of P (NHWC, small grid).
// Ca is a multiple of 32, so a BK chunk lies inside one tap t.
template <int ROWS, int NTH>
struct UpGather {
  static constexpr int NV = (ROWS * BK / 4 + NTH - 1) / NTH;  // a 32-row tile under 512 threads: half a slot
  static constexpr bool FULL = ROWS * BK / 4 % NTH == 0;
  const float* P;
  int Ca, lSH, lSW, M;
  int pix[NV], pu[NV], pv[NV];
  __device__ void init(int m0, int cls) {
    const int cy = cls >> 1, cx = cls & 1;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v, m = m0 + (idx >> 3);
      const int n = m >> (lSH + lSW), u = (m >> lSW) & ((1 << lSH) - 1), w = m & ((1 << lSW) - 1);
      pix[v] = (m < M && (FULL || idx < ROWS * BK / 4)) ? n << (lSH + lSW) : -1;
      pu[v] = u + cy;
      pv[v] = w + cx;
    }
  }
  __device__ void load(int k0, f4* r) const {
    const int SH = 1 << lSH, SW = 1 << lSW;
    const int t = k0 / Ca, a0 = k0 - t * Ca, dy = t >> 1, dx = t & 1;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int a = a0 + 4 * ((threadIdx.x + NTH * v) & 7);
      const int p = pu[v] - dy, q = pv[v] - dx;
      const bool ok = pix[v] >= 0 && p >= 0 && p < SH && q >= 0 && q < SW;
      r[v] = *(const f4*)zsrc(ok, P + ((pix[v] + p * SW + q) * Ca + a));  // < 2^31 (host-checked)
    }
  }
  __device__ void store(const f4* r, float* s) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      if (FULL || idx < ROWS * BK / 4) *(f4*)(s + (idx >> 3) * LDK + 4 * (idx & 7)) = r[v];
    }
  }
};

// Packed weights, rows = output columns, k contiguous: W + (n0 + row) * K + k (+ class offset).
template <int ROWS, int NTH>
struct Dense {
  static constexpr int NV = ROWS * BK / 4 / NTH;
  const float* W;
  int K;
  size_t cls_stride;  // UP: per parity-class packed block; 0 otherwise
  const float* base;
  __device__ void init(int n0, int cls) { base = W + cls_stride * cls + (size_t)n0 * K; }
  __device__ void load(int k0, f4* r) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      r[v] = *(const f4*)(base + (size_t)(idx >> 3) * K + k0 + 4 * (idx & 7));
    }
  }
  __device__ void store(const f4* r, float* s) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      *(f4*)(s + (idx >> 3) * LDK + 4 * (idx & 7)) = r[v];
    }
  }
};

// WGRAD operand A: rows = channels a of P (NHWC, small grid), k = pixels: float4 along a, transposed
// into LDS (4 scalar writes; consecutive lanes = consecutive pixels: conflict-free).
template <int ROWS, int NTH>
struct WgP {
  static constexpr int NV = ROWS * BK / 4 / NTH;
  const float* P;
  int Ca, M, a0;
  __device__ void init(int r0) { a0 = r0; }
  __device__ void load(int k0, f4* r) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      const int m = k0 + (idx & 31), a = a0 + 4 * (idx >> 5);
      r[v] = *(const f4*)zsrc(m < M, P + (m * Ca + a));
    }
  }
  __device__ void store(const f4* r, float* s) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      float* d = s + 4 * (idx >> 5) * LDK + (idx & 31);
      d[0] = r[v][0];
      d[LDK] = r[v][1];
      d[2 * LDK] = r[v][2];
      d[3 * LDK] = r[v][3];
    }
  }
};

// WGRAD operand B: rows j = tap*Cb + b, k = small-grid pixels m=(n,p,q); value Q[n, 2p-1+kh, 2q-1+kw, b].
// A thread's rows are fixed for the whole launch: their (tap, b) split is done once in init.
template <int ROWS, int NTH>
struct WgQ {
  static constexpr int NV = ROWS * BK / 4 / NTH;
  const float* Q;
  int Cb, lSH, lSW, M;
  int dy[NV], dx[NV], bo[NV];
  __device__ void init(int j0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int j = j0 + 4 * ((threadIdx.x + NTH * v) >> 5);
      const int tap = j / Cb;
      dy[v] = (tap >> 2) - 1;
      dx[v] = (tap & 3) - 1;
      bo[v] = j - tap * Cb;
    }
  }
  __device__ void load(int k0, f4* r) const {
    const int LH = 2 << lSH, LW = 2 << lSW;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      const int m = k0 + (idx & 31);
      const int n = m >> (lSH + lSW), p = (m >> lSW) & ((1 << lSH) - 1), q = m & ((1 << lSW) - 1);
      const int iy = 2 * p + dy[v], ix = 2 * q + dx[v];
      const bool ok = m < M && iy >= 0 && iy < LH && ix >= 0 && ix < LW;
      r[v] = *(const f4*)zsrc(ok, Q + (((n * LH + iy) * LW + ix) * Cb + bo[v]));
    }
  }
  __device__ void store(const f4* r, float* s) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      float* d = s + 4 * (idx >> 5) * LDK + (idx & 31);
      d[0] = r[v][0];
      d[LDK] = r[v][1];
      d[2 * LDK] = r[v][2];
      d[3 * LDK] = r[v][3];
    }
  }
};

// ------------------------------------------------------------------------------ row geometry
// Maps a GEMM output row (pixel of the kernel's M space) to its pixel index in the output grid.
struct RowDown {  // rows are the output pixels themselves
  int cls;
  __device__ int operator()(int m) const { return m; }
};
struct RowUp {  // rows are parity-class pixels of the large grid
  int lSH, lSW;
  int cls;  // parity class of this workgroup (set by the kernel)
  __device__ int operator()(int m) const {
    const int n = m >> (lSH + lSW), u = (m >> lSW) & ((1 << lSH) - 1), v = m & ((1 << lSW) - 1);
    const int cy = cls >> 1, cx = cls & 1;
    return ((n << (lSH + 1)) + 2 * u + cy) * (2 << lSW) + 2 * v + cx;
  }
};

// acc element (i, j, r) of a wave -> tile row / col (v_mfma_f32_32x32x2_f32 C/D layout)
template <int TM, int TN, int WN>
struct Frag {
  int wm, wn, lane;
  __device__ int row(int i, int r) const { return wm * TM * 32 + i * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3); }
  __device__ int col(int j) const { return wn * TN * 32 + j * 32 + (lane & 31); }
};

// The LayerNorm epilogues work on whole channel rows: the accumulator tile is staged through LDS
// in TM chunks of WM*32 rows ([row][BN + 4] floats, fits the main-loop LDS), then every row is
// processed by LPR lanes (CPL contiguous channels each: vector loads/stores, row reductions by xor
// shuffles inside the LPR-lane segment).  This keeps the epilogue's register footprint small, so
// the MFMA main loop keeps its occupancy.
// Four channels per lane up to 256 channels (16 B vector LDS reads / global stores; a row of 32
// channels is 8 lanes, so a row reduction is 3 xor levels and a wave covers 8 rows per pass); wider
// rows use all 64 lanes (8 / 12 / 16 channels per lane at 512 / 768 / 1024), and the 3 x 2^k widths
// (96, 192, 384, 768: the XL multiplier) take 3 / 6 / 12 channels per lane.  One channel per lane
// (the first version, 32/64 lanes per row) made the LN epilogue of the narrow E1 / D4 layers
// (K = 64: two main-loop stages) dominate their kernels: 14% MFMA busy, 57% of wave cycles parked.
__host__ __device__ constexpr int pow2_part(int v) { return v & -v; }
template <int BN>
struct RowGeo {
  static constexpr int P2 = pow2_part(BN);
  static constexpr int LPR = (BN == P2 ? (BN / 4 < 64 ? BN / 4 : 64) : (P2 < 64 ? P2 : 64));  // lanes per row
  static constexpr int CPL = BN / LPR;                                                    // channels per lane
  static constexpr int RPW = 64 / LPR;                                                    // rows per wave pass
  static constexpr int PITCH = BN + 4;                                                    // LDS row pitch (floats)
  static_assert(LPR >= 1 && LPR <= 64 && (LPR & (LPR - 1)) == 0 && CPL * LPR == BN && CPL <= 16, "RowGeo: BN");
};

template <int TM, int TN, int WN>
__device__ __forceinline__ void stage_chunk(const f16v (&acc)[TM][TN], int i, const Frag<TM, TN, WN>& f, float* s,
                                            int pitch) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      s[(f.wm * 32 + 8 * (r >> 2) + 4 * (f.lane >> 5) + (r & 3)) * pitch + f.col(j)] = acc[i][j][r];
}

// sum over aligned segments of LPR lanes, every lane of the segment gets it: DPP quad butterflies, half-row /
// row mirrors (8 / 16 lanes), readlanes across rows (32 / 64) - no LDS-crossbar shuffles (common.h)
template <int LPR>
__device__ __forceinline__ float lseg_sum(float v) {
  static_assert(LPR == 1 || LPR == 2 || LPR == 4 || LPR == 8 || LPR == 16 || LPR == 32 || LPR == 64, "lseg_sum: LPR");
  if constexpr (LPR >= 2) v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (LPR >= 4) v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (LPR >= 8) v += dpp_f<0x141>(v);  // row_half_mirror
  if constexpr (LPR >= 16) v += dpp_f<0x140>(v); // row_mirror
  if constexpr (LPR == 32) {
    const float a = lane_f(v, 0) + lane_f(v, 16), b = lane_f(v, 32) + lane_f(v, 48);
    v = (threadIdx.x & 32) ? b : a;
  } else if constexpr (LPR == 64) {
    v = (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
  }
  return v;
}

// CPL contiguous floats at p (16-B aligned when CPL % 4 == 0, 8-B when CPL % 2 == 0)
template <int CPL>
__device__ __forceinline__ void ld_cpl(const float* p, float (&v)[CPL]) {
  if constexpr (CPL % 4 == 0) {
#pragma unroll
    for (int e = 0; e < CPL; e += 4) {
      const f4 t = *(const f4*)(p + e);
      v[e] = t[0]; v[e + 1] = t[1]; v[e + 2] = t[2]; v[e + 3] = t[3];
    }
  } else if constexpr (CPL % 2 == 0) {
#pragma unroll
    for (int e = 0; e < CPL; e += 2) {
      const float2 t = *(const float2*)(p + e);
      v[e] = t.x; v[e + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < CPL; ++e) v[e] = p[e];
  }
}
template <int CPL>
__device__ __forceinline__ void st_cpl(float* p, const float (&v)[CPL]) {
  if constexpr (CPL % 4 == 0) {
#pragma unroll
    for (int e = 0; e < CPL; e += 4) *(f4*)(p + e) = f4{v[e], v[e + 1], v[e + 2], v[e + 3]};
  } else if constexpr (CPL % 2 == 0) {
#pragma unroll
    for (int e = 0; e < CPL; e += 2) *(float2*)(p + e) = make_float2(v[e], v[e + 1]);
  } else {
#pragma unroll
    for (int e = 0; e < CPL; ++e) p[e] = v[e];
  }
}

// ------------------------------------------------------------------------------------ epilogues
// NW = waves of the workgroup (WM x WN); the tile rows of one staged chunk are R = WM * 32.
struct EpiLNAct : EpiLNActP {  // z = acc (NHWC), y = act(LN_c(z)) (NHWC or NCHW-flat), mean/rstd per pixel
  template <int BM, int BN, int TM, int TN, int WM, int WN, class RM>
  __device__ void run(f16v (&acc)[TM][TN], const Frag<TM, TN, WN>& f, int m0, float* lds, const RM& rm) {
    SRL_ACT_SPECIALIZE(act, (run_t<BM, BN, TM, TN, WM, WN, RM, ACTC>(acc, f, m0, lds, rm)));
  }
  template <int BM, int BN, int TM, int TN, int WM, int WN, class RM, int ACTC>
  __device__ void run_t(f16v (&acc)[TM][TN], const Frag<TM, TN, WN>& f, int m0, float* lds, const RM& rm) {
    using G = RowGeo<BN>;
    constexpr int NW = WM * WN, R = WM * 32, CPL = G::CPL, LPR = G::LPR;
    const int w = threadIdx.x >> 6, lr = f.lane / LPR, lc = f.lane % LPR, c0 = lc * CPL;
    float gam[CPL], bet[CPL];
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      gam[e] = gamma ? gamma[c0 + e] : 1.f;
      bet[e] = beta ? beta[c0 + e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      __syncthreads();
      stage_chunk<TM, TN, WN>(acc, i, f, lds, G::PITCH);
      __syncthreads();
      for (int q0 = w * G::RPW; q0 < R; q0 += NW * G::RPW) {
        const int q = q0 + lr;
        const int m = m0 + (q >> 5) * TM * 32 + i * 32 + (q & 31);
        float v[CPL];
        ld_cpl<CPL>(lds + q * G::PITCH + c0, v);
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < CPL; ++e) s += v[e];
        const float mu = lseg_sum<LPR>(s) * (1.f / BN);
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < CPL; ++e) d += (v[e] - mu) * (v[e] - mu);
        const float rs = rsqrtf(lseg_sum<LPR>(d) * (1.f / BN) + eps);
        if (m < M) {
          const int pix = rm(m);
          st_cpl<CPL>(z + (size_t)pix * BN + c0, v);
          float yv[CPL];
#pragma unroll
          for (int e = 0; e < CPL; ++e) yv[e] = cact_c<ACTC>((v[e] - mu) * rs * gam[e] + bet[e], act);
          if (y_nchw) {
            const int n = pix >> lHW, hw = pix & ((1 << lHW) - 1);
#pragma unroll
            for (int e = 0; e < CPL; ++e) y[(((size_t)n * BN + c0 + e) << lHW) + hw] = yv[e];
          } else {
            st_cpl<CPL>(y + (size_t)pix * BN + c0, yv);
          }
          if (lc == 0) {
            mean[pix] = mu;
            rstd[pix] = rs;
          }
        }
      }
    }
  }
};

struct EpiLNBwd : EpiLNBwdP {  // acc = dy (grad of y = act(LN(z))); dz = d/dz; dgamma/dbeta += column sums
  template <int BM, int BN, int TM, int TN, int WM, int WN, class RM>
  __device__ void run(f16v (&acc)[TM][TN], const Frag<TM, TN, WN>& f, int m0, float* lds, const RM& rm) {
    SRL_ACT_SPECIALIZE(act, (run_t<BM, BN, TM, TN, WM, WN, RM, ACTC>(acc, f, m0, lds, rm)));
  }
  template <int BM, int BN, int TM, int TN, int WM, int WN, class RM, int ACTC>
  __device__ void run_t(f16v (&acc)[TM][TN], const Frag<TM, TN, WN>& f, int m0, float* lds, const RM& rm) {
    using G = RowGeo<BN>;
    constexpr int NW = WM * WN, NTH = 64 * NW, R = WM * 32, CPL = G::CPL, LPR = G::LPR;
    const int w = threadIdx.x >> 6, lr = f.lane / LPR, lc = f.lane % LPR, c0 = lc * CPL;
    float gam[CPL], bet[CPL], cg[CPL], cb[CPL];
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      gam[e] = gamma ? gamma[c0 + e] : 1.f;
      bet[e] = beta ? beta[c0 + e] : 0.f;
      cg[e] = 0.f;
      cb[e] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      __syncthreads();
      stage_chunk<TM, TN, WN>(acc, i, f, lds, G::PITCH);
      __syncthreads();
      for (int q0 = w * G::RPW; q0 < R; q0 += NW * G::RPW) {
        const int q = q0 + lr;
        const int m = m0 + (q >> 5) * TM * 32 + i * 32 + (q & 31);
        const bool ok = m < M;
        const int pix = ok ? rm(m) : 0;
        float dy[CPL], zz[CPL], x[CPL], dx[CPL];
        ld_cpl<CPL>(lds + q * G::PITCH + c0, dy);
        if (ok) {
          ld_cpl<CPL>(z + (size_t)pix * BN + c0, zz);
        } else {
#pragma unroll
          for (int e = 0; e < CPL; ++e) zz[e] = 0.f;
        }
        const float mu = ok ? mean[pix] : 0.f, rs = ok ? rstd[pix] : 0.f;
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          x[e] = (zz[e] - mu) * rs;
          const float da = ok ? dy[e] * cact_grad_c<ACTC>(x[e] * gam[e] + bet[e], act) : 0.f;
          cg[e] += da * x[e];
          cb[e] += da;
          dx[e] = da * gam[e];
          a1 += dx[e];
          a2 += dx[e] * x[e];
        }
        a1 = lseg_sum<LPR>(a1) * (1.f / BN);
        a2 = lseg_sum<LPR>(a2) * (1.f / BN);
        if (ok) {
          float o[CPL];
#pragma unroll
          for (int e = 0; e < CPL; ++e) o[e] = rs * (dx[e] - a1 - x[e] * a2);
          st_cpl<CPL>(dz + (size_t)pix * BN + c0, o);
        }
      }
    }
    if (part || dgamma || dbeta) {
      // rows of a wave pass share columns: fold the RPW row groups, then the NW waves through LDS
#pragma unroll
      for (int e = 0; e < CPL; ++e)
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) {
          cg[e] += __shfl_xor(cg[e], o, 64);
          cb[e] += __shfl_xor(cb[e], o, 64);
        }
      __syncthreads();
      if (lr == 0) {
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          lds[w * BN + c0 + e] = cg[e];
          lds[NW * BN + w * BN + c0 + e] = cb[e];
        }
      }
      __syncthreads();
      // one row of 2 * BN column sums per workgroup (reduced later in a fixed order), or float atomics
      float* prow = part ? part + (size_t)(blockIdx.x + gridDim.x * blockIdx.z) * 2 * BN : nullptr;
      for (int c = threadIdx.x; c < BN; c += NTH) {
        float sg = 0.f, sb = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          sg += lds[q * BN + c];
          sb += lds[NW * BN + q * BN + c];
        }
        if (prow) {
          prow[c] = sg;
          prow[BN + c] = sb;
        } else {
          if (dgamma) atomicAdd(dgamma + c, sg);
          if (dbeta) atomicAdd(dbeta + c, sb);
        }
      }
    }
  }
};

struct EpiPlain : EpiPlainP {  // out = acc + bias[c] + c0 for c < Nreal; NHWC (ld = Nreal) or NCHW-flat
  template <int BM, int BN, int TM, int TN, int WM, int WN, class RM>
  __device__ void run(f16v (&acc)[TM][TN], const Frag<TM, TN, WN>& f, int m0, float*, const RM& rm) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + f.row(i, r);
        if (m >= M) continue;
        const int pix = rm(m);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int c = f.col(j);
          if (c >= Nreal) continue;
          const float v = acc[i][j][r] + (bias ? bias[c] : 0.f) + c0;
          if (nchw) {
            const int n = pix >> lHW, hw = pix & ((1 << lHW) - 1);
            out[(((size_t)n * Nreal + c) << lHW) + hw] = v;
          } else {
            out[(size_t)pix * Nreal + c] = v;
          }
        }
      }
  }
};

// --------------------------------------------------------------------------- GEMM main loops
// Tile BM x BN, WM x WN waves of (TM*32) x (TN*32); 64*WM*WN threads; one LDS stage + register
// prefetch of the next stage (a double-buffered form with one barrier per stage measured no gain:
// profiles/r4_conv_ab.md, profiles/r4_conv_db_wide.md; removed).
// Waves per SIMD the register allocation targets: 3 for the 4-wave 32 / 64 / 128-column tiles (<= 168 VGPRs, no
// spill: three workgroups per CU overlap one another's prologue / epilogue; Atari-100k stack -1 %), the compiler's
// default (2) elsewhere - the 96 / 192 / 384-column XL tiles miss the target and slow down 2-40 % when forced.
constexpr int igemm_min_waves(int BN, int WM, int WN) { return (WM * WN == 4 && (BN == 32 || BN == 64 || BN == 128)) ? 3 : 1; }

template <int BM, int BN, int WM, int WN, class LA, class LB, class EP, class RM>
__global__ __launch_bounds__(64 * WM * WN, igemm_min_waves(BN, WM, WN)) void igemm_kernel(LA la, LB lb, EP ep, RM rm, int K,
                                                                                         int ncls, int remap) {
  constexpr int NTH = 64 * WM * WN, TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && TM * WM * 32 == BM && TN * WN * 32 == BN, "bad tile");
  constexpr int LDS_MAIN = (BM + BN) * LDK;
  constexpr int LDS_EPI = WM * 32 * (BN + 4) > 2 * WM * WN * BN ? WM * 32 * (BN + 4) : 2 * WM * WN * BN;
  __shared__ float lds[LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI];
  float* As = lds;
  float* Bs = lds + BM * LDK;
  // XCD-aware tile order (remap): the hardware deals workgroups round-robin over the 8 XCDs, so
  // XCD x runs blocks x, x+8, ...; give it a contiguous run of M tiles (halo rows shared in its L2)
  // with the ncls parity classes of a tile back to back (UP: the 4 classes read the same input pixels)
  int mt, cls;
  if (remap) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, per = ((int)gridDim.x >> 3) / ncls;
    cls = j % ncls;
    mt = x * per + j / ncls;
  } else {
    mt = blockIdx.x;
    cls = blockIdx.z;
  }
  const int m0 = mt * BM, n0 = blockIdx.y * BN;
  la.init(m0, cls);
  lb.init(n0, cls);
  rm.cls = cls;
  Frag<TM, TN, WN> f;
  f.lane = threadIdx.x & 63;
  f.wm = (threadIdx.x >> 6) / WN;
  f.wn = (threadIdx.x >> 6) % WN;
  f16v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f4 ra[LA::NV], rb[LB::NV];
  la.load(0, ra);
  lb.load(0, rb);
  const int arow = f.wm * TM * 32 + (f.lane & 31), brow = f.wn * TN * 32 + (f.lane & 31), kof = 4 * (f.lane >> 5);
  auto stage_mfma = [&](const float* A_, const float* B_) {
#pragma unroll
    for (int s = 0; s < BK / 8; ++s) {
      f4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *(const f4*)(A_ + (arow + 32 * i) * LDK + 8 * s + kof);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *(const f4*)(B_ + (brow + 32 * j) * LDK + 8 * s + kof);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    }
  };
  for (int k0 = 0; k0 < K; k0 += BK) {
    __syncthreads();
    la.store(ra, As);
    lb.store(rb, Bs);
    __syncthreads();
    if (k0 + BK < K) {
      la.load(k0 + BK, ra);
      lb.load(k0 + BK, rb);
    }
    stage_mfma(As, Bs);
  }
  __syncthreads();
  ep.template run<BM, BN, TM, TN, WM, WN>(acc, f, m0, lds, rm);
}

// WGRAD: rows a (Ca), cols (tap,b) (16 Cb), K = pixel range of split blockIdx.z; writes the partial slab.
// MINW: waves per SIMD targeted by the register allocation (3 = the short-K form, see wgrad_cfg)
template <int BM, int BN, int WM, int WN, int MINW = 1>
__global__ __launch_bounds__(64 * WM * WN, MINW) void wgrad_kernel(WgP<BM, 64 * WM * WN> la, WgQ<BN, 64 * WM * WN> lb,
                                                              float* slab, int ldn, int Mrows, int kper, int remap) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  __shared__ float lds[(BM + BN) * LDK];
  float* As = lds;
  float* Bs = lds + BM * LDK;
  // XCD-aware order (remap, grid size a multiple of 8): workgroups are dealt round-robin over the 8 XCDs, so
  // XCD x runs linear ids x, x + 8, ...; give it a contiguous run of (split, tile) pairs instead, i.e. whole
  // K splits, so every output tile of a split reads that split's P / Q pixels from the same L2
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (remap) {
    const int gxy = gridDim.x * gridDim.y;
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int L = (b & 7) * ((gxy * (int)gridDim.z) >> 3) + (b >> 3);
    bz = L / gxy;
    const int t = L - bz * gxy;
    by = t / gridDim.x;
    bx = t - by * gridDim.x;
  }
  const int r0 = bx * BM, c0 = by * BN;
  la.init(r0);
  lb.init(c0);
  const int kb = bz * kper, ke = kb + kper;
  Frag<TM, TN, WN> f;
  f.lane = threadIdx.x & 63;
  f.wm = (threadIdx.x >> 6) / WN;
  f.wn = (threadIdx.x >> 6) % WN;
  f16v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f4 ra[WgP<BM, 64 * WM * WN>::NV], rb[WgQ<BN, 64 * WM * WN>::NV];
  la.load(kb, ra);
  lb.load(kb, rb);
  const int arow = f.wm * TM * 32 + (f.lane & 31), brow = f.wn * TN * 32 + (f.lane & 31), kof = 4 * (f.lane >> 5);
  for (int k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();
    la.store(ra, As);
    lb.store(rb, Bs);
    __syncthreads();
    if (k0 + BK < ke) {
      la.load(k0 + BK, ra);
      lb.load(k0 + BK, rb);
    }
#pragma unroll
    for (int s = 0; s < BK / 8; ++s) {
      f4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *(const f4*)(As + (arow + 32 * i) * LDK + 8 * s + kof);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *(const f4*)(Bs + (brow + 32 * j) * LDK + 8 * s + kof);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    }
  }
  float* out = slab + (size_t)bz * Mrows * ldn;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j) out[(size_t)(r0 + f.row(i, r)) * ldn + c0 + f.col(j)] = acc[i][j][r];
}

// dW[a][b][kh][kw] = sum_s slab[s][a][tap*Cbp + b]   (b < Cb).  Block = 16 float4 columns (64 slab
// entries) x 16 split groups; each thread sums every 16th split of its float4, LDS combines the groups.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw, int S,
                                                           int Ca, int Cbp, int Cb) {
  __shared__ f4 part[16][17];
  const int per = 16 * Cbp, tot = Ca * per;
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int idx = (blockIdx.x * 16 + col) * 4;  // first of 4 consecutive slab entries
  f4 acc = zero4();
  if (idx < tot) {
    const f4* src = (const f4*)(slab + idx);
    const size_t stride = (size_t)tot / 4;
    // splits summed in split order; 8 loads issued before their adds (the single-tile layers run S = 1024
    // splits through 32 workgroups: 64 splits per thread, one memory latency per batch instead of per load)
    int k = grp;
    for (; k + 7 * 16 < S; k += 8 * 16) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(k + 16 * u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; k < S; k += 16) acc += src[(size_t)k * stride];
  }
  part[grp][col] = acc;
  __syncthreads();
  if (grp == 0 && idx < tot) {
    f4 s = zero4();
#pragma unroll
    for (int g = 0; g < 16; ++g) s += part[g][col];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = idx + e, a = i / per, rem = i - a * per, tap = rem / Cbp, b = rem - tap * Cbp;
      if (b < Cb) dw[((size_t)a * Cb + b) * 16 + tap] = s[e];
    }
  }
}

// W[A][B][4][4] -> DOWN pack [A][16][Bp] (b >= B zero)
__global__ void pack_down_kernel(const float* __restrict__ w, float* __restrict__ out, int A, int B, int Bp) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= A * 16 * Bp) return;
  const int a = idx / (16 * Bp), rem = idx - a * 16 * Bp, tap = rem / Bp, b = rem - tap * Bp;
  out[idx] = b < B ? w[((size_t)a * B + b) * 16 + tap] : 0.f;
}

// W[A][B][4][4] -> UP pack [4 classes][Bp][4 t][A]: class (cy,cx), t = (th,tw), kh = 1-cy+2th, kw = 1-cx+2tw
__global__ void pack_up_kernel(const float* __restrict__ w, float* __restrict__ out, int A, int B, int Bp) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 4 * Bp * 4 * A) return;
  const int a = idx % A, t = (idx / A) & 3, b = (idx / (4 * A)) % Bp, cls = idx / (4 * A * Bp);
  const int kh = 1 - (cls >> 1) + 2 * (t >> 1), kw = 1 - (cls & 1) + 2 * (t & 1);
  out[idx] = b < B ? w[((size_t)a * B + b) * 16 + kh * 4 + kw] : 0.f;
}

// Every weight pack of a conv stack in ONE launch (the forward's and the backward's forms of every layer: they depend
// only on the weights, which are fixed for the whole step): job j = blockIdx.y, kind 0 = DOWN, 1 = UP (as above).
constexpr int MAX_PACK_JOBS = 16;
struct PackJobs {
  const float* w[MAX_PACK_JOBS];
  float* out[MAX_PACK_JOBS];
  int A[MAX_PACK_JOBS], B[MAX_PACK_JOBS], Bp[MAX_PACK_JOBS], kind[MAX_PACK_JOBS];
};
__global__ void multi_pack_kernel(PackJobs jobs) {
  const int j = blockIdx.y;
  const int A = jobs.A[j], B = jobs.B[j], Bp = jobs.Bp[j];
  const float* __restrict__ w = jobs.w[j];
  float* __restrict__ out = jobs.out[j];
  const int tot = A * 16 * Bp;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += gridDim.x * blockDim.x) {
    if (jobs.kind[j] == 0) {
      const int a = idx / (16 * Bp), rem = idx - a * 16 * Bp, tap = rem / Bp, b = rem - tap * Bp;
      out[idx] = b < B ? w[((size_t)a * B + b) * 16 + tap] : 0.f;
    } else {
      const int a = idx % A, t = (idx / A) & 3, b = (idx / (4 * A)) % Bp, cls = idx / (4 * A * Bp);
      const int kh = 1 - (cls >> 1) + 2 * (t >> 1), kw = 1 - (cls & 1) + 2 * (t & 1);
      out[idx] = b < B ? w[((size_t)a * B + b) * 16 + kh * 4 + kw] : 0.f;
    }
  }
}

// NCHW (uint8 or f32) with C <= 4 channels -> NHWC4 f32, scaled; channel C..3 = 0
template <typename T>
__global__ void to_nhwc4_kernel(const T* __restrict__ x, f4* __restrict__ out, int N, int C, int HW, float scale) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * HW) return;
  const int n = idx / HW, hw = idx - n * HW;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < C; ++c) v[c] = (float)x[((size_t)n * C + c) * HW + hw] * scale;
  out[idx] = f4{v[0], v[1], v[2], v[3]};
}

// to_nhwc4 of an f32 NCHW tensor (the image gradient entering the decoder backward) that also sums each channel over
// the block's pixels: part[block][c] (c < C), summed over the blocks in a fixed order by ln_part_reduce_kernel - the
// last layer's bias gradient without a second pass over the 50 MB gradient
__global__ __launch_bounds__(256) void to_nhwc4_sum_kernel(const float* __restrict__ x, f4* __restrict__ out, int N, int C,
                                                           int HW, float* __restrict__ part) {
  __shared__ float red[4][4];
  const int idx = blockIdx.x * 256 + threadIdx.x;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (idx < N * HW) {
    const int n = idx / HW, hw = idx - n * HW;
    for (int c = 0; c < C; ++c) v[c] = x[((size_t)n * C + c) * HW + hw];
    out[idx] = f4{v[0], v[1], v[2], v[3]};
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float s = wave_sum_dpp(v[c]);
    if ((threadIdx.x & 63) == 0) red[w][c] = s;
  }
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    part[(size_t)blockIdx.x * C + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  }
}

// Row LayerNorm+act backward with dy in NCHW-flat order (the encoder's last stage feeds the flat
// embedding); z NHWC [M][C]; one wave per pixel row, channel c = lane + 64 e (e < CPL, c < C); column
// partials per block, one atomic per channel per block.
template <int CPL, int ACTC>
__global__ __launch_bounds__(256) void ln_bwd_flat_kernel(const float* __restrict__ dy, const float* __restrict__ z,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          float* __restrict__ dz, float* dgamma, float* dbeta, int M, int C,
                                                          int lHW, int act, int rows_per_block) {
  __shared__ float cr[2][4][64 * CPL];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float invC = 1.f / (float)C;
  float cg[CPL], cb[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) cg[e] = cb[e] = 0.f;
  const int rb = blockIdx.x * rows_per_block;
  for (int m = rb + w; m < min(M, rb + rows_per_block); m += 4) {
    const float mu = mean[m], rs = rstd[m];
    const int n = m >> lHW, hw = m & ((1 << lHW) - 1);
    float xh[CPL], dxh[CPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < CPL; ++e) {
      const int c = lane + 64 * e;
      xh[e] = dxh[e] = 0.f;
      if (c < C) {
        const float g = gamma ? gamma[c] : 1.f;
        xh[e] = (z[(size_t)m * C + c] - mu) * rs;
        const float a = xh[e] * g + (beta ? beta[c] : 0.f);
        const float da = dy[(((size_t)n * C + c) << lHW) + hw] * cact_grad_c<ACTC>(a, act);
        cg[e] += da * xh[e];
        cb[e] += da;
        dxh[e] = da * g;
      }
      s1 += dxh[e];
      s2 += dxh[e] * xh[e];
    }
    s1 = wave_sum(s1) * invC;
    s2 = wave_sum(s2) * invC;
#pragma unroll
    for (int e = 0; e < CPL; ++e)
      if (lane + 64 * e < C) dz[(size_t)m * C + lane + 64 * e] = rs * (dxh[e] - s1 - xh[e] * s2);
  }
#pragma unroll
  for (int e = 0; e < CPL; ++e) {
    cr[0][w][lane + 64 * e] = cg[e];
    cr[1][w][lane + 64 * e] = cb[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const float sg = cr[0][0][c] + cr[0][1][c] + cr[0][2][c] + cr[0][3][c];
    const float sb = cr[1][0][c] + cr[1][1][c] + cr[1][2][c] + cr[1][3][c];
    if (dgamma) atomicAdd(dgamma + c, sg);
    if (dbeta) atomicAdd(dbeta + c, sb);
  }
}

// The same backward one IMAGE per iteration: the image's dy block (C x HW floats, contiguous in NCHW) is read with
// coalesced loads and transposed through LDS ([hw][C + 1]: conflict-free both ways), so no load touches a cache
// line per lane (ln_bwd_flat_kernel's dy reads stride HW floats across the lanes).  Every workgroup holds its
// channel partials of dgamma / dbeta in registers over its images and writes them to part[block][2C]; a second
// kernel (ln_part_reduce_kernel) sums the blocks in a fixed order - no float atomics, bitwise reproducible.
template <int CPL, int ACTC>
__global__ __launch_bounds__(256) void ln_bwd_img_kernel(const float* __restrict__ dy, const float* __restrict__ z,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float* __restrict__ dz, float* __restrict__ part, int N, int C,
                                                         int lHW, int act, int ipb) {
  extern __shared__ float sm[];  // [HW][C + 1] dy tile, then [2][4][64 * CPL] partials
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int HW = 1 << lHW, ld = C + 1, CHW = C << lHW;
  const float invC = 1.f / (float)C;
  float cg[CPL], cb[CPL], g[CPL], bt[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) {
    const int c = lane + 64 * e;
    cg[e] = cb[e] = 0.f;
    g[e] = (c < C && gamma) ? gamma[c] : 1.f;
    bt[e] = (c < C && beta) ? beta[c] : 0.f;
  }
  const int n0 = blockIdx.x * ipb, n1 = min(N, n0 + ipb);
  for (int n = n0; n < n1; ++n) {
    const float* dyn = dy + (size_t)n * CHW;
    for (int e = threadIdx.x; e < CHW; e += 256) sm[(e & (HW - 1)) * ld + (e >> lHW)] = dyn[e];
    __syncthreads();
    for (int hw = w; hw < HW; hw += 4) {
      const int m = (n << lHW) + hw;
      const float mu = mean[m], rs = rstd[m];
      float xh[CPL], dxh[CPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        const int c = lane + 64 * e;
        xh[e] = dxh[e] = 0.f;
        if (c < C) {
          xh[e] = (z[(size_t)m * C + c] - mu) * rs;
          const float da = sm[hw * ld + c] * cact_grad_c<ACTC>(xh[e] * g[e] + bt[e], act);
          cg[e] += da * xh[e];
          cb[e] += da;
          dxh[e] = da * g[e];
        }
        s1 += dxh[e];
        s2 += dxh[e] * xh[e];
      }
      s1 = wave_sum(s1) * invC;
      s2 = wave_sum(s2) * invC;
#pragma unroll
      for (int e = 0; e < CPL; ++e)
        if (lane + 64 * e < C) dz[(size_t)m * C + lane + 64 * e] = rs * (dxh[e] - s1 - xh[e] * s2);
    }
    __syncthreads();
  }
  float* cr = sm;  // [2][4][64 * CPL]
#pragma unroll
  for (int e = 0; e < CPL; ++e) {
    cr[(0 * 4 + w) * 64 * CPL + lane + 64 * e] = cg[e];
    cr[(1 * 4 + w) * 64 * CPL + lane + 64 * e] = cb[e];
  }
  __syncthreads();
  float* pb = part + (size_t)blockIdx.x * 2 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float* a = cr + c;
    pb[c] = (a[0] + a[64 * CPL]) + (a[2 * 64 * CPL] + a[3 * 64 * CPL]);
    pb[C + c] = (a[4 * 64 * CPL] + a[5 * 64 * CPL]) + (a[6 * 64 * CPL] + a[7 * 64 * CPL]);
  }
}

// Sum of the rows [lo, hi) of column col of part[.][W] in a fixed order: 64 columns x 16 row groups per workgroup
// (each thread's rows lo + grp, lo + grp + 16, ... summed in 4 independent chains so their loads are in flight
// together), LDS combine in order; the result is valid on the threads of row group 0.
__device__ __forceinline__ float part_block_sum(const float* __restrict__ part, int lo, int hi, int W, int col,
                                                float (*red)[64]) {
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < W) {
    int b = lo + grp;
    for (; b + 48 < hi; b += 64) {
      s0 += part[(size_t)b * W + col];
      s1 += part[(size_t)(b + 16) * W + col];
      s2 += part[(size_t)(b + 32) * W + col];
      s3 += part[(size_t)(b + 48) * W + col];
    }
    for (; b < hi; b += 16) s0 += part[(size_t)b * W + col];
  }
  red[grp][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  float v = 0.f;
  if (grp == 0) {
#pragma unroll
    for (int g = 0; g < 16; ++g) v += red[g][cl];
  }
  return v;
}

// Rows [blockIdx.y * rpb, min(nb, (blockIdx.y + 1) * rpb)) of part[nb][W] summed (part_block_sum).  stage != null:
// stage[blockIdx.y][col] = sum (first pass of a two-pass reduction of a tall part); else out0[col] += sum (col < C),
// out1[col - C] += sum (C <= col < W) (= with assign).
__global__ __launch_bounds__(1024) void ln_part_reduce_kernel(const float* __restrict__ part, int nb, int W, int rpb,
                                                              float* __restrict__ stage, float* __restrict__ out0,
                                                              float* __restrict__ out1, int C, int assign) {
  __shared__ float red[16][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lo = blockIdx.y * rpb, hi = min(nb, lo + rpb);
  const float v = part_block_sum(part, lo, hi, W, col, red);
  if (threadIdx.x < 64 && col < W) {
    if (stage) {
      stage[(size_t)blockIdx.y * W + col] = v;
    } else if (col < C) {
      if (out0) out0[col] = assign ? v : out0[col] + v;
    } else if (out1) {
      out1[col - C] = assign ? v : out1[col - C] + v;
    }
  }
}

// rows of part summed per workgroup in the first pass of a two-pass reduction; a part buffer of nb rows needs
// part_stage_rows(nb) more rows behind it for the first pass's output
constexpr int PART_RPB = 64;
inline int part_stage_rows(int nb) { return (nb + PART_RPB - 1) / PART_RPB; }

// dgamma (columns < C) / dbeta (columns C..W) += column sums of part[nb][W]; part has part_stage_rows(nb) spare rows
// behind its nb rows when stage_ok (tall parts: a 64-rows-per-workgroup first pass spreads the loads over the chip)
static void launch_part_reduce(float* part, int nb, int W, float* out0, float* out1, int C, bool stage_ok, hipStream_t st,
                               bool assign = false) {
  const int cb = (W + 63) / 64, as = assign ? 1 : 0;
  if (stage_ok && nb > 2 * PART_RPB) {
    const int g = part_stage_rows(nb);
    float* stage = part + (size_t)nb * W;
    hipLaunchKernelGGL(ln_part_reduce_kernel, dim3(cb, g), dim3(1024), 0, st, part, nb, W, PART_RPB, stage, out0, out1, C,
                       0);
    hipLaunchKernelGGL(ln_part_reduce_kernel, dim3(cb, 1), dim3(1024), 0, st, stage, g, W, g, (float*)nullptr, out0,
                       out1, C, as);
  } else {
    hipLaunchKernelGGL(ln_part_reduce_kernel, dim3(cb, 1), dim3(1024), 0, st, part, nb, W, nb, (float*)nullptr, out0,
                       out1, C, as);
  }
}

// ConvT forward to a tiny channel count (the decoder's last layer: 1 or 3 image channels), on VALU:
// a workgroup owns a 16x16 tile of small-grid pixels of one image (+1 halo) staged in LDS (NHWC,
// 32 input channels per pass, CA / 32 passes); thread = one small-grid pixel (u, v), producing its 2x2
// large-grid outputs (the 4 parity classes).  The class / tap loops are workgroup-uniform, so the
// weights are read as LDS broadcasts ([tap][a][CO padded to 4]: one 16 B read per (tap, a)), one
// per-lane LDS read of the input channel feeds CO FMAs, and each output row pair is written as float2
// (x = 2v, 2v+1).  (First version: lanes of one wave mixed parity classes, so every FMA needed its own
// divergent LDS weight read - LDS-bound at ~180 us for N=1024.)
// out NCHW [n][co][y][x] = bias[co] + c0 + sum.
template <int CO>
__global__ __launch_bounds__(256) void up_small_kernel(const float* __restrict__ P, const float* __restrict__ W,
                                                       const float* __restrict__ bias, float c0, float* __restrict__ out,
                                                       int lSH, int lSW, int CA) {
  static_assert(CO >= 1 && CO <= 4, "up_small: CO <= 4");
  constexpr int T = 16, TH = T + 2, CC = 32;
  __shared__ float tile[TH * TH * (CC + 1)];
  __shared__ f4 ws[16 * CC];  // [kh*4+kw][a] -> (co 0..3)
  const int SH = 1 << lSH, SW = 1 << lSW;
  const int tx = SW / T;
  const int n = blockIdx.y, ty0 = (blockIdx.x / tx) * T, tx0 = (blockIdx.x % tx) * T;
  const int u = threadIdx.x >> 4, v = threadIdx.x & 15;
  float s[2][2][CO];
#pragma unroll
  for (int cy = 0; cy < 2; ++cy)
#pragma unroll
    for (int cx = 0; cx < 2; ++cx)
#pragma unroll
      for (int c = 0; c < CO; ++c) s[cy][cx][c] = 0.f;
  for (int a0 = 0; a0 < CA; a0 += CC) {
    __syncthreads();
    for (int i = threadIdx.x; i < 16 * CC; i += 256) {
      const int tap = i / CC, a = i % CC;
      f4 w = zero4();
#pragma unroll
      for (int c = 0; c < CO; ++c) w[c] = W[((a0 + a) * CO + c) * 16 + tap];
      ws[i] = w;
    }
    for (int i = threadIdx.x; i < TH * TH * (CC / 4); i += 256) {
      const int pixl = i / (CC / 4), aq = i % (CC / 4);
      const int p = ty0 - 1 + pixl / TH, q = tx0 - 1 + pixl % TH;
      f4 val = zero4();
      if (p >= 0 && p < SH && q >= 0 && q < SW) val = *(const f4*)(P + ((((size_t)n * SH + p) * SW + q) * CA) + a0 + 4 * aq);
      float* d = tile + pixl * (CC + 1) + 4 * aq;
      d[0] = val[0];
      d[1] = val[1];
      d[2] = val[2];
      d[3] = val[3];
    }
    __syncthreads();
#pragma unroll
    for (int cy = 0; cy < 2; ++cy)
#pragma unroll
      for (int cx = 0; cx < 2; ++cx)
#pragma unroll
        for (int th = 0; th < 2; ++th)
#pragma unroll
          for (int tw = 0; tw < 2; ++tw) {
            const float* src = tile + ((u + cy - th + 1) * TH + (v + cx - tw + 1)) * (CC + 1);
            const f4* wt = ws + ((1 - cy + 2 * th) * 4 + (1 - cx + 2 * tw)) * CC;
#pragma unroll 8
            for (int a = 0; a < CC; ++a) {
              const float pv = src[a];
              const f4 w = wt[a];
#pragma unroll
              for (int c = 0; c < CO; ++c) s[cy][cx][c] += pv * w[c];
            }
          }
  }
  const int LH = 2 * SH, LW = 2 * SW;
  const int y0 = 2 * (ty0 + u), x0 = 2 * (tx0 + v);
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    const float b = (bias ? bias[c] : 0.f) + c0;
#pragma unroll
    for (int cy = 0; cy < 2; ++cy)
      *(float2*)(out + (((size_t)n * CO + c) * LH + y0 + cy) * LW + x0) = make_float2(s[cy][0][c] + b, s[cy][1][c] + b);
  }
}

}  // namespace conv
}  // namespace srl

// =============================================================================== host launchers
using namespace srl::conv;

namespace {
int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}
template <class K, class... Args>
void launch(K kernel, dim3 grid, dim3 block, hipStream_t st, Args... args) {
  hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
}
}  // namespace

template <int BM, int BN, int WM, int WN, class LA, class RM>
static void dispatch_epi(const LA& la, const Dense<BN, 64 * WM * WN>& lb, const ConvEpi& e, const RM& rm, int K, int mtiles,
                         int ncls, hipStream_t st) {
  dim3 block(64 * WM * WN);
  const int remap = mtiles % 8 == 0 ? 1 : 0;
  const dim3 grid = remap ? dim3(mtiles * ncls, 1, 1) : dim3(mtiles, 1, ncls);
  if (e.mode == 0) {
    EpiLNAct ep;
    static_cast<EpiLNActP&>(ep) = e.ln;
    launch(igemm_kernel<BM, BN, WM, WN, LA, Dense<BN, 64 * WM * WN>, EpiLNAct, RM>, grid, block, st, la, lb, ep, rm, K, ncls, remap);
  } else if (e.mode == 1) {
    EpiLNBwd ep;
    static_cast<EpiLNBwdP&>(ep) = e.lb;
    const int nblk = mtiles * ncls;
    const bool sums = ep.dgamma || ep.dbeta;
    if (!(sums || ep.defer) || nblk > ep.part_rows) ep.part = nullptr;
    launch(igemm_kernel<BM, BN, WM, WN, LA, Dense<BN, 64 * WM * WN>, EpiLNBwd, RM>, grid, block, st, la, lb, ep, rm, K, ncls, remap);
    if (ep.part && !ep.defer) launch_part_reduce(ep.part, nblk, 2 * BN, ep.dgamma, ep.dbeta, BN, true, st);
  } else {
    EpiPlain ep;
    static_cast<EpiPlainP&>(ep) = e.pl;
    launch(igemm_kernel<BM, BN, WM, WN, LA, Dense<BN, 64 * WM * WN>, EpiPlain, RM>, grid, block, st, la, lb, ep, rm, K, ncls, remap);
  }
}

// Output-channel tiles: the workgroup tile spans the whole channel row (the LayerNorm epilogues need
// it), so the tile width is the layer's channel count:
//   32 / 64     256 (or 128) x C, 4 x 1 (or 2 x 2) waves         (Atari-100k E1 / D3)
//   96          128 x 96,   4 x 1 waves (TN 3)                     (XL E1)
//   128 / 192   128 x C,    2 x 2 waves (TM 2, TN 2 / 3)
//   256 / 384   64 x C,     1 x 4 waves (TM 2, TN 2 / 3)
//   512 / 768   64 x C, 1 x 8 waves (TM 2, TN 2 / 3; 512 threads keep the B-tile prefetch at 8 / 12
//               float4 per thread; LDS 83 / 120 KB)
//   1024        32 x C, 1 x 8 waves (TM 1, TN 4: no register spill; LDS 152 KB)
// 32-channel tile variants: 0 = 256 x 32 on 4 waves, 1 = 128 x 32 on 2 waves, 2 = 256 x 32 on 2 waves (TM 4), 3 = 128 x
// 32 on 4 waves (TM 1).  Default (SRL_CONV_T32 unset = -1): 3 for the forward LayerNorm+act epilogue, 0 otherwise -
// per-launch medians at the Atari-100k shapes (profiles/r6_conv_t32.md): E1 fwd 83.5 -> 80.0 us, D3 fwd 211.6 -> 193.6
// us with 3; the LayerNorm-backward epilogues (D4 dgrad 134 vs 222 us, E2 dgrad 243 vs 245 us) keep 0
static int conv_t32(int mode) {
  static const int v = [] {
    const char* e = getenv("SRL_CONV_T32");
    return e ? atoi(e) : -1;
  }();
  return v >= 0 ? v : (mode == 0 ? 3 : 0);
}
#define CONV_T32(X, ...)                                                                           \
  do {                                                                                              \
    switch (conv_t32(e.mode)) {                                                                     \
      case 1: X<128, 32, 2, 1>(__VA_ARGS__); break;                                                 \
      case 2: X<256, 32, 2, 1>(__VA_ARGS__); break;                                                 \
      case 3: X<128, 32, 4, 1>(__VA_ARGS__); break;                                                 \
      default: X<256, 32, 4, 1>(__VA_ARGS__); break;                                                \
    }                                                                                               \
  } while (0)
#define CONV_TILES(X, ...)                                                                         \
  switch (Nc) {                                                                                     \
    case 32: CONV_T32(X, __VA_ARGS__); return true;                                                 \
    case 64: X<128, 64, 2, 2>(__VA_ARGS__); return true;                                            \
    case 96: X<128, 96, 4, 1>(__VA_ARGS__); return true;                                            \
    case 128: X<128, 128, 2, 2>(__VA_ARGS__); return true;                                          \
    case 192: X<128, 192, 2, 2>(__VA_ARGS__); return true;                                          \
    case 256: X<64, 256, 1, 4>(__VA_ARGS__); return true;                                           \
    case 384: X<64, 384, 1, 4>(__VA_ARGS__); return true;                                           \
    case 512: X<64, 512, 1, 8>(__VA_ARGS__); return true;                                           \
    case 768: X<64, 768, 1, 8>(__VA_ARGS__); return true;                                           \
    case 1024: X<32, 1024, 1, 8>(__VA_ARGS__); return true;                                         \
    default: return false;                                                                          \
  }

// rows to allocate for a dgamma / dbeta partial buffer of nb workgroup rows (+ the two-pass reduction's stage rows)
int conv_part_alloc_rows(int nb) { return nb + part_stage_rows(nb); }

// rows (BM) of the workgroup tile CONV_TILES picks for Nc output channels and epilogue mode (0 if unsupported)
int conv_tile_rows(int Nc, int mode) {
  switch (Nc) {
    case 32: {
      const int v = conv_t32(mode);
      return (v == 1 || v == 3) ? 128 : 256;
    }
    case 64: case 96: case 128: case 192: return 128;
    case 256: case 384: case 512: case 768: return 64;
    case 1024: return 32;
    default: return 0;
  }
}

bool conv_channels_supported(int Nc) {
  switch (Nc) {
    case 32: case 64: case 96: case 128: case 192: case 256: case 384: case 512: case 768: case 1024: return true;
    default: return false;
  }
}

// DOWN: out grid (N, SH, SW) with Nc output channels, input Q NHWC (N, 2SH, 2SW, Cb); Cb is a
// multiple of 32 or a power of two below 32
template <int BM, int BN, int WM, int WN>
static void down_cfg(const float* Q, const float* Wp, int N, int SH, int SW, int Cb, const ConvEpi& e, hipStream_t st) {
  constexpr int NTH = 64 * WM * WN;
  const int M = N * SH * SW;
  DownGather<BM, NTH> la;
  la.Q = Q;
  la.Cb = Cb;
  la.lCb = ilog2(Cb);
  la.lSH = ilog2(SH);
  la.lSW = ilog2(SW);
  la.M = M;
  Dense<BN, NTH> lb;
  lb.W = Wp;
  lb.K = 16 * Cb;
  lb.cls_stride = 0;
  dispatch_epi<BM, BN, WM, WN>(la, lb, e, RowDown{0}, 16 * Cb, (M + BM - 1) / BM, 1, st);
}

bool launch_conv_down(const float* Q, const float* Wp, int N, int SH, int SW, int Cb, int Nc, const ConvEpi& e,
                      hipStream_t st) {
  if (!(Cb % 32 == 0 || (Cb >= 4 && Cb < 32 && (Cb & (Cb - 1)) == 0))) return false;
  CONV_TILES(down_cfg, Q, Wp, N, SH, SW, Cb, e, st)
}

template <int BM, int BN, int WM, int WN>
static void up_cfg(const float* P, const float* Wp, int N, int SH, int SW, int Ca, int Bp, const ConvEpi& e, hipStream_t st) {
  constexpr int NTH = 64 * WM * WN;
  const int M = N * SH * SW;
  UpGather<BM, NTH> la;
  la.P = P;
  la.Ca = Ca;
  la.lSH = ilog2(SH);
  la.lSW = ilog2(SW);
  la.M = M;
  Dense<BN, NTH> lb;
  lb.W = Wp;
  lb.K = 4 * Ca;
  lb.cls_stride = (size_t)Bp * 4 * Ca;
  RowUp rm{ilog2(SH), ilog2(SW), 0};
  dispatch_epi<BM, BN, WM, WN>(la, lb, e, rm, 4 * Ca, (M + BM - 1) / BM, 4, st);
}

// UP: P NHWC (N, SH, SW, Ca) -> out grid (N, 2SH, 2SW) with Bp output channels (pack padding)
bool launch_conv_up(const float* P, const float* Wp, int N, int SH, int SW, int Ca, int Bp, const ConvEpi& e,
                    hipStream_t st) {
  if (Ca % 32 != 0) return false;
  const int Nc = Bp;
  CONV_TILES(up_cfg, P, Wp, N, SH, SW, Ca, Bp, e, st)
}

template <int BM, int BN, int WM, int WN>
static void wgrad_cfg(const float* P, const float* Q, float* slab, int S, int kper, int N, int SH, int SW, int Ca, int Cbp,
                      hipStream_t st) {
  constexpr int NTH = 64 * WM * WN;
  const int M = N * SH * SW;
  WgP<BM, NTH> la;
  la.P = P;
  la.Ca = Ca;
  la.M = M;
  WgQ<BN, NTH> lb;
  lb.Q = Q;
  lb.Cb = Cbp;
  lb.lSH = ilog2(SH);
  lb.lSW = ilog2(SW);
  lb.M = M;
  dim3 grid(Ca / BM, 16 * Cbp / BN, S);
  // XCD-ordered splits (profiles/r4_wgrad_remap_{on,off}.txt: Atari layers 1.165 -> 1.126 ms)
  const int remap = (grid.x * grid.y * grid.z) % 8 == 0;
  // few 128 x 128 tiles (<= 32) with short K splits (<= 2048 pixels: the Atari-100k layers) as 3 waves per SIMD
  // (<= 168 VGPRs, no spill: 148-152 vs 155-157 us per launch); the XL layers (72-288 tiles) keep 2 (3 measured +3.4 %)
  if constexpr (BM == 128 && BN == 128 && WM * WN == 4) {
    if (kper <= 2048 && grid.x * grid.y <= 32) {
      hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 3>), grid, dim3(NTH), 0, st, la, lb, slab, 16 * Cbp, Ca, kper, remap);
      return;
    }
  }
  hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN>), grid, dim3(NTH), 0, st, la, lb, slab, 16 * Cbp, Ca, kper, remap);
}

// WGRAD tile: rows = Ca (the largest of 128 / 64 / 32 dividing it), columns = 16 * Cbp (128, or 64 for
// the 4-channel image side)
static void wgrad_tile(int Ca, int Cbp, int* BM, int* BN) {
  *BM = Ca % 128 == 0 ? 128 : (Ca % 64 == 0 ? 64 : 32);
  *BN = (16 * Cbp) % 128 == 0 ? 128 : 64;
}

// resident workgroups per CU of a WGRAD tile config (occupancy query, cached) and the CU count
static int wgrad_occ(int BM, int BN) {
  static int cache[3][2] = {{0, 0}, {0, 0}, {0, 0}};
  const int i = BM == 128 ? 0 : (BM == 64 ? 1 : 2), j = BN == 128 ? 0 : 1;
  if (cache[i][j] == 0) {
    const void* fn = nullptr;
    int nth = 256;
    if (BN == 128) {
      if (BM == 128) fn = reinterpret_cast<const void*>(wgrad_kernel<128, 128, 2, 2>);
      else if (BM == 64) fn = reinterpret_cast<const void*>(wgrad_kernel<64, 128, 1, 4>);
      else fn = reinterpret_cast<const void*>(wgrad_kernel<32, 128, 1, 4>);
    } else {
      nth = BM == 128 ? 256 : 128;
      if (BM == 128) fn = reinterpret_cast<const void*>(wgrad_kernel<128, 64, 2, 2>);
      else if (BM == 64) fn = reinterpret_cast<const void*>(wgrad_kernel<64, 64, 1, 2>);
      else fn = reinterpret_cast<const void*>(wgrad_kernel<32, 64, 1, 2>);
    }
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, nth, 0) != hipSuccess || n < 1) n = 2;
    cache[i][j] = n;
  }
  return cache[i][j];
}

static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1) v = 256;
    return v;
  }();
  return n;
}

// number of K splits (and pixels per split) for a WGRAD problem; slab = S * Ca * 16 * Cbp floats.
// Rounds-aware: with T output tiles and R resident slots (occupancy x CUs) a launch of T * S workgroups runs
// ceil(T * S / R) rounds of M / S pixels each, so its time goes as ceil(T S / R) / S: a grid just over a
// multiple of R (the XL layers: 540 / 576 workgroups on 512 slots) pays a nearly empty extra round.  S is
// picked by a small time model (rounds x tile time + partial-slab traffic), with at least 1024 pixels per split.
void conv_wgrad_plan(int N, int SH, int SW, int Ca, int Cbp, int* S, int* kper) {
  const int M = N * SH * SW;
  int BM, BN;
  wgrad_tile(Ca, Cbp, &BM, &BN);
  const int tiles = (Ca / BM) * (16 * Cbp / BN);
  // previous rule: ~512 workgroups (2 per CU); 1024 for a single-tile problem (E1 / D4: 2K outputs, 1M pixels)
  const int want = tiles == 1 ? 1024 : (512 + tiles - 1) / tiles;
  int kp = (M + want - 1) / want;
  kp = ((kp + 31) / 32) * 32;
  if (kp < 1024) kp = 1024;
  {
    const int occ = wgrad_occ(BM, BN);
    const int R = occ * num_cus();
    const int smax = std::max(1, M / 1024);
    // estimated microseconds: rounds x one workgroup's tile at 1/occ of a CU's fp32 MFMA rate (~0.61 TF/s)
    // + the partial slab written and re-read at ~5 TB/s
    const double wg_rate = 0.61e6 / occ;                    // FLOP per microsecond per resident workgroup
    const double slab_us = 2.0 * Ca * 16.0 * Cbp * 4 / 5e6;  // per split
    double best = 1e30;
    int bs = 1;
    for (int s = 1; s <= smax; ++s) {
      int k = (M + s - 1) / s;
      k = ((k + 31) / 32) * 32;
      const int se = (M + k - 1) / k;  // effective splits after rounding
      const long total = (long)tiles * se;
      const double rounds = (double)((total + R - 1) / R);
      const double cost = rounds * (2.0 * k * BM * BN / wg_rate) + se * slab_us;
      if (cost < best - 1e-9) {
        best = cost;
        bs = se;
      }
    }
    // keep the previous split unless the model predicts a clear (> 10 %) gain
    const int so = (M + kp - 1) / kp;
    const double old_cost = (double)(((long)tiles * so + R - 1) / R) * (2.0 * kp * BM * BN / wg_rate) + so * slab_us;
    if (best < 0.9 * old_cost) {
      kp = (M + bs - 1) / bs;
      kp = ((kp + 31) / 32) * 32;
    }
  }
  *kper = kp;
  *S = (M + kp - 1) / kp;
}

bool launch_conv_wgrad(const float* P, const float* Q, float* slab, float* dw, int N, int SH, int SW, int Ca, int Cbp, int Cb,
                       hipStream_t st) {
  if (Ca % 32 != 0 || (16 * Cbp) % 64 != 0) return false;
  int S, kper, BM, BN;
  conv_wgrad_plan(N, SH, SW, Ca, Cbp, &S, &kper);
  wgrad_tile(Ca, Cbp, &BM, &BN);
  if (BN == 128) {
    if (BM == 128) wgrad_cfg<128, 128, 2, 2>(P, Q, slab, S, kper, N, SH, SW, Ca, Cbp, st);
    else if (BM == 64) wgrad_cfg<64, 128, 1, 4>(P, Q, slab, S, kper, N, SH, SW, Ca, Cbp, st);
    else wgrad_cfg<32, 128, 1, 4>(P, Q, slab, S, kper, N, SH, SW, Ca, Cbp, st);
  } else {
    if (BM == 128) wgrad_cfg<128, 64, 2, 2>(P, Q, slab, S, kper, N, SH, SW, Ca, Cbp, st);
    else if (BM == 64) wgrad_cfg<64, 64, 1, 2>(P, Q, slab, S, kper, N, SH, SW, Ca, Cbp, st);
    else wgrad_cfg<32, 64, 1, 2>(P, Q, slab, S, kper, N, SH, SW, Ca, Cbp, st);
  }
  const int tot = Ca * 16 * Cbp;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((tot + 63) / 64), dim3(256), 0, st, slab, dw, S, Ca, Cbp, Cb);
  return true;
}

void launch_pack_down(const float* w, float* out, int A, int B, int Bp, hipStream_t st) {
  const int tot = A * 16 * Bp;
  hipLaunchKernelGGL(pack_down_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, w, out, A, B, Bp);
}

bool launch_multi_pack(const float* const* w, float* const* out, const int* A, const int* B, const int* Bp, const int* kind,
                       int n, hipStream_t st) {
  if (n < 1 || n > MAX_PACK_JOBS) return false;
  PackJobs jobs{};
  int mx = 0;
  for (int j = 0; j < n; ++j) {
    jobs.w[j] = w[j];
    jobs.out[j] = out[j];
    jobs.A[j] = A[j];
    jobs.B[j] = B[j];
    jobs.Bp[j] = Bp[j];
    jobs.kind[j] = kind[j];
    mx = std::max(mx, A[j] * 16 * Bp[j]);
  }
  // one thread per packed element of the largest job (the XL weights reach 4.7 M elements: a capped grid walking them
  // in a stride loop measured 140 us per launch), capped only at 16384 workgroups per job
  const int bx = std::min((mx + 255) / 256, 16384);
  hipLaunchKernelGGL(multi_pack_kernel, dim3(bx, n), dim3(256), 0, st, jobs);
  return true;
}

void launch_pack_up(const float* w, float* out, int A, int B, int Bp, hipStream_t st) {
  const int tot = 16 * Bp * A;
  hipLaunchKernelGGL(pack_up_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, w, out, A, B, Bp);
}

// Every deferred dgamma / dbeta partial of a stack's backward in two launches (instead of two per layer): pass 0 sums
// 64-row groups of every job's part into its stage rows, pass 1 sums the stage rows into the outputs.  Same fixed
// order as launch_part_reduce.
constexpr int MAX_PR_JOBS = 16;
struct PRJobs {
  const float* part[MAX_PR_JOBS];
  float* stage[MAX_PR_JOBS];
  float* out0[MAX_PR_JOBS];
  float* out1[MAX_PR_JOBS];
  int nb[MAX_PR_JOBS], W[MAX_PR_JOBS], C[MAX_PR_JOBS], g[MAX_PR_JOBS];
  int off[MAX_PR_JOBS + 1];  // first workgroup of each job in this pass
  int n, assign;
};

__global__ __launch_bounds__(1024) void part_reduce_many_kernel(PRJobs J, int pass) {
  __shared__ float red[16][64];
  int j = 0;
  while (j + 1 < J.n && (int)blockIdx.x >= J.off[j + 1]) ++j;  // workgroup-uniform
  const int local = blockIdx.x - J.off[j], W = J.W[j], cb = (W + 63) / 64;
  const int cbi = local % cb, gi = local / cb;
  const int col = cbi * 64 + (threadIdx.x & 63);
  const float v = pass == 0 ? part_block_sum(J.part[j], gi * PART_RPB, min(J.nb[j], (gi + 1) * PART_RPB), W, col, red)
                            : part_block_sum(J.stage[j], 0, J.g[j], W, col, red);
  if (threadIdx.x < 64 && col < W) {
    if (pass == 0) {
      J.stage[j][(size_t)gi * W + col] = v;
    } else {
      const int C = J.C[j];
      float* o = col < C ? J.out0[j] : J.out1[j];
      const int c = col < C ? col : col - C;
      if (o) o[c] = J.assign ? v : o[c] + v;
    }
  }
}

// stage: sum over jobs of part_stage_rows(nb) * W floats
bool launch_part_reduce_many(const float* const* parts, const int* nbs, const int* Ws, float* const* out0,
                             float* const* out1, const int* Cs, int n, float* stage, bool assign, hipStream_t st) {
  if (n < 1 || n > MAX_PR_JOBS) return false;
  PRJobs J{};
  J.n = n;
  J.assign = assign ? 1 : 0;
  size_t so = 0;
  for (int j = 0; j < n; ++j) {
    J.part[j] = parts[j];
    J.nb[j] = nbs[j];
    J.W[j] = Ws[j];
    J.C[j] = Cs[j];
    J.out0[j] = out0[j];
    J.out1[j] = out1[j];
    J.g[j] = part_stage_rows(nbs[j]);
    J.stage[j] = stage + so;
    so += (size_t)J.g[j] * Ws[j];
  }
  for (int pass = 0; pass < 2; ++pass) {
    int tot = 0;
    for (int j = 0; j < n; ++j) {
      J.off[j] = tot;
      tot += (Ws[j] + 63) / 64 * (pass == 0 ? J.g[j] : 1);
    }
    J.off[n] = tot;
    hipLaunchKernelGGL(part_reduce_many_kernel, dim3(tot), dim3(1024), 0, st, J, pass);
  }
  return true;
}

// NCHW f32 -> NHWC4 + per-channel sums over (N, H, W) into csum[C] (assigned); part: conv_part_alloc_rows(blocks) x C
void launch_to_nhwc4_sum(const float* x, float* out, int N, int C, int HW, float* csum, float* part, hipStream_t st) {
  const int nb = (N * HW + 255) / 256;
  hipLaunchKernelGGL(to_nhwc4_sum_kernel, dim3(nb), dim3(256), 0, st, x, (f4*)out, N, C, HW, part);
  launch_part_reduce(part, nb, C, csum, nullptr, C, true, st, true);
}

void launch_to_nhwc4(const void* x, bool u8, float* out, int N, int C, int HW, float scale, hipStream_t st) {
  const int tot = N * HW;
  if (u8)
    hipLaunchKernelGGL(to_nhwc4_kernel<uint8_t>, dim3((tot + 255) / 256), dim3(256), 0, st, (const uint8_t*)x, (f4*)out, N,
                       C, HW, scale);
  else
    hipLaunchKernelGGL(to_nhwc4_kernel<float>, dim3((tot + 255) / 256), dim3(256), 0, st, (const float*)x, (f4*)out, N, C,
                       HW, scale);
}

bool launch_ln_bwd_flat(const float* dy, const float* z, const float* mean, const float* rstd, const float* gamma,
                        const float* beta, float* dz, float* dgamma, float* dbeta, int M, int C, int HW, int act,
                        float* part, int part_blocks, hipStream_t st) {
  if (C % 32 != 0 || C > 1024) return false;
  const int lHW = ilog2(HW);
  // image-tiled form (coalesced dy, deterministic partials) whenever the caller gave a partial buffer and the
  // [HW][C + 1] tile fits the default 64 KB of LDS
  const int N = M / HW;
  const size_t shm = std::max((size_t)HW * (C + 1), (size_t)8 * 64 * ((C + 63) / 64)) * sizeof(float);
  if (part != nullptr && part_blocks > 0 && N * HW == M && shm <= 64 * 1024) {
    const int ipb = (N + part_blocks - 1) / part_blocks;
    const int nb = (N + ipb - 1) / ipb;
    dim3 grid(nb);
#define SRL_LNBI(K)                                                                                                    \
  do {                                                                                                                 \
    if (act == srl::ACT_SILU)                                                                                          \
      hipLaunchKernelGGL((ln_bwd_img_kernel<K, srl::ACT_SILU>), grid, dim3(256), shm, st, dy, z, mean, rstd, gamma,   \
                         beta, dz, part, N, C, lHW, act, ipb);                                                         \
    else                                                                                                               \
      hipLaunchKernelGGL((ln_bwd_img_kernel<K, -1>), grid, dim3(256), shm, st, dy, z, mean, rstd, gamma, beta, dz,     \
                         part, N, C, lHW, act, ipb);                                                                   \
  } while (0)
    switch ((C + 63) / 64) {
      case 1: SRL_LNBI(1); break;
      case 2: SRL_LNBI(2); break;
      case 3: SRL_LNBI(3); break;
      case 4: SRL_LNBI(4); break;
      case 5: case 6: SRL_LNBI(6); break;
      case 7: case 8: SRL_LNBI(8); break;
      case 9: case 10: case 11: case 12: SRL_LNBI(12); break;
      default: SRL_LNBI(16); break;
    }
#undef SRL_LNBI
    if (dgamma || dbeta) launch_part_reduce(part, nb, 2 * C, dgamma, dbeta, C, true, st);
    return true;
  }
  const int rpb = 64;
  dim3 grid((M + rpb - 1) / rpb);
#define SRL_LNBF(K)                                                                                                    \
  do {                                                                                                                 \
    if (act == srl::ACT_SILU)                                                                                          \
      hipLaunchKernelGGL((ln_bwd_flat_kernel<K, srl::ACT_SILU>), grid, dim3(256), 0, st, dy, z, mean, rstd, gamma, beta, dz, \
                         dgamma, dbeta, M, C, lHW, act, rpb);                                                          \
    else                                                                                                               \
      hipLaunchKernelGGL((ln_bwd_flat_kernel<K, -1>), grid, dim3(256), 0, st, dy, z, mean, rstd, gamma, beta, dz,       \
                         dgamma, dbeta, M, C, lHW, act, rpb);                                                          \
  } while (0)
  switch ((C + 63) / 64) {
    case 1: SRL_LNBF(1); return true;
    case 2: SRL_LNBF(2); return true;
    case 3: SRL_LNBF(3); return true;
    case 4: SRL_LNBF(4); return true;
    case 5: case 6: SRL_LNBF(6); return true;
    case 7: case 8: SRL_LNBF(8); return true;
    case 9: case 10: case 11: case 12: SRL_LNBF(12); return true;
    default: SRL_LNBF(16); return true;
  }
#undef SRL_LNBF
}

// The final ConvTranspose2d (Ca -> CO <= 4 image channels, k4 s2 p1), second form: one 256-thread block per 32 x 32
// small-grid tile, each thread owning a 2 x 2 block of small pixels = a 4 x 4 block of output pixels.  A thread
// reads its 4 x 4 input window straight from global memory (NHWC, 16-byte channel quads; neighbouring threads'
// windows overlap, so those reads hit L1), the weights come from LDS as wave-uniform broadcasts, and every weight
// read now feeds 4 small pixels x CO FMAs (the first form: 1 small pixel per thread, ~1.5 FMA per LDS read - LDS-
// bound at 134 us for 1024 frames of 32 -> 3 channels).  Output rows of 4 pixels are float4 stores.
// (MFMA does not pay here: N = CO = 3 would pad to 16 - more MFMA work than the VALU FMAs.)  Measured 122.5 us vs
// 134 us for the first form (now only used for 16-pixel-multiple grids); still 1 wave per SIMD (280 VGPRs: the
// compiler keeps a whole channel quad's 64 weight vectors live).
template <int CO>
__global__ __launch_bounds__(256) void up_small2_kernel(const float* __restrict__ P, const float* __restrict__ W,
                                                        const float* __restrict__ bias, float c0, float* __restrict__ out,
                                                        int SH, int SW, int CA) {
  static_assert(CO >= 1 && CO <= 4, "up_small2: CO <= 4");
  extern __shared__ f4 wsh[];  // [a][kh*4 + kw] -> (co 0..3)
  const int tiles_x = SW / 32;
  const int n = blockIdx.y, ty0 = (blockIdx.x / tiles_x) * 32, tx0 = (blockIdx.x % tiles_x) * 32;
  for (int i = threadIdx.x; i < CA * 16; i += 256) {
    const int a = i >> 4, tap = i & 15;
    f4 w = zero4();
#pragma unroll
    for (int c = 0; c < CO; ++c) w[c] = W[(a * CO + c) * 16 + tap];
    wsh[i] = w;
  }
  __syncthreads();
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
  const int p0 = ty0 + 2 * ty, q0 = tx0 + 2 * tx;  // first small pixel of the thread's 2 x 2 block
  // window rows / cols p0 - 1 .. p0 + 2 (q0 - 1 .. q0 + 2); out-of-grid entries read the zero vector
  const float* base = P + (((long)n * SH + p0 - 1) * SW + q0 - 1) * CA;
  int okm = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 - 1 + i, q = q0 - 1 + j;
      okm |= (p >= 0 && p < SH && q >= 0 && q < SW) ? 1 << (4 * i + j) : 0;
    }
  // acc[dy][dx][cy][cx][co]: small pixel (p0 + dy, q0 + dx), output parity (cy, cx)
  float acc[2][2][2][2][CO];
#pragma unroll
  for (int i = 0; i < 16 * CO; ++i) (&acc[0][0][0][0][0])[i] = 0.f;
  for (int a0 = 0; a0 < CA; a0 += 4) {
    f4 win[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) win[i][j] = *(const f4*)zsrc((okm >> (4 * i + j)) & 1, base + (i * SW + j) * CA + a0);
    const f4* wa = wsh + a0 * 16;
#pragma unroll
    for (int cy = 0; cy < 2; ++cy)
#pragma unroll
      for (int cx = 0; cx < 2; ++cx)
#pragma unroll
        for (int th = 0; th < 2; ++th)
#pragma unroll
          for (int tw = 0; tw < 2; ++tw) {
            const int tap = (1 - cy + 2 * th) * 4 + (1 - cx + 2 * tw);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f4 w = wa[e * 16 + tap];
#pragma unroll
              for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                  // source small pixel (p0 + dy + cy - th, q0 + dx + cx - tw) -> window (dy + cy - th + 1, ...)
                  const float v = win[dy + cy - th + 1][dx + cx - tw + 1][e];
#pragma unroll
                  for (int c = 0; c < CO; ++c) acc[dy][dx][cy][cx][c] += v * w[c];
                }
            }
          }
  }
  const int LH = 2 * SH, LW = 2 * SW;
  const int y0 = 2 * p0, x0 = 2 * q0;
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    const float b = (bias ? bias[c] : 0.f) + c0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int cy = 0; cy < 2; ++cy) {
        const f4 o = f4{acc[dy][0][cy][0][c] + b, acc[dy][0][cy][1][c] + b, acc[dy][1][cy][0][c] + b,
                        acc[dy][1][cy][1][c] + b};
        *(f4*)(out + (((size_t)n * CO + c) * LH + y0 + 2 * dy + cy) * LW + x0) = o;
      }
  }
}

// The final ConvTranspose2d (Ca -> CO <= 4 image channels, k4 s2 p1) on MFMA, input-centric: for every small-grid
// pixel (p, q) the 16 taps x CO outputs it feeds are ONE row of a dense GEMM
//     C[(p,q)][tap * CO + co] = sum_a P[p,q,a] W[a][co][tap]        (M = pixels, N = 16 CO, K = Ca)
// so N = 48 for RGB fills three 16-wide MFMA tiles exactly (the output-centric form would pad N = CO to 16),
// and no K entry is a structural zero.  A workgroup owns a 16 x 16 small-pixel tile of one image: it stages the
// 18 x 18 halo window (32 channels per pass) in LDS, runs the window's 21 x CO 16x16 tiles on
// v_mfma_f32_16x16x4_f32 (B fragments - the packed weights - held in registers for the whole pass).  The columns
// are channel-major (col = 16 co + tap), so MFMA column tile t is output channel t: each channel's C is parked in
// LDS over the dead window on its own (22 KB, not the whole 64 KB C: three workgroups fit a CU instead of two), and
// each thread sums the 4 (tap, neighbour) contributions of each of its 2 x 2 output pixels (col2im) and writes the
// NCHW image rows as float2.
template <int CO>
__global__ __launch_bounds__(256) void up_last_mfma_kernel(const float* __restrict__ P, const float* __restrict__ W,
                                                           const float* __restrict__ bias, float c0, float* __restrict__ out,
                                                           int SH, int SW, int CA) {
  static_assert(CO >= 1 && CO <= 4, "up_last_mfma: CO <= 4");
  constexpr int T = 16, TH = T + 2, NPIX = TH * TH;  // 324 window pixels
  constexpr int MT = (NPIX + 15) / 16;               // 21 M tiles
  constexpr int MPW = (MT + 3) / 4;                  // M tiles per wave
  constexpr int LDA = 36, LDC = 17;                  // C of ONE output channel: [pixel][16 taps] (+1 pad)
  constexpr int LDS_A = MT * 16 * LDA, LDS_C = MT * 16 * LDC;
  __shared__ float sm[LDS_A > LDS_C ? LDS_A : LDS_C];
  const int tiles_x = SW / T;
  const int n = blockIdx.y, ty0 = (blockIdx.x / tiles_x) * T, tx0 = (blockIdx.x % tiles_x) * T;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  f4 acc[MPW][CO];
#pragma unroll
  for (int m = 0; m < MPW; ++m)
#pragma unroll
    for (int t = 0; t < CO; ++t) acc[m][t] = zero4();
  for (int a0 = 0; a0 < CA; a0 += 32) {
    __syncthreads();  // the previous pass's A reads are done
    for (int e = threadIdx.x; e < MT * 16 * 8; e += 256) {
      const int r = e >> 3, q4 = (e & 7) * 4;
      f4 v = zero4();
      if (r < NPIX) {
        const int p = ty0 - 1 + r / TH, q = tx0 - 1 + r % TH;
        if (p >= 0 && p < SH && q >= 0 && q < SW) v = *(const f4*)(P + (((size_t)n * SH + p) * SW + q) * CA + a0 + q4);
      }
      *(f4*)(sm + r * LDA + q4) = v;
    }
    // B fragments: lane (i, g) of MFMA j in K chunk c holds B[k = a0 + 16c + 4g + j][col = 16t + i]: channel t, tap i
    float b[2][CO][4];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int t = 0; t < CO; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) b[c][t][j] = W[((size_t)(a0 + 16 * c + 4 * g + j) * CO + t) * 16 + i];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MPW; ++m) {
      const int mt = w + 4 * m;
      if (mt < MT) {  // wave-uniform
        const float* arow = sm + (mt * 16 + i) * LDA + 4 * g;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const f4 a = *(const f4*)(arow + 16 * c);
#pragma unroll
          for (int t = 0; t < CO; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[c][t][j], acc[m][t], 0, 0, 0);
        }
      }
    }
  }
  // col2im per output channel: thread = small pixel (u, v); output (2u + cy, 2v + cx) sums taps (1 - cy + 2th,
  // 1 - cx + 2tw) of the small pixels (u + cy - th, v + cx - tw), th, tw in {0, 1}
  const int u = threadIdx.x >> 4, v = threadIdx.x & 15;
  const int LH = 2 * SH, LW = 2 * SW;
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    __syncthreads();  // every wave's A reads (co = 0) / the previous channel's col2im reads are done
#pragma unroll
    for (int m = 0; m < MPW; ++m) {
      const int mt = w + 4 * m;
      if (mt < MT) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sm[(mt * 16 + 4 * g + e) * LDC + i] = acc[m][co][e];
      }
    }
    __syncthreads();
    const float bb = (bias ? bias[co] : 0.f) + c0;
#pragma unroll
    for (int cy = 0; cy < 2; ++cy) {
      float o[2];
#pragma unroll
      for (int cx = 0; cx < 2; ++cx) {
        float s = bb;
#pragma unroll
        for (int th = 0; th < 2; ++th)
#pragma unroll
          for (int tw = 0; tw < 2; ++tw) {
            const int r = (u + cy - th + 1) * TH + (v + cx - tw + 1);
            const int tap = (1 - cy + 2 * th) * 4 + (1 - cx + 2 * tw);
            s += sm[r * LDC + tap];
          }
        o[cx] = s;
      }
      *(float2*)(out + (((size_t)n * CO + co) * LH + 2 * (ty0 + u) + cy) * LW + 2 * (tx0 + v)) = make_float2(o[0], o[1]);
    }
  }
}

// final-layer form: 0 = MFMA (default: 96.6 vs 120.2 us at the Atari-100k shape, profiles/r4_up_last.json),
// 1 = the VALU kernels below (tests only: set_up_last_form)
static int g_up_last_form = 0;
void set_up_last_form(int f) { g_up_last_form = f; }

bool launch_up_small(const float* P, const float* W, const float* bias, float c0, float* out, int N, int SH, int SW, int Ca,
                     int CO, hipStream_t st) {
  if (SH % 16 || SW % 16 || CO < 1 || CO > 4 || Ca % 32 != 0) return false;
  if (g_up_last_form == 0) {
    dim3 g1((SH / 16) * (SW / 16), N);
    switch (CO) {
      case 1: hipLaunchKernelGGL((up_last_mfma_kernel<1>), g1, dim3(256), 0, st, P, W, bias, c0, out, SH, SW, Ca); break;
      case 2: hipLaunchKernelGGL((up_last_mfma_kernel<2>), g1, dim3(256), 0, st, P, W, bias, c0, out, SH, SW, Ca); break;
      case 3: hipLaunchKernelGGL((up_last_mfma_kernel<3>), g1, dim3(256), 0, st, P, W, bias, c0, out, SH, SW, Ca); break;
      default: hipLaunchKernelGGL((up_last_mfma_kernel<4>), g1, dim3(256), 0, st, P, W, bias, c0, out, SH, SW, Ca); break;
    }
    return true;
  }
  if (SH % 32 == 0 && SW % 32 == 0 && Ca <= 512) {  // 122.5 vs 134 us at 1024 x 32x32x32 -> 3 channels
    dim3 g2((SH / 32) * (SW / 32), N);
    const size_t lds = (size_t)Ca * 16 * sizeof(f4);
    switch (CO) {
      case 1: hipLaunchKernelGGL((up_small2_kernel<1>), g2, dim3(256), lds, st, P, W, bias, c0, out, SH, SW, Ca); break;
      case 2: hipLaunchKernelGGL((up_small2_kernel<2>), g2, dim3(256), lds, st, P, W, bias, c0, out, SH, SW, Ca); break;
      case 3: hipLaunchKernelGGL((up_small2_kernel<3>), g2, dim3(256), lds, st, P, W, bias, c0, out, SH, SW, Ca); break;
      default: hipLaunchKernelGGL((up_small2_kernel<4>), g2, dim3(256), lds, st, P, W, bias, c0, out, SH, SW, Ca); break;
    }
    return true;
  }
  dim3 grid((SH / 16) * (SW / 16), N);
  const int lSH = ilog2(SH), lSW = ilog2(SW);
  switch (CO) {
    case 1: hipLaunchKernelGGL((up_small_kernel<1>), grid, dim3(256), 0, st, P, W, bias, c0, out, lSH, lSW, Ca); break;
    case 2: hipLaunchKernelGGL((up_small_kernel<2>), grid, dim3(256), 0, st, P, W, bias, c0, out, lSH, lSW, Ca); break;
    case 3: hipLaunchKernelGGL((up_small_kernel<3>), grid, dim3(256), 0, st, P, W, bias, c0, out, lSH, lSW, Ca); break;
    default: hipLaunchKernelGGL((up_small_kernel<4>), grid, dim3(256), 0, st, P, W, bias, c0, out, lSH, lSW, Ca); break;
  }
  return true;
}
