// Weight gradients of tall linear layers: dW[N, K] = dZ[M, N]^T X[M, K] and db[N] = sum_m dZ[m, :] for M >> N, K
// (the DreamerV3 behaviour heads back-propagate over M = (H+1)*B*T = 16384 imagined rows with N, K <= 1536).
//
// Library GEMMs tile the [N, K] output and run the whole M reduction inside each tile: at N = K = 512 that is
// 16-64 workgroups for a 256-CU chip (measured 105-245 us per layer, 31-106 TF/s).  Here:
//
//  * dense part (split-K over M): grid = (128 x 128 output tiles) x S row chunks, XCD-aware (the chunks of one
//    XCD's workgroups are contiguous, so the dZ / X rows a chunk reads are shared through that XCD's L2).  Four
//    waves per tile, 2 x 2 of v_mfma_f32_32x32x2f32 per wave.  Both operands come straight from global memory
//    in MFMA layout (A[i=n][k=m] = dZ[m][n]: lanes 0-31 read 32 consecutive columns of row m, lanes 32-63 of row
//    m+1 - 128-byte coalesced rows; B likewise from X), double-buffered in registers 16 rows ahead.  The bias
//    column sum rides on the A loads of the tile-column-0 waves.
//  * one-hot part: the first-layer inputs of the heads are [z | h] with z the exact one-hot sample of G
//    categoricals; their dW columns are sums of dZ rows (dW[:, t] = sum_{m : t hot in row m} dZ[m, :]).  As a
//    dense GEMM that is 2/3 of the layer's weight-gradient FLOPs (K 1536 of which 1024 one-hot); here each wave
//    owns one group and 128 output rows and adds every dZ row into the LDS table row of its hot class.
//  * both write per-chunk partials [S, N, Kpart]; a reduce kernel sums them in chunk order into the output
//    (deterministic: fixed chunk split, fixed in-chunk order).
#include <stdlib.h>

#include "common.h"

namespace srl {
namespace wgrad {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BT = 128;  // output tile (n and k)
constexpr int U = 8;     // MFMA steps (2 rows each) per register batch

struct DP {
  const float* dz;
  const float* x;
  float* part;   // [S, N, K]
  float* bpart;  // [S, N] or null
  long ldz, ldx;
  int M, N, K, S, rows;  // rows per chunk (multiple of 2*U except the last)
  int tn, tk;            // tiles along N, K
};

// Full batches: unconditional loads, no selects (lanes past N / K read a clamped column; their accumulator rows
// / columns are never stored), so the wait-count pass can leave the next batch's prefetch in flight across
// this batch's MFMAs.  (A first version zeroed every value with a select right after its load - the selects
// pulled vmcnt(0) waits for the prefetch in front of the current batch's MFMAs: 55 TF/s at 16384 x 512 x 512.)
__device__ __forceinline__ void load_full(const float* __restrict__ dz, const float* __restrict__ x, long ldz, long ldx,
                                          int m, int oa, int ob, float (&a0)[U], float (&a1)[U], float (&b0)[U],
                                          float (&b1)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float* zr = dz + (long)(m + 2 * u) * ldz;
    const float* xr = x + (long)(m + 2 * u) * ldx;
    a0[u] = zr[0];
    a1[u] = zr[oa];
    b0[u] = xr[0];
    b1[u] = xr[ob];
  }
}

// the chunk's last partial batch: rows past the chunk read as 0
__device__ __forceinline__ void load_tail(const float* __restrict__ dz, const float* __restrict__ x, long ldz, long ldx,
                                          int m, int m1, int oa, int ob, float (&a0)[U], float (&a1)[U], float (&b0)[U],
                                          float (&b1)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = m + 2 * u;
    const bool ok = r < m1;
    const int rc = ok ? r : m1 - 1;
    const float* zr = dz + (long)rc * ldz;
    const float* xr = x + (long)rc * ldx;
    const float za = zr[0], zb = zr[oa], xa = xr[0], xb = xr[ob];
    a0[u] = ok ? za : 0.f;
    a1[u] = ok ? zb : 0.f;
    b0[u] = ok ? xa : 0.f;
    b1[u] = ok ? xb : 0.f;
  }
}

#define WG_MFMA_BATCH(A0, A1, B0, B1)                                                 \
  _Pragma("unroll") for (int u = 0; u < U; ++u) {                                     \
    acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[u], B0[u], acc00, 0, 0, 0);       \
    acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[u], B1[u], acc01, 0, 0, 0);       \
    acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[u], B0[u], acc10, 0, 0, 0);       \
    acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[u], B1[u], acc11, 0, 0, 0);       \
    if (BIAS) {                                                                       \
      bs0 += A0[u];                                                                   \
      bs1 += A1[u];                                                                   \
    }                                                                                 \
  }

template <bool BIAS>
__global__ void __launch_bounds__(256, 2) dense_kernel(DP p) {
  const int nblk = gridDim.x;
  int bid = blockIdx.x;
  // hardware dispatch puts block b on XCD b % 8: renumber so that each XCD works on a contiguous range of
  // (chunk, tile) pairs - the tiles of one chunk share its dZ / X rows in that XCD's L2
  if ((nblk & 7) == 0) bid = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int tiles = p.tn * p.tk;
  const int s = bid / tiles, t = bid - s * tiles;
  const int tni = t / p.tk, tki = t - tni * p.tk;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wn = wave >> 1, wk = wave & 1;
  const int col = lane & 31, half = lane >> 5;
  const int n0 = tni * BT + wn * 64, k0 = tki * BT + wk * 64;
  const int m0 = s * p.rows;
  const int m1 = min(p.M, m0 + p.rows);
  const bool va0 = n0 + col < p.N, va1 = n0 + 32 + col < p.N;
  const bool vb0 = k0 + col < p.K, vb1 = k0 + 32 + col < p.K;
  // lanes past N / K read a clamped column of their row (valid memory; results never stored)
  const float* dz = p.dz + (va0 ? n0 + col : 0) + (long)half * p.ldz;
  const float* x = p.x + (vb0 ? k0 + col : 0) + (long)half * p.ldx;
  const int oa = va1 ? 32 : 0, ob = vb1 ? 32 : 0;
  const int mfull = m0 + ((m1 - m0) / (2 * U)) * (2 * U);  // end of the chunk's full 16-row batches

  floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
  float bs0 = 0.f, bs1 = 0.f;
  float a0[U], a1[U], b0[U], b1[U];
  float c0[U], c1[U], d0[U], d1[U];
  if (m0 < mfull) {
    int m = m0;
    load_full(dz, x, p.ldz, p.ldx, m, oa, ob, a0, a1, b0, b1);
    while (true) {
      // batch a (rows m..m+15) is in flight; prefetch batch c, consume a
      if (m + 2 * U >= mfull) {
        WG_MFMA_BATCH(a0, a1, b0, b1);
        break;
      }
      load_full(dz, x, p.ldz, p.ldx, m + 2 * U, oa, ob, c0, c1, d0, d1);
      WG_MFMA_BATCH(a0, a1, b0, b1);
      m += 2 * U;
      if (m + 2 * U >= mfull) {
        WG_MFMA_BATCH(c0, c1, d0, d1);
        break;
      }
      load_full(dz, x, p.ldz, p.ldx, m + 2 * U, oa, ob, a0, a1, b0, b1);
      WG_MFMA_BATCH(c0, c1, d0, d1);
      m += 2 * U;
    }
  }
  if (mfull < m1) {
    load_tail(dz, x, p.ldz, p.ldx, mfull, m1 - half, oa, ob, a0, a1, b0, b1);
    WG_MFMA_BATCH(a0, a1, b0, b1);
  }
  // C/D layout of the 32x32 tiles: col = lane & 31 (k), row = (r & 3) + 8 * (r >> 2) + 4 * half (n)
  float* out = p.part + (long)s * p.N * p.K;
  const int kc0 = k0 + col, kc1 = k0 + 32 + col;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * half;
    const int na = n0 + i, nb = n0 + 32 + i;
    if (na < p.N) {
      if (vb0) out[(long)na * p.K + kc0] = acc00[r];
      if (vb1) out[(long)na * p.K + kc1] = acc01[r];
    }
    if (nb < p.N) {
      if (vb0) out[(long)nb * p.K + kc0] = acc10[r];
      if (vb1) out[(long)nb * p.K + kc1] = acc11[r];
    }
  }
  if (BIAS && tki == 0 && wk == 0) {
    bs0 += __shfl_xor(bs0, 32, 64);
    bs1 += __shfl_xor(bs1, 32, 64);
    if (half == 0) {
      if (va0) p.bpart[(long)s * p.N + n0 + col] = bs0;
      if (va1) p.bpart[(long)s * p.N + n0 + 32 + col] = bs1;
    }
  }
}

// LDS-staged form for 16-byte aligned rows (N, K, ldz, ldx % 4 == 0): the dword loads of dense_kernel are
// address-bound in the texture unit (64 addresses per 256 bytes); here a 16-row batch of each operand is fetched
// with dwordx4 loads (2 per thread per operand), stored row-major into LDS (conflict-free b128 writes) and read
// back in MFMA layout (32 consecutive columns per half-wave: conflict-free b32 reads).  Double-buffered LDS,
// global loads of batch b+1 in flight across batch b's MFMAs, one barrier per batch.
constexpr int LBM = 32;             // rows per batch (the next batch's loads cover ~3 us of MFMAs)
constexpr int LROW = BT + 4;        // LDS row stride (floats)

// A4 = false: dZ rows not 16-byte aligned (the two-hot heads' 255-wide gradients): its batch is staged with dword
// loads (4 per float4 slot, columns clamped to N - 1: those accumulator rows are never stored).
template <bool A4>
__global__ void __launch_bounds__(256, 2) dense_lds_kernel(DP p, int bias) {
  __shared__ float As[2][LBM][LROW];
  __shared__ float Bs[2][LBM][LROW];
  const int nblk = gridDim.x;
  int bid = blockIdx.x;
  if ((nblk & 7) == 0) bid = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int tiles = p.tn * p.tk;
  const int s = bid / tiles, t = bid - s * tiles;
  const int tni = t / p.tk, tki = t - tni * p.tk;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wn = wave >> 1, wk = wave & 1;
  const int col = lane & 31, half = lane >> 5;
  const int nb0 = tni * BT, kb0 = tki * BT;
  const int m0 = s * p.rows;
  const int m1 = min(p.M, m0 + p.rows);
  // global -> register mapping: thread tid loads columns 4 * (tid % 32) of rows tid / 32 + 8 j
  const int lr = tid >> 5, lc = (tid & 31) * 4;
  const bool an = nb0 + lc < p.N, bk = kb0 + lc < p.K;
  const float* za = p.dz + (an ? nb0 + lc : 0);
  const float* xa = p.x + (bk ? kb0 + lc : 0);
  const int c1 = A4 ? 1 : (nb0 + lc + 1 < p.N ? 1 : 0), c2 = A4 ? 2 : (nb0 + lc + 2 < p.N ? 2 : 0),
            c3 = A4 ? 3 : (nb0 + lc + 3 < p.N ? 3 : 0);
  auto aload = [&](int r) -> float4 {
    const float* zr = za + (long)r * p.ldz;
    if (A4) return *reinterpret_cast<const float4*>(zr);
    return make_float4(zr[0], zr[c1], zr[c2], zr[c3]);
  };
  static_assert(LBM == 32, "4 rows per thread per operand below");
  // (named registers, not arrays captured by a lambda: those were demoted to scratch)
  float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
  const long sx = 8 * p.ldx;
#define WG_GLOAD(m)                                                                            \
  do {                                                                                         \
    const int r_ = (m) + lr;                                                                   \
    ra0 = aload(r_);                                                                           \
    ra1 = aload(r_ + 8);                                                                       \
    ra2 = aload(r_ + 16);                                                                      \
    ra3 = aload(r_ + 24);                                                                      \
    const float* xr_ = xa + (long)r_ * p.ldx;                                                  \
    rb0 = *reinterpret_cast<const float4*>(xr_);                                               \
    rb1 = *reinterpret_cast<const float4*>(xr_ + sx);                                          \
    rb2 = *reinterpret_cast<const float4*>(xr_ + 2 * sx);                                      \
    rb3 = *reinterpret_cast<const float4*>(xr_ + 3 * sx);                                      \
  } while (0)
#define WG_SSTORE(b)                                                                           \
  do {                                                                                         \
    *reinterpret_cast<float4*>(&As[b][lr][lc]) = ra0;                                          \
    *reinterpret_cast<float4*>(&As[b][lr + 8][lc]) = ra1;                                      \
    *reinterpret_cast<float4*>(&As[b][lr + 16][lc]) = ra2;                                     \
    *reinterpret_cast<float4*>(&As[b][lr + 24][lc]) = ra3;                                     \
    *reinterpret_cast<float4*>(&Bs[b][lr][lc]) = rb0;                                          \
    *reinterpret_cast<float4*>(&Bs[b][lr + 8][lc]) = rb1;                                      \
    *reinterpret_cast<float4*>(&Bs[b][lr + 16][lc]) = rb2;                                     \
    *reinterpret_cast<float4*>(&Bs[b][lr + 24][lc]) = rb3;                                     \
  } while (0)
  floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
  float bs0 = 0.f, bs1 = 0.f;
  const bool do_bias = bias && tki == 0 && wk == 0;
  const int an0 = wn * 64 + col, bk0 = wk * 64 + col;
  auto compute = [&](int b) {
    float a0[LBM / 2], a1[LBM / 2], b0[LBM / 2], b1[LBM / 2];
#pragma unroll
    for (int u = 0; u < LBM / 2; ++u) {
      const int r = 2 * u + half;
      a0[u] = As[b][r][an0];
      a1[u] = As[b][r][an0 + 32];
      b0[u] = Bs[b][r][bk0];
      b1[u] = Bs[b][r][bk0 + 32];
    }
#pragma unroll
    for (int u = 0; u < LBM / 2; ++u) {
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], b0[u], acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[u], b1[u], acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], b0[u], acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[u], b1[u], acc11, 0, 0, 0);
      if (do_bias) {
        bs0 += a0[u];
        bs1 += a1[u];
      }
    }
  };
  const int mf = m0 + (max(m1 - m0, 0) / LBM) * LBM;
  int b = 0;
  if (m0 < mf) WG_GLOAD(m0);
  for (int m = m0; m < mf; m += LBM) {
    WG_SSTORE(b);
    if (m + LBM < mf) WG_GLOAD(m + LBM);
    __syncthreads();
    compute(b);
    b ^= 1;
  }
  if (mf < m1) {  // the chunk's last partial batch: rows past it contribute 0
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const int r_ = mf + lr;
    ra0 = r_ < m1 ? aload(r_) : z4;
    ra1 = r_ + 8 < m1 ? aload(r_ + 8) : z4;
    ra2 = r_ + 16 < m1 ? aload(r_ + 16) : z4;
    ra3 = r_ + 24 < m1 ? aload(r_ + 24) : z4;
    rb0 = r_ < m1 ? *reinterpret_cast<const float4*>(xa + (long)r_ * p.ldx) : z4;
    rb1 = r_ + 8 < m1 ? *reinterpret_cast<const float4*>(xa + (long)(r_ + 8) * p.ldx) : z4;
    rb2 = r_ + 16 < m1 ? *reinterpret_cast<const float4*>(xa + (long)(r_ + 16) * p.ldx) : z4;
    rb3 = r_ + 24 < m1 ? *reinterpret_cast<const float4*>(xa + (long)(r_ + 24) * p.ldx) : z4;
    WG_SSTORE(b);
    __syncthreads();
    compute(b);
  }
#undef WG_GLOAD
#undef WG_SSTORE
  const int n0 = nb0 + wn * 64, k0 = kb0 + wk * 64;
  float* out = p.part + (long)s * p.N * p.K;
  const int kc0 = k0 + col, kc1 = k0 + 32 + col;
  const bool vb0 = kc0 < p.K, vb1 = kc1 < p.K;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * half;
    const int na = n0 + i, nb = n0 + 32 + i;
    if (na < p.N) {
      if (vb0) out[(long)na * p.K + kc0] = acc00[r];
      if (vb1) out[(long)na * p.K + kc1] = acc01[r];
    }
    if (nb < p.N) {
      if (vb0) out[(long)nb * p.K + kc0] = acc10[r];
      if (vb1) out[(long)nb * p.K + kc1] = acc11[r];
    }
  }
  if (do_bias) {
    bs0 += __shfl_xor(bs0, 32, 64);
    bs1 += __shfl_xor(bs1, 32, 64);
    if (half == 0) {
      if (n0 + col < p.N) p.bpart[(long)s * p.N + n0 + col] = bs0;
      if (n0 + 32 + col < p.N) p.bpart[(long)s * p.N + n0 + 32 + col] = bs1;
    }
  }
}

// ------------------------------------------------------------------ one-hot columns
// One wave per (group g, 128 output rows n, row chunk); 8 waves (8 groups) per workgroup share the dZ rows through
// L1.  Each wave owns a private LDS table acc[c][n] (C <= 32 classes x 128 n, row stride 130 floats) and adds each
// dZ row slice (float2 per lane) into the row of its hot class with plain LDS read-modify-writes - no atomics:
// only this wave touches its table, lanes own distinct words, and LDS ops of a wave complete in order.  A batch of
// OH_RB rows is processed together: rows whose (wave-uniform) class repeats later in the batch are folded into the
// later row first (scalar compares, uniform branches: nearly free without repeats), so the batch's reads of
// distinct classes can all be in flight before its writes.  dZ rows and hot indices are prefetched one batch
// ahead.  (LDS float atomics - ds_add_f32 - ran this at 1.35 ms for 16384 x 512 x 32 groups; relative VGPR
// indexing into per-lane class registers at 250 us.)
constexpr int OH_RB = 8;
constexpr int OH_CMAX = 32;
constexpr int OH_WAVES = 8;
constexpr int OH_COLS = 128;
constexpr int OH_LDS = OH_COLS + 2;  // row stride: the transposed write-out reads down columns conflict-free

struct OP {
  const float* dz;
  const int* idx;
  float* part;  // [S, N, KO]
  long ldz, ldi;
  int M, N, G, C, off, S, rows;
  int KO;  // = G * C
};

// write-out of a wave's table, transposed: part[s][nb + j][g*C + c], c fastest (float4 over 4 classes when C % 4 == 0)
__device__ __forceinline__ void oh_writeout(const float* T, const OP& p, int s, int g, int nb, int lane) {
  float* out = p.part + (long)s * p.N * p.KO + (long)g * p.C;
  if ((p.C & 3) == 0 && (p.KO & 3) == 0) {
    const int q4 = p.C >> 2;
    for (int i = lane; i < OH_COLS * q4; i += 64) {
      const int j = i / q4, c4 = (i - j * q4) * 4;
      if (nb + j < p.N) {
        const float4 o = make_float4(T[(c4 + 0) * OH_LDS + j], T[(c4 + 1) * OH_LDS + j], T[(c4 + 2) * OH_LDS + j],
                                     T[(c4 + 3) * OH_LDS + j]);
        *reinterpret_cast<float4*>(out + (long)(nb + j) * p.KO + c4) = o;
      }
    }
  } else {
    for (int i = lane; i < OH_COLS * p.C; i += 64) {
      const int j = i / p.C, c = i - j * p.C;
      if (nb + j < p.N) out[(long)(nb + j) * p.KO + c] = T[c * OH_LDS + j];
    }
  }
}

__global__ void __launch_bounds__(OH_WAVES * 64) onehot_kernel(OP p) {
  __shared__ float tab[OH_WAVES][OH_CMAX + 1][OH_LDS];  // + the junk row
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.y * OH_WAVES + wave;
  const int s = blockIdx.z;
  const int nb = blockIdx.x * OH_COLS;
  const int n = nb + 2 * lane;
  float* T = &tab[wave][0][0];
  for (int i = lane; i < (OH_CMAX + 1) * OH_LDS; i += 64) T[i] = 0.f;
  if (g >= p.G) return;  // whole wave (no block-level barrier below)
  const int m0 = s * p.rows, m1 = min(p.M, m0 + p.rows);
  const int mf = m0 + (max(m1 - m0, 0) / OH_RB) * OH_RB;
  const float2* dz = reinterpret_cast<const float2*>(p.dz + (n < p.N ? n : 0));
  const long ldz2 = p.ldz >> 1;
  const int* ip = p.idx + g;
  const int base = g * p.C + p.off;
  float2* T2 = reinterpret_cast<float2*>(T) + lane;  // this lane's column pair
  constexpr int LD2 = OH_LDS / 2;
  float2 v[OH_RB], w[OH_RB];
  int t = 0, u = 0;
  auto load = [&](int r, float2 (&vv)[OH_RB], int& tt) {
#pragma unroll
    for (int q = 0; q < OH_RB; ++q) vv[q] = dz[(long)(r + q) * ldz2];
    tt = ip[(long)(r + (lane & (OH_RB - 1))) * p.ldi];
  };
  // Two sub-batches of 4 rows.  Within one, row q's contribution is the sum of the rows p <= q of the same class
  // (selects on scalar class compares); only the LAST row of each class reads + writes the table, the others
  // read + write the junk row OH_CMAX - all branch-free, so the next batch's prefetch stays in flight.
  auto batch = [&](float2 (&vv)[OH_RB], int tt) {
#pragma unroll
    for (int h = 0; h < OH_RB; h += 4) {
      const int c0 = (__builtin_amdgcn_readlane(tt, h + 0) - base) & (OH_CMAX - 1);
      const int c1 = (__builtin_amdgcn_readlane(tt, h + 1) - base) & (OH_CMAX - 1);
      const int c2 = (__builtin_amdgcn_readlane(tt, h + 2) - base) & (OH_CMAX - 1);
      const int c3 = (__builtin_amdgcn_readlane(tt, h + 3) - base) & (OH_CMAX - 1);
      const bool e01 = c0 == c1, e02 = c0 == c2, e03 = c0 == c3, e12 = c1 == c2, e13 = c1 == c3, e23 = c2 == c3;
      const float2 v0 = vv[h], v1 = vv[h + 1], v2 = vv[h + 2], v3 = vv[h + 3];
      const float2 s1 = make_float2(v1.x + (e01 ? v0.x : 0.f), v1.y + (e01 ? v0.y : 0.f));
      const float2 s2 = make_float2(v2.x + (e02 ? v0.x : 0.f) + (e12 ? v1.x : 0.f), v2.y + (e02 ? v0.y : 0.f) + (e12 ? v1.y : 0.f));
      const float2 s3 = make_float2(v3.x + (e03 ? v0.x : 0.f) + (e13 ? v1.x : 0.f) + (e23 ? v2.x : 0.f),
                                    v3.y + (e03 ? v0.y : 0.f) + (e13 ? v1.y : 0.f) + (e23 ? v2.y : 0.f));
      const int a0 = (e01 || e02 || e03) ? OH_CMAX : c0;
      const int a1 = (e12 || e13) ? OH_CMAX : c1;
      const int a2 = e23 ? OH_CMAX : c2;
      const float2 o0 = T2[a0 * LD2], o1 = T2[a1 * LD2], o2 = T2[a2 * LD2], o3 = T2[c3 * LD2];
      T2[a0 * LD2] = make_float2(o0.x + v0.x, o0.y + v0.y);
      T2[a1 * LD2] = make_float2(o1.x + s1.x, o1.y + s1.y);
      T2[a2 * LD2] = make_float2(o2.x + s2.x, o2.y + s2.y);
      T2[c3 * LD2] = make_float2(o3.x + s3.x, o3.y + s3.y);
    }
  };
  if (m0 < mf) {
    int r = m0;
    load(r, v, t);
    while (true) {
      if (r + OH_RB >= mf) {
        batch(v, t);
        break;
      }
      load(r + OH_RB, w, u);
      batch(v, t);
      r += OH_RB;
      if (r + OH_RB >= mf) {
        batch(w, u);
        break;
      }
      load(r + OH_RB, v, t);
      batch(w, u);
      r += OH_RB;
    }
  }
  for (int r = mf; r < m1; ++r) {
    const float2 x = dz[(long)r * ldz2];
    const int c = (__builtin_amdgcn_readfirstlane(ip[(long)r * p.ldi]) - base) & (OH_CMAX - 1);
    const float2 o = T2[c * LD2];
    T2[c * LD2] = make_float2(o.x + x.x, o.y + x.y);
  }
  oh_writeout(T, p, s, g, nb, lane);
}

// Same scatter with the dZ rows and hot classes staged ONCE per workgroup in LDS (the version above has each of
// the 8 waves load the same 512-byte row slices itself: 8x the TA / L1 work, and only one 8-row batch - 4 KB
// per CU - in flight, so at 16384 x 512 x 32 groups it sat at ~103 us, latency-bound on the dZ stream).  Units of
// OS_RU = 16 rows: every thread loads one float4 of dZ (row tid / 32, 4 columns), threads 0-127 one hot index
// (row tid / 8, group tid % 8) mapped to its class (OH_CMAX = junk row for rows past the chunk), all loads
// issued two units ahead (32 KB in flight per CU) into named registers, then parked in a double-buffered LDS
// stage; one barrier per unit.  The per-wave table update is the batch fold above on 4 rows at a time.
constexpr int OS_RU = 16;

__global__ void __launch_bounds__(OH_WAVES * 64) onehot_stg_kernel(OP p) {
  __shared__ float tab[OH_WAVES][OH_CMAX + 1][OH_LDS];
  __shared__ float4 stg[2][OS_RU][OH_COLS / 4];
  __shared__ int4 cls[2][OH_WAVES][OS_RU / 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.y * OH_WAVES + wave;  // >= G: the wave computes junk and writes nothing
  const int s = blockIdx.z;
  const int nb = blockIdx.x * OH_COLS;
  float* T = &tab[wave][0][0];
  for (int i = lane; i < (OH_CMAX + 1) * OH_LDS; i += 64) T[i] = 0.f;
  const int m0 = s * p.rows, m1 = min(p.M, m0 + p.rows);
  const int nu = (max(m1 - m0, 0) + OS_RU - 1) / OS_RU;
  // staging roles (all loads unconditional, from clamped addresses)
  const int lq = tid >> 5, lc4 = tid & 31;
  const int iq = (tid >> 3) & (OS_RU - 1), iw = tid & 7;
  const bool has_i = tid < OS_RU * OH_WAVES;
  const int ig = min(blockIdx.y * OH_WAVES + iw, p.G - 1);
  const float* dzp = p.dz + min(nb + 4 * lc4, p.N - 4);
  const int* ipp = p.idx + ig;
  const int ibase = ig * p.C + p.off;
  int* clsw = reinterpret_cast<int*>(&cls[0][0][0]) + iw * OS_RU + iq;
  const float2* S2 = reinterpret_cast<const float2*>(&stg[0][0][0]) + lane;
  float2* T2 = reinterpret_cast<float2*>(T) + lane;
  constexpr int LD2 = OH_LDS / 2;
#define OS_LOAD(u, rv, ri)                                                             \
  do {                                                                                 \
    rv = *reinterpret_cast<const float4*>(dzp + (long)min(m0 + (u) * OS_RU + lq, m1 - 1) * p.ldz); \
    ri = ipp[(long)min(m0 + (u) * OS_RU + iq, m1 - 1) * p.ldi];                        \
  } while (0)
#define OS_STORE(u, b, rv, ri)                                                                          \
  do {                                                                                                  \
    stg[b][lq][lc4] = rv;                                                                               \
    if (has_i) clsw[(b) * OH_WAVES * OS_RU] = m0 + (u) * OS_RU + iq < m1 ? ((ri - ibase) & (OH_CMAX - 1)) : OH_CMAX; \
  } while (0)
  // 4 rows (q0..q0+3 of stage b) into the table: repeats folded into the last row of their class (see above)
  auto quad = [&](int b, int q0, int4 cc) {
    const int c0 = __builtin_amdgcn_readfirstlane(cc.x), c1 = __builtin_amdgcn_readfirstlane(cc.y);
    const int c2 = __builtin_amdgcn_readfirstlane(cc.z), c3 = __builtin_amdgcn_readfirstlane(cc.w);
    const float2* sv = S2 + (b * OS_RU + q0) * (OH_COLS / 2);
    const float2 v0 = sv[0], v1 = sv[OH_COLS / 2], v2 = sv[OH_COLS], v3 = sv[3 * OH_COLS / 2];
    const bool e01 = c0 == c1, e02 = c0 == c2, e03 = c0 == c3, e12 = c1 == c2, e13 = c1 == c3, e23 = c2 == c3;
    const float2 s1 = make_float2(v1.x + (e01 ? v0.x : 0.f), v1.y + (e01 ? v0.y : 0.f));
    const float2 s2 = make_float2(v2.x + (e02 ? v0.x : 0.f) + (e12 ? v1.x : 0.f), v2.y + (e02 ? v0.y : 0.f) + (e12 ? v1.y : 0.f));
    const float2 s3 = make_float2(v3.x + (e03 ? v0.x : 0.f) + (e13 ? v1.x : 0.f) + (e23 ? v2.x : 0.f),
                                  v3.y + (e03 ? v0.y : 0.f) + (e13 ? v1.y : 0.f) + (e23 ? v2.y : 0.f));
    const int a0 = (e01 || e02 || e03) ? OH_CMAX : c0;
    const int a1 = (e12 || e13) ? OH_CMAX : c1;
    const int a2 = e23 ? OH_CMAX : c2;
    const float2 o0 = T2[a0 * LD2], o1 = T2[a1 * LD2], o2 = T2[a2 * LD2], o3 = T2[c3 * LD2];
    T2[a0 * LD2] = make_float2(o0.x + v0.x, o0.y + v0.y);
    T2[a1 * LD2] = make_float2(o1.x + s1.x, o1.y + s1.y);
    T2[a2 * LD2] = make_float2(o2.x + s2.x, o2.y + s2.y);
    T2[c3 * LD2] = make_float2(o3.x + s3.x, o3.y + s3.y);
  };
  auto unit = [&](int b) {
    const int4 k0 = cls[b][wave][0], k1 = cls[b][wave][1], k2 = cls[b][wave][2], k3 = cls[b][wave][3];
    quad(b, 0, k0);
    quad(b, 4, k1);
    quad(b, 8, k2);
    quad(b, 12, k3);
  };
  if (nu > 0) {
    float4 ra, rb;
    int ia, ib;
    OS_LOAD(0, ra, ia);
    OS_LOAD(min(1, nu - 1), rb, ib);
    OS_STORE(0, 0, ra, ia);
    __syncthreads();
    for (int u = 0; u < nu; u += 2) {
      OS_LOAD(min(u + 2, nu - 1), ra, ia);
      unit(0);
      OS_STORE(u + 1, 1, rb, ib);  // past the last unit: every row junk, never read
      __syncthreads();
      if (u + 1 >= nu) break;
      OS_LOAD(min(u + 3, nu - 1), rb, ib);
      unit(1);
      OS_STORE(u + 2, 0, ra, ia);
      __syncthreads();
    }
  }
#undef OS_LOAD
#undef OS_STORE
  if (g < p.G) oh_writeout(T, p, s, g, nb, lane);
}

// ------------------------------------------------------------------ partial-sum reduction
// out[n * ldo + coff + k] = (acc ? out : 0) + sum_s part[s][n][k] for k < K (float4 when K % 4 == 0)
__global__ void __launch_bounds__(256) reduce_kernel(const float* __restrict__ part, int S, int N, int K, float* __restrict__ out,
                                                     long ldo, int coff, int accumulate) {
  const long total = (long)N * K;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if ((K & 3) == 0 && (ldo & 3) == 0 && (coff & 3) == 0) {
    const long i4 = i * 4;
    if (i4 >= total) return;
    // the S chunk partials summed in chunk order (deterministic); 8 loads issued before their adds so the chunk loads
    // are in flight together (the one-at-a-time loop waited a full memory latency per chunk: 19.5 us at 32 x 512 x 512)
    float4 a = reinterpret_cast<const float4*>(part + i4)[0];
    int s = 1;
    for (; s + 8 <= S; s += 8) {
      float4 b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = reinterpret_cast<const float4*>(part + (long)(s + j) * total + i4)[0];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a.x += b[j].x; a.y += b[j].y; a.z += b[j].z; a.w += b[j].w;
      }
    }
    for (; s < S; ++s) {
      const float4 b = reinterpret_cast<const float4*>(part + (long)s * total + i4)[0];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    const long n = i4 / K, k = i4 - n * K;
    float4* o = reinterpret_cast<float4*>(out + n * ldo + coff + k);
    if (accumulate) {
      const float4 c = o[0];
      a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
    }
    o[0] = a;
    return;
  }
  if (i >= total) return;
  float a = part[i];
  int s = 1;
  for (; s + 8 <= S; s += 8) {
    float b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = part[(long)(s + j) * total + i];
#pragma unroll
    for (int j = 0; j < 8; ++j) a += b[j];
  }
  for (; s < S; ++s) a += part[(long)s * total + i];
  const long n = i / K, k = i - n * K;
  float* o = out + n * ldo + coff + k;
  *o = accumulate ? *o + a : a;
}

}  // namespace wgrad
}  // namespace srl

using namespace srl;

// Chunks for the dense split: ~2 workgroups per CU over the output tiles, chunks of >= 256 rows, a
// multiple of 16 rows (one register batch).
int wgrad_dense_chunks(int M, int N, int K) {
  const int tiles = cdiv(N, wgrad::BT) * cdiv(K, wgrad::BT);
  constexpr int target = 512;  // tuned with scripts/wgrad_timing.py
  int S = cdiv(target, tiles);
  const int maxS = cdiv(M, 256);
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  return S;
}

static int dense_rows(int M, int S) {
  int rows = cdiv(M, S);
  rows = cdiv(rows, 2 * wgrad::U) * 2 * wgrad::U;
  return rows;
}

void launch_wgrad_dense(const float* dz, long ldz, const float* x, long ldx, float* part, float* bpart, int M, int N, int K,
                        int S, hipStream_t st) {
  wgrad::DP p;
  p.dz = dz;
  p.x = x;
  p.part = part;
  p.bpart = bpart;
  p.ldz = ldz;
  p.ldx = ldx;
  p.M = M;
  p.N = N;
  p.K = K;
  p.rows = dense_rows(M, S);
  p.S = S;  // trailing chunks past M (rows rounded up) compute and write zero partials
  p.tn = cdiv(N, wgrad::BT);
  p.tk = cdiv(K, wgrad::BT);
  const int grid = p.tn * p.tk * p.S;
  const bool a16 = (N & 3) == 0 && (ldz & 3) == 0 && ((uintptr_t)dz & 15) == 0;
  const bool b16 = (K & 3) == 0 && (ldx & 3) == 0 && ((uintptr_t)x & 15) == 0;
  if (b16) {
    if (a16)
      hipLaunchKernelGGL(wgrad::dense_lds_kernel<true>, dim3(grid), dim3(256), 0, st, p, bpart ? 1 : 0);
    else
      hipLaunchKernelGGL(wgrad::dense_lds_kernel<false>, dim3(grid), dim3(256), 0, st, p, bpart ? 1 : 0);
    return;
  }
  if (bpart)
    hipLaunchKernelGGL(wgrad::dense_kernel<true>, dim3(grid), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(wgrad::dense_kernel<false>, dim3(grid), dim3(256), 0, st, p);
}

// chunks of the one-hot scatter (0 = shape not covered: > 32 classes, odd N / row stride)
int wgrad_onehot_chunks(int M, int N, int G, int C) {
  if (C > wgrad::OH_CMAX || C < 1 || (N & 1)) return 0;
  const int blocks = cdiv(N, wgrad::OH_COLS) * cdiv(G, wgrad::OH_WAVES);
  constexpr int target = 256;
  int S = cdiv(target, blocks);  // one 133 KB-LDS workgroup per CU
  const int maxS = cdiv(M, 256);
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  return S;
}

bool launch_wgrad_onehot(const float* dz, long ldz, const int* idx, long ldi, int off, float* part, int M, int N, int G, int C,
                         int S, hipStream_t st) {
  if (C > wgrad::OH_CMAX || (N & 1) || (ldz & 1) || ((uintptr_t)dz & 7)) return false;
  wgrad::OP p;
  p.dz = dz;
  p.idx = idx;
  p.part = part;
  p.ldz = ldz;
  p.ldi = ldi;
  p.M = M;
  p.N = N;
  p.G = G;
  p.C = C;
  p.off = off;
  p.S = S;
  p.KO = G * C;
  const dim3 grid(cdiv(N, wgrad::OH_COLS), cdiv(G, wgrad::OH_WAVES), S);
  if ((N & 3) == 0 && (ldz & 3) == 0 && ((uintptr_t)dz & 15) == 0) {
    p.rows = cdiv(cdiv(M, S), wgrad::OS_RU) * wgrad::OS_RU;
    hipLaunchKernelGGL(wgrad::onehot_stg_kernel, grid, dim3(wgrad::OH_WAVES * 64), 0, st, p);
    return true;
  }
  p.rows = cdiv(cdiv(M, S), wgrad::OH_RB) * wgrad::OH_RB;
  hipLaunchKernelGGL(wgrad::onehot_kernel, grid, dim3(wgrad::OH_WAVES * 64), 0, st, p);
  return true;
}

void launch_wgrad_reduce(const float* part, int S, int N, int K, float* out, long ldo, int coff, bool accumulate,
                         hipStream_t st) {
  const long total = (long)N * K;
  const bool vec = (K % 4) == 0 && (ldo % 4) == 0 && (coff % 4) == 0;
  const long threads = vec ? total / 4 : total;
  hipLaunchKernelGGL(wgrad::reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, part, S, N, K, out,
                     ldo, coff, accumulate ? 1 : 0);
}
