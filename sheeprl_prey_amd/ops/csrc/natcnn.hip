// NatureCNN convolutions (reference: sheeprl/models/models.py:287-327; conv 8x8 s4 -> 4x4 s2 -> 3x3 s1,
// ReLU after each, "valid" padding) as implicit GEMMs on v_mfma_f32_32x32x2_f32 (exact fp32).
//
// Activations are NHWC, so the GEMM K index of a conv, k = (kh, kw, ci), runs over contiguous
// channels; weights are packed [Co][KH][KW][Ci] (k-contiguous rows).  Three GEMMs per layer:
//
//   FWD    y[m][co]    = relu(b[co] + sum_k col[m][k] W[co][k])          m = (n, oh, ow)
//   WGRAD  dW[co][j]   = sum_m dz[m][co] col[m][j],  db[co] = sum_m dz[m][co]
//          (the bias is one more B row of ones: C[co][K]); split-K over m, fp32 atomics into dW
//   DCOL   dcol[m][j]  = sum_co dz[m][co] W[co][j], then a gather kernel (col2im) sums each input
//          pixel's taps into dx
//
// with dz = dy * (y > 0) applied while staging (the ReLU mask comes from the saved output; no
// pre-activation is stored) and col[m][k] gathered from x on the fly (no im2col buffer).
// Tile 64 x 64 x 32, 4 waves as 2 x 2 of 32 x 32, one LDS stage + register prefetch of the next.
#include "common.h"

#include <algorithm>

namespace srl {
namespace natcnn {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 32, LDK = BK + 4, NTH = 256;
constexpr int NV = 64 * BK / 4 / NTH;  // float4 slots per thread per operand stage (2)

__device__ __forceinline__ f4 z4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// Out-of-range operand slots load this zero vector (unconditional loads, values not selected after the load:
// either made the wait-count pass wait for the next K stage's loads before the current stage's MFMAs).
// The ReLU masks are applied when the registers are written to LDS, after the wait that store needs anyway.
__device__ __attribute__((aligned(16))) float nc_zero16[4];
__device__ __forceinline__ const float* zsrc(bool ok, const float* p) { return ok ? p : nc_zero16; }
__device__ __attribute__((aligned(16))) float nc_one16[4] = {1.f, 0.f, 0.f, 0.f};  // the wgrad bias row's first float4

// Conv geometry: x NHWC [Nb][H][W][Ci] -> y NHWC [Nb][OH][OW][Co], kernel KH x KW, stride S.
struct Geo {
  int Nb, H, W, Ci, OH, OW, Co, KH, KW, S;
  __device__ int M() const { return Nb * OH * OW; }
  __device__ int K() const { return KH * KW * Ci; }
  // NHWC offset of the top-left input pixel of output pixel m
  __device__ int base(int m) const {
    const int ow = m % OW, t = m / OW, oh = t % OH, n = t / OH;
    return ((n * H + oh * S) * W + ow * S) * Ci;
  }
  // offset of tap index k = (kh, kw, ci) relative to base
  __device__ int tap(int k) const {
    const int ci = k % Ci, t = k / Ci, kw = t % KW, kh = t / KW;
    return (kh * W + kw) * Ci + ci;
  }
};

// ---------------------------------------------------------------- loaders (row-major, k contiguous)
// slot v of thread t: row = (t + NTH v) >> 3, k4 = 4 * ((t + NTH v) & 7)
__device__ __forceinline__ void store_rows(const f4* r, float* s) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int idx = threadIdx.x + NTH * v;
    *(f4*)(s + (idx >> 3) * LDK + 4 * (idx & 7)) = r[v];
  }
}
// transposed loaders: slot v: k-dim index kk = idx & 31, rows 4*(idx >> 5) .. +3 (a float4 along rows)
__device__ __forceinline__ void store_trans(const f4* r, float* s) {
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

// FWD A: rows = output pixels m, k = (kh, kw, ci) gathered from x.
struct LIm2col {
  const float* x;
  Geo g;
  int M, K;
  int b[NV];
  __device__ void init(int r0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int m = r0 + ((threadIdx.x + NTH * v) >> 3);
      b[v] = m < M ? g.base(m) : -1;
    }
  }
  __device__ void load(int k0, f4* r) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int k = k0 + 4 * ((threadIdx.x + NTH * v) & 7);
      r[v] = *(const f4*)zsrc(b[v] >= 0 && k < K, x + b[v] + g.tap(k));
    }
  }
  __device__ void store(const f4* r, float* s) const { store_rows(r, s); }
};

// Dense rows [R][ld] (k contiguous), rows >= R or k >= K are zero.  With `mask`: value * (mask > 0)
// (dz = dy * relu'(y) from the saved output y).
struct LRows {
  const float* p;
  const float* mask;
  int R, K, ld;
  int row[NV];
  __device__ void init(int r0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) row[v] = r0 + ((threadIdx.x + NTH * v) >> 3);
  }
  mutable f4 mk[NV];
  __device__ void load(int k0, f4* r) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int k = k0 + 4 * ((threadIdx.x + NTH * v) & 7);
      const bool ok = row[v] < R && k < K;
      r[v] = *(const f4*)zsrc(ok, p + (size_t)row[v] * ld + k);
      if (mask) mk[v] = *(const f4*)zsrc(ok, mask + (size_t)row[v] * ld + k);
    }
  }
  __device__ void store(const f4* r, float* s) const {
    if (!mask) {
      store_rows(r, s);
      return;
    }
    f4 m[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) m[v][e] = mk[v][e] > 0.f ? r[v][e] : 0.f;
    store_rows(m, s);
  }
};

// Transposed dense: GEMM rows j come from columns of p [Kdim][ld] (float4 along j), k-dim = rows of p.
// With `mask`: value * (mask > 0) (same layout as p).
struct LCols {
  const float* p;
  const float* mask;
  int R, Kd, ld;  // R = GEMM rows (columns of p), Kd = rows of p
  int j0;
  __device__ void init(int r0) { j0 = r0; }
  mutable f4 mk[NV];
  __device__ void load(int k0, f4* r) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      const int kk = k0 + (idx & 31), j = j0 + 4 * (idx >> 5);
      const bool ok = kk < Kd && j < R;
      r[v] = *(const f4*)zsrc(ok, p + (size_t)kk * ld + j);
      if (mask) mk[v] = *(const f4*)zsrc(ok, mask + (size_t)kk * ld + j);
    }
  }
  __device__ void store(const f4* r, float* s) const {
    if (!mask) {
      store_trans(r, s);
      return;
    }
    f4 m[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) m[v][e] = mk[v][e] > 0.f ? r[v][e] : 0.f;
    store_trans(m, s);
  }
};

// WGRAD B: GEMM rows j = (kh, kw, ci) (plus row K = the bias: all ones), k-dim = output pixels m;
// value col[m][j] gathered from x (float4 along ci).
struct LIm2colT {
  const float* x;
  Geo g;
  int M, K, j0;
  __device__ void init(int r0) { j0 = r0; }
  __device__ void load(int k0, f4* r) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int idx = threadIdx.x + NTH * v;
      const int m = k0 + (idx & 31), j = j0 + 4 * (idx >> 5);
      // bias row (K % 4 == 0, so j == K starts a float4): (1, 0, 0, 0); past it / past M: zeros
      const float* src = (m < M && j < K) ? x + g.base(m) + g.tap(j) : ((m < M && j == K) ? nc_one16 : nc_zero16);
      r[v] = *(const f4*)src;
    }
  }
  __device__ void store(const f4* r, float* s) const { store_trans(r, s); }
};

// ---------------------------------------------------------------- epilogues
// acc (32x32x2 C/D layout): element r of lane -> row 8*(r>>2) + 4*(lane>>5) + (r&3), col lane&31
struct EBiasRelu {  // y[m][c] = relu(acc + b[c])
  float* y;
  const float* b;
  int M, N;
  __device__ void run(const f16v& acc, int r0, int c0) const {
    const int lane = threadIdx.x & 63, c = c0 + (lane & 31);
    if (c >= N) return;
    const float bc = b ? b[c] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = r0 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      if (m < M) y[(size_t)m * N + c] = fmaxf(acc[r] + bc, 0.f);
    }
  }
};
struct EStore {  // out[m][c] = acc
  float* out;
  int M, N;
  __device__ void run(const f16v& acc, int r0, int c0) const {
    const int lane = threadIdx.x & 63, c = c0 + (lane & 31);
    if (c >= N) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = r0 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      if (m < M) out[(size_t)m * N + c] = acc[r];
    }
  }
};
struct EWgrad {  // split-K partial: dW[co][j] += acc (j < K), db[co] += acc (j == K)
  float* dw;
  float* db;
  int M, K;
  __device__ void run(const f16v& acc, int r0, int c0) const {
    const int lane = threadIdx.x & 63, j = c0 + (lane & 31);
    if (j > K) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = r0 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      if (co >= M) continue;
      if (j < K)
        atomicAdd(dw + (size_t)co * K + j, acc[r]);
      else if (db)
        atomicAdd(db + co, acc[r]);
    }
  }
};

// ---------------------------------------------------------------- GEMM main loop
// C[BM x BN tile] over k in [kz * kper, min(Ktot, (kz + 1) * kper))
template <class LA, class LB, class EP>
__global__ __launch_bounds__(NTH) void gemm_kernel(LA la, LB lb, EP ep, int Ktot, int kper) {
  __shared__ float lds[(BM + BN) * LDK];
  float* As = lds;
  float* Bs = lds + BM * LDK;
  const int r0 = blockIdx.x * BM, c0 = blockIdx.y * BN;
  const int kb = blockIdx.z * kper, ke = min(Ktot, kb + kper);
  la.init(r0);
  lb.init(c0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  f16v acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  f4 ra[NV], rb[NV];
  la.load(kb, ra);
  lb.load(kb, rb);
  const int arow = wm * 32 + (lane & 31), brow = wn * 32 + (lane & 31), kof = 4 * (lane >> 5);
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
      const f4 a = *(const f4*)(As + arow * LDK + 8 * s + kof);
      const f4 b = *(const f4*)(Bs + brow * LDK + 8 * s + kof);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q], b[q], acc, 0, 0, 0);
    }
  }
  ep.run(acc, r0 + wm * 32, c0 + wn * 32);
}

// dx[n][ih][iw][ci] = sum over taps (kh, kw) with oh = (ih - kh) / S, ow = (iw - kw) / S integral and
// in range of dcol[(n, oh, ow)][(kh, kw, ci)].  One thread per 4 channels of an input pixel.
__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcol, float* __restrict__ dx, Geo g) {
  const int c4 = g.Ci / 4;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= g.Nb * g.H * g.W * c4) return;
  const int ci = 4 * (idx % c4), pix = idx / c4;
  const int iw = pix % g.W, t = pix / g.W, ih = t % g.H, n = t / g.H;
  const int K = g.KH * g.KW * g.Ci;
  f4 s = z4();
  for (int kh = ih % g.S; kh < g.KH; kh += g.S) {
    const int oh = (ih - kh) / g.S;
    if (oh < 0 || oh >= g.OH || ih - kh < 0) continue;
    for (int kw = iw % g.S; kw < g.KW; kw += g.S) {
      const int ow = (iw - kw) / g.S;
      if (ow < 0 || ow >= g.OW || iw - kw < 0) continue;
      const int m = (n * g.OH + oh) * g.OW + ow;
      s += *(const f4*)(dcol + (size_t)m * K + (kh * g.KW + kw) * g.Ci + ci);
    }
  }
  *(f4*)(dx + (size_t)pix * g.Ci + ci) = s;
}

}  // namespace natcnn
}  // namespace srl

using namespace srl::natcnn;

namespace {
Geo geo(int Nb, int H, int W, int Ci, int Co, int KH, int KW, int S) {
  Geo g{Nb, H, W, Ci, (H - KH) / S + 1, (W - KW) / S + 1, Co, KH, KW, S};
  return g;
}
inline int cdiv_(int a, int b) { return (a + b - 1) / b; }
}  // namespace

// y [Nb*OH*OW][Co] = relu(conv(x) + b); w packed [Co][KH*KW*Ci]
void natcnn_fwd(const float* x, const float* w, const float* b, float* y, int Nb, int H, int W, int Ci, int Co, int KH,
                int KW, int S, hipStream_t st) {
  const Geo g = geo(Nb, H, W, Ci, Co, KH, KW, S);
  const int M = g.Nb * g.OH * g.OW, K = KH * KW * Ci;
  LIm2col la{x, g, M, K, {}};
  LRows lb{w, nullptr, Co, K, K, {}};
  EBiasRelu ep{y, b, M, Co};
  hipLaunchKernelGGL((gemm_kernel<LIm2col, LRows, EBiasRelu>), dim3(cdiv_(M, BM), cdiv_(Co, BN), 1), dim3(NTH), 0, st, la,
                     lb, ep, K, K);
}

// dw [Co][K] and db [Co] ACCUMULATE (zero them first): dz = dy * (y > 0)
void natcnn_wgrad(const float* x, const float* dy, const float* y, float* dw, float* db, int Nb, int H, int W, int Ci,
                  int Co, int KH, int KW, int S, hipStream_t st) {
  const Geo g = geo(Nb, H, W, Ci, Co, KH, KW, S);
  const int M = g.Nb * g.OH * g.OW, K = KH * KW * Ci;
  LCols la{dy, y, Co, M, Co, 0};
  LIm2colT lb{x, g, M, K, 0};
  EWgrad ep{dw, db, Co, K};
  const int tiles = cdiv_(Co, BM) * cdiv_(K + 1, BN);
  int split = std::max(1, std::min(64, 512 / std::max(1, tiles)));  // ~2 workgroups per CU overall
  int kper = cdiv_(cdiv_(M, split), BK) * BK;
  split = cdiv_(M, kper);
  hipLaunchKernelGGL((gemm_kernel<LCols, LIm2colT, EWgrad>), dim3(cdiv_(Co, BM), cdiv_(K + 1, BN), split), dim3(NTH), 0, st,
                     la, lb, ep, M, kper);
}

// dx NHWC [Nb][H][W][Ci] from dy (masked by y > 0); dcol scratch [M][K]
void natcnn_dgrad(const float* dy, const float* y, const float* w, float* dcol, float* dx, int Nb, int H, int W, int Ci,
                  int Co, int KH, int KW, int S, hipStream_t st) {
  const Geo g = geo(Nb, H, W, Ci, Co, KH, KW, S);
  const int M = g.Nb * g.OH * g.OW, K = KH * KW * Ci;
  LRows la{dy, y, M, Co, Co, {}};
  LCols lb{w, nullptr, K, Co, K, 0};
  EStore ep{dcol, M, K};
  hipLaunchKernelGGL((gemm_kernel<LRows, LCols, EStore>), dim3(cdiv_(M, BM), cdiv_(K, BN), 1), dim3(NTH), 0, st, la, lb, ep,
                     Co, Co);
  const int n = Nb * H * W * (Ci / 4);
  hipLaunchKernelGGL(col2im_kernel, dim3(cdiv_(n, 256)), dim3(256), 0, st, dcol, dx, g);
}
