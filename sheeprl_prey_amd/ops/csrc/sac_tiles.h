// 16-row fp32 MFMA tiles of the SAC MLP kernels (sac_critic.hip, sac_fused.hip): batch-256 MLPs with 256-wide
// hidden layers are latency-bound, so every helper computes one 16 x 16 output tile per wave with
// v_mfma_f32_16x16x4f32 and issues the loads of KC K-steps before the MFMAs that consume them (one L2
// latency per chunk instead of one per K-step).
//
// Operand layout (all helpers): lane (j = lane & 15, q = lane >> 4) of MFMA e supplies A[row j][k] and
// B[k][col j] for k = k0 + 4 q + e, so neither operand needs a shuffle; the result acc[e] of lane (j, q) is
// C[row 4 q + e][col j].
#pragma once
#include <hip/hip_runtime.h>

namespace srl {
namespace sactile {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int KC = 8;

__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

// acc (16 rows x 16 cols from weight row n0) += act[16][K] . W[n0.., K]^T ; act in LDS (stride lda), W row-major.
// K % 16 == 0.
__device__ __forceinline__ floatx4 tile_gemm_nt(const float* act, int lda, const float* W, int ldw, int n0, int K, int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* wr = W + (long)(n0 + j) * ldw + 4 * q;
  const float* ar = act + j * lda + 4 * q;
  for (int kb = 0; kb < K; kb += 16 * KC) {
    float4 w[KC], a[KC];
#pragma unroll
    for (int u = 0; u < KC; ++u)
      if (kb + 16 * u < K) w[u] = *reinterpret_cast<const float4*>(wr + kb + 16 * u);
#pragma unroll
    for (int u = 0; u < KC; ++u)
      if (kb + 16 * u < K) a[u] = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (kb + 16 * u < K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a[u], e), comp(w[u], e), acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

// Same product with one weight row pointer per lane (row j of the tile), nullptr = a zero row: heads whose
// output columns come from several weight matrices (SAC actor mean / log-std).  K % 16 == 0, rows 16-byte aligned.
__device__ __forceinline__ floatx4 tile_gemm_rows(const float* act, int lda, const float* wrow, int K, int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* ar = act + j * lda + 4 * q;
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kb = 0; kb < K; kb += 16 * KC) {
    float4 w[KC], a[KC];
#pragma unroll
    for (int u = 0; u < KC; ++u)
      if (kb + 16 * u < K) w[u] = wrow ? *reinterpret_cast<const float4*>(wrow + kb + 16 * u + 4 * q) : zero;
#pragma unroll
    for (int u = 0; u < KC; ++u)
      if (kb + 16 * u < K) a[u] = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (kb + 16 * u < K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a[u], e), comp(w[u], e), acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

// acc (16 rows x 16 cols from weight row n0) += act[16][Kp] . W[n0.., K]^T for a K that is not a multiple of 16
// (first layers: observation / action widths).  Columns k >= K read as zero.  CH K-steps (4 CH columns) of weight
// loads in flight per chunk: a per-step load -> MFMA loop waits one memory round trip per 4 columns.  CH = 1 where
// the enclosing kernel is at its register limit (the compiler spills the chunked form there).
template <int CH = 16>
__device__ __forceinline__ floatx4 tile_gemm_nt_small(const float* act, int lda, const float* W, int ldw, int n0, int K,
                                                      int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* wr = W + (long)(n0 + j) * ldw;
  for (int k0 = 0; k0 < K; k0 += 4 * CH) {
    float w[CH], a[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = k0 + 4 * u + q;
      w[u] = k < K ? wr[k] : 0.f;
      a[u] = k < K ? act[j * lda + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (k0 + 4 * u < K) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], w[u], acc, 0, 0, 0);
  }
  return acc;
}

// Two tiles of tile_gemm_nt_small at once (both tiles' weight loads in flight together).
template <int CH = 16>
__device__ __forceinline__ void tile2_gemm_nt_small(const float* act, int lda, const float* W, int ldw, int n0a, int n0b,
                                                    int K, int lane, floatx4& ca, floatx4& cb) {
  const int j = lane & 15, q = lane >> 4;
  ca = floatx4{0.f, 0.f, 0.f, 0.f};
  cb = ca;
  const float* wa = W + (long)(n0a + j) * ldw;
  const float* wb = W + (long)(n0b + j) * ldw;
  for (int k0 = 0; k0 < K; k0 += 4 * CH) {
    float xa[CH], xb[CH], a[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int k = k0 + 4 * u + q;
      xa[u] = k < K ? wa[k] : 0.f;
      xb[u] = k < K ? wb[k] : 0.f;
      a[u] = k < K ? act[j * lda + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (k0 + 4 * u < K) {
        ca = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], xa[u], ca, 0, 0, 0);
        cb = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], xb[u], cb, 0, 0, 0);
      }
  }
}

// acc (16 rows x 16 cols from column n0) += act[16][K] . W[K, n0..]   (W row-major [K][ldw]: read K-major)
__device__ __forceinline__ floatx4 tile_gemm_nn(const float* act, int lda, const float* W, int ldw, int n0, int K, int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* wc = W + n0 + j;
  const float* ar = act + j * lda + 4 * q;
  for (int kb = 0; kb < K; kb += 16 * KC) {
    float w[KC][4];
#pragma unroll
    for (int u = 0; u < KC; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) w[u][e] = kb + 16 * u < K ? wc[(long)(kb + 16 * u + 4 * q + e) * ldw] : 0.f;
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (kb + 16 * u < K) {
        const float4 a = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), w[u][e], acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

// tile_gemm_nn restricted to the first `ncols` columns of the tile (columns >= ncols read as zero): the
// action-input slice of a critic's first layer.  K % 16 == 0; 8 K-steps of weight loads in flight per chunk.
__device__ __forceinline__ floatx4 tile_gemm_nn_cols(const float* act, int lda, const float* W, int ldw, int ncols, int K,
                                                     int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const bool ok = j < ncols;
  const float* ar = act + j * lda + 4 * q;
  for (int kb = 0; kb < K; kb += 64) {
    float w[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) w[u][e] = ok && kb + 16 * u < K ? W[(long)(kb + 16 * u + 4 * q + e) * ldw + j] : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (kb + 16 * u < K) {
        const float4 a = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), w[u][e], acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

// Two tiles (weight rows n0a.., n0b..) of act[16][K] . W^T at once, KC2 = 16 K-steps of BOTH tiles' weight loads in
// flight per chunk (one memory round trip per 256-deep layer instead of four), the activation operand read once per
// K-step for both tiles.  The layers of the SAC MLPs are latency-bound: a 16-row block's whole layer is 32 tiles x 1
// MFMA chain, so cutting round trips is what cuts time.  K % 16 == 0.
constexpr int KC2 = 16;
__device__ __forceinline__ void tile2_gemm_nt(const float* act, int lda, const float* W, int ldw, int n0a, int n0b, int K,
                                              int lane, floatx4& ca, floatx4& cb) {
  const int j = lane & 15, q = lane >> 4;
  const float* wa = W + (long)(n0a + j) * ldw + 4 * q;
  const float* wb = W + (long)(n0b + j) * ldw + 4 * q;
  const float* ar = act + j * lda + 4 * q;
  ca = floatx4{0.f, 0.f, 0.f, 0.f};
  cb = ca;
  for (int kb = 0; kb < K; kb += 16 * KC2) {
    float4 xa[KC2], xb[KC2];
#pragma unroll
    for (int u = 0; u < KC2; ++u)
      if (kb + 16 * u < K) {
        xa[u] = *reinterpret_cast<const float4*>(wa + kb + 16 * u);
        xb[u] = *reinterpret_cast<const float4*>(wb + kb + 16 * u);
      }
#pragma unroll
    for (int u = 0; u < KC2; ++u) {
      if (kb + 16 * u < K) {
        const float4 a = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ca = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), comp(xa[u], e), ca, 0, 0, 0);
          cb = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), comp(xb[u], e), cb, 0, 0, 0);
        }
      }
    }
  }
}

// Two tiles (columns n0a.., n0b..) of act[16][K] . W[K, :] (W row-major [K][ldw], read K-major), KC2 K-steps of both
// tiles' weight loads in flight per chunk.  K % 16 == 0.
__device__ __forceinline__ void tile2_gemm_nn(const float* act, int lda, const float* W, int ldw, int n0a, int n0b, int K,
                                              int lane, floatx4& ca, floatx4& cb) {
  const int j = lane & 15, q = lane >> 4;
  const float* wa = W + n0a + j;
  const float* wb = W + n0b + j;
  const float* ar = act + j * lda + 4 * q;
  ca = floatx4{0.f, 0.f, 0.f, 0.f};
  cb = ca;
  for (int kb = 0; kb < K; kb += 16 * KC2) {
    float xa[KC2][4], xb[KC2][4];
#pragma unroll
    for (int u = 0; u < KC2; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = kb + 16 * u < K;
        const long r = (long)(kb + 16 * u + 4 * q + e) * ldw;
        xa[u][e] = ok ? wa[r] : 0.f;
        xb[u][e] = ok ? wb[r] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < KC2; ++u) {
      if (kb + 16 * u < K) {
        const float4 a = *reinterpret_cast<const float4*>(ar + kb + 16 * u);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ca = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), xa[u][e], ca, 0, 0, 0);
          cb = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), xb[u][e], cb, 0, 0, 0);
        }
      }
    }
  }
}

// Every 16-column tile a wave owns in an N-wide layer over NW waves (tiles wave * T .. wave * T + T - 1,
// T = N / (16 NW)), two at a time: epi(n0, acc) for each.  FORM 0: W rows (tile2_gemm_nt, K % 16 == 0), 1: W read
// K-major (tile2_gemm_nn), 2: W rows with any K (tile2_gemm_nt_small: first layers), 3: as 2 with one K-step per
// chunk (kernels at their register limit).
template <int FORM, int NW, typename Epi>
__device__ __forceinline__ void wave_tiles(const float* act, int lda, const float* W, int ldw, int N, int K, int lane,
                                           int wave, Epi epi) {
  const int T = N / (16 * NW);
  for (int t = 0; t < T; t += 2) {
    const int n0a = (wave * T + t) * 16;
    if (t + 1 < T) {
      floatx4 ca, cb;
      if (FORM == 1) tile2_gemm_nn(act, lda, W, ldw, n0a, n0a + 16, K, lane, ca, cb);
      else if (FORM == 2) tile2_gemm_nt_small<16>(act, lda, W, ldw, n0a, n0a + 16, K, lane, ca, cb);
      else if (FORM == 3) tile2_gemm_nt_small<1>(act, lda, W, ldw, n0a, n0a + 16, K, lane, ca, cb);
      else tile2_gemm_nt(act, lda, W, ldw, n0a, n0a + 16, K, lane, ca, cb);
      epi(n0a, ca);
      epi(n0a + 16, cb);
    } else {
      epi(n0a, FORM == 1   ? tile_gemm_nn(act, lda, W, ldw, n0a, K, lane)
               : FORM == 2 ? tile_gemm_nt_small<16>(act, lda, W, ldw, n0a, K, lane)
               : FORM == 3 ? tile_gemm_nt_small<1>(act, lda, W, ldw, n0a, K, lane)
                           : tile_gemm_nt(act, lda, W, ldw, n0a, K, lane));
    }
  }
}

// out tile (16 x 16) = sum_r G[r][i0 + i] * A[r][j0 + jj]  (both row-major, row strides ldg / lda); KC/2
// row steps of loads in flight per chunk.  Rows r >= M read as zero.
__device__ __forceinline__ floatx4 tile_wgrad(const float* G, int ldg, const float* A, int lda, int i0, int j0, int M,
                                              int lane) {
  const int j = lane & 15, q = lane >> 4;
  constexpr int RC = KC / 2;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* gc = G + i0 + j;
  const float* ac = A + j0 + j;
  for (int kb = 0; kb < M; kb += 16 * RC) {
    float a[RC][4], b[RC][4];
#pragma unroll
    for (int u = 0; u < RC; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = kb + 16 * u + 4 * q + e;
        a[u][e] = r < M ? gc[(long)r * ldg] : 0.f;
        b[u][e] = r < M ? ac[(long)r * lda] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < RC; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][e], b[u][e], acc, 0, 0, 0);
  }
  return acc;
}

}  // namespace sactile
}  // namespace srl
