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
// (first layers: observation / action widths).  Columns k >= K of act are multiplied by zero weights.
__device__ __forceinline__ floatx4 tile_gemm_nt_small(const float* act, int lda, const float* W, int ldw, int n0, int K,
                                                      int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* wr = W + (long)(n0 + j) * ldw;
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + q;
    const float w = k < K ? wr[k] : 0.f;
    const float a = k < K ? act[j * lda + k] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w, acc, 0, 0, 0);
  }
  return acc;
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
// action-input slice of a critic's first layer.  K % 16 == 0.
__device__ __forceinline__ floatx4 tile_gemm_nn_cols(const float* act, int lda, const float* W, int ldw, int ncols, int K,
                                                     int lane) {
  const int j = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const bool ok = j < ncols;
  const float* ar = act + j * lda + 4 * q;
  for (int kb = 0; kb < K; kb += 16) {
    const float4 a = *reinterpret_cast<const float4*>(ar + kb);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float w = ok ? W[(long)(kb + 4 * q + e) * ldw + j] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), w, acc, 0, 0, 0);
    }
  }
  return acc;
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
