// Plan2Explore disagreement reward (K20; reference p2e_dv1/p2e_dv1.py and p2e_dv2/p2e_dv2.py: the
// intrinsic reward is the variance over the ensemble members' next-state predictions, averaged over
// the prediction features):
//
//   pred_i = X_i W_i^T + b_i          X: [n, M, H] last hidden layer of every member, W: [n, O, H]
//   r[m]   = mean_c var_i pred_i[m, c]  (unbiased variance over the n members)
//
// The head GEMMs of all members and the variance are ONE kernel: the [n, M, O] prediction tensor
// (n x 16384 x 1024 floats = 671 MB for DreamerV2 P2E) is never written or read back.  Workgroup
// tile 128 rows x 64 features, 4 waves (32 rows each: 2 x 4 tiles of 16x16 MFMA); per member the K
// loop stages 64-wide chunks of X_i and W_i through LDS (the next chunk - or the next member's first -
// is fetched into registers behind the MFMAs) and runs v_mfma_f32_16x16x4f32; the member results are
// folded into a per-element Welford (mean, M2) in registers (64 per lane survive across members).
// Each workgroup writes one partial per row (sum over its 64 features of the variance); the caller
// sums the O/64 partials (fixed order, deterministic).
#include "common.h"


namespace srl {
namespace ens {

constexpr int NTH = 256;
constexpr int BM = 128, BN = 64, KC = 64;
constexpr int NA = BM * KC / 4 / NTH, NB = BN * KC / 4 / NTH;  // float4 per thread per chunk: 8, 4

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct EP {
  const float* X;  // [n, M, H]
  const float* W;  // [n, O, H]
  const float* b;  // [n, O] or null
  float* part;     // [ceil(O / 64), M]
  int n, M, O, H;
};

__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

// chunk rows [r0, r0 + R) x k [k0, k0 + KC) of a row-major [rows, H] matrix into registers; zero
// outside [0, nrows) x [0, H).  H % 4 == 0, so a float4 never straddles the K edge.
template <int NV>
__device__ __forceinline__ void fetch(float4* reg, const float* src, int nrows, int H, int r0, int k0) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int idx = threadIdx.x + NTH * v;
    const int r = idx / (KC / 4), c4 = idx % (KC / 4);
    const int row = r0 + r, k = k0 + 4 * c4;
    reg[v] = (row < nrows && k < H) ? *reinterpret_cast<const float4*>(src + (size_t)row * H + k) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int NV, int LDK>
__device__ __forceinline__ void put(float* dst, const float4* reg) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int idx = threadIdx.x + NTH * v;
    *reinterpret_cast<float4*>(dst + (idx / (KC / 4)) * LDK + 4 * (idx % (KC / 4))) = reg[v];
  }
}

template <int LDK>
__global__ __launch_bounds__(NTH) void disagreement_kernel(EP p) {
  __shared__ float As[BM * LDK];
  __shared__ float Bs[BN * LDK];
  __shared__ float red[4][32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * BM, c0 = blockIdx.y * BN;
  // wave w: rows 32w .. 32w + 31 (row tiles rt = 0, 1) x the workgroup's 64 features (column tiles t)
  float mean[2][4][4], m2[2][4][4];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) mean[rt][t][e] = m2[rt][t][e] = 0.f;
  const int nk = (p.H + KC - 1) / KC;
  float4 ra[NA], rb[NB];
  fetch<NA>(ra, p.X, p.M, p.H, r0, 0);
  fetch<NB>(rb, p.W, p.O, p.H, c0, 0);
  for (int i = 0; i < p.n; ++i) {
    floatx4 acc[2][4];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[rt][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < nk; ++kc) {
      __syncthreads();  // previous chunk's readers are done
      put<NA, LDK>(As, ra);
      put<NB, LDK>(Bs, rb);
      __syncthreads();
      // prefetch the next chunk (this member's next K chunk, or the next member's first) behind the MFMAs
      {
        const int ni = kc + 1 < nk ? i : i + 1, nk0 = kc + 1 < nk ? (kc + 1) * KC : 0;
        if (ni < p.n) {
          fetch<NA>(ra, p.X + (size_t)ni * p.M * p.H, p.M, p.H, r0, nk0);
          fetch<NB>(rb, p.W + (size_t)ni * p.O * p.H, p.O, p.H, c0, nk0);
        }
      }
#pragma unroll
      for (int kk = 0; kk < KC; kk += 16) {
        // permuted K: lane (j, q) feeds k = kk + 4q + e to MFMA e, for both operands
        float4 a[2], bv[4];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) a[rt] = *reinterpret_cast<const float4*>(As + (32 * w + 16 * rt + j) * LDK + 4 * q + kk);
#pragma unroll
        for (int t = 0; t < 4; ++t) bv[t] = *reinterpret_cast<const float4*>(Bs + (16 * t + j) * LDK + 4 * q + kk);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 4; ++t)
              acc[rt][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a[rt], e), comp(bv[t], e), acc[rt][t], 0, 0, 0);
      }
    }
    // member i's tile -> Welford over members (acc[rt][t][e]: row 32w + 16rt + 4q + e, feature c0 + 16t + j)
    const float inv = 1.f / (float)(i + 1);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = c0 + 16 * t + j;
      const float bb = (p.b && c < p.O) ? p.b[(size_t)i * p.O + c] : 0.f;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = acc[rt][t][e] + bb;
          const float d = x - mean[rt][t][e];
          mean[rt][t][e] += d * inv;
          m2[rt][t][e] += d * (x - mean[rt][t][e]);
        }
    }
  }
  // unbiased variance, summed over this workgroup's features (features >= O are all-zero: var 0)
  const float den = p.n > 1 ? 1.f / (float)(p.n - 1) : 0.f;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) s += m2[rt][t][e] * den;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (j == 0) red[w][16 * rt + 4 * q + e] = s;
    }
  __syncthreads();
  if (threadIdx.x < BM) {
    const int r = threadIdx.x, row = r0 + r;
    if (row < p.M) p.part[(size_t)blockIdx.y * p.M + row] = red[r >> 5][r & 31];
  }
}

}  // namespace ens
}  // namespace srl

bool launch_ens_disagreement(const float* X, const float* W, const float* b, float* part, int n, int M, int O, int H,
                             hipStream_t st) {
  if (n < 1 || M < 1 || O < 1 || H < 4 || (H & 3)) return false;
  srl::ens::EP p{X, W, b, part, n, M, O, H};
  dim3 grid((M + srl::ens::BM - 1) / srl::ens::BM, (O + srl::ens::BN - 1) / srl::ens::BN);
  // LDS row stride 72 floats (64-wide K chunk + padding): measured fastest for the DV2-P2E shape (1479 us vs
  // 1518 at 68 and 1514 at 80, profiles/r2_p2e_disagreement.md)
  hipLaunchKernelGGL(srl::ens::disagreement_kernel<72>, grid, dim3(srl::ens::NTH), 0, st, p);
  return true;
}
