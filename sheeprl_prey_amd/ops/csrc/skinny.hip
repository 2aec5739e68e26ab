// Skinny weight-streaming GEMM:  out[z] = A[z] . W[z]^T (+ add[z])   with  M <= 16 activation rows.
//
// The DreamerV3-XL recurrence (deter 4096, dense 1024; reference configs/exp/dreamer_v3_XL_crafter.yaml,
// loop dreamer_v3/agent.py:350-388) multiplies B = 16 state rows by ~300 MB of weights per time step:
// 16 x 5120 x 12288 for the GRU projection alone.  That is pure weight streaming (16 FLOP per byte), so
// the kernel is built for HBM3E, not for MFMA peak:
//
//  * W is read exactly once, straight from HBM into registers (no LDS round trip): each wave owns 32
//    weight rows x one K chunk; lane (j, q) reads 64 contiguous bytes of row j per load, eight loads per
//    row group per 128-wide K step, and the next step's loads are issued before this step's MFMAs
//    (16 KiB in flight per wave).
//  * split-K over the grid: N/128 row blocks x ~K/kc chunks ~ 640 workgroups so every CU streams; the
//    per-chunk partials (~WGs x 8 KiB) are summed, with the addend (bias / action projection), by a
//    second small kernel that spreads the chunks over 4 waves per output tile.
//    (an in-launch ticket combine of the partials measured slower - profiles/r4_skinny_fused.md - and was removed)
//  * the A chunk (16 x kc) is staged once per workgroup in LDS (row stride kc+4) and shared by its 4 waves.
//  * v_mfma_f32_16x16x4_f32 with a permuted K order: lane (j, q) of float4 i, component e feeds MFMA
//    k = 16 i + 4 q + e for both operands, so one 64 B load per row maps onto the MFMA B layout
//    (B[k = lane>>4][col = lane&15]) without shuffles.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace srl {
namespace skinny {

constexpr int NTH = 256;
constexpr int WG_ROWS = 128;  // weight rows per workgroup (4 waves x 32)
constexpr int KSTEP = 128;
constexpr int TARGET_WGS = 1024;  // ~2.5 per CU: 40 KiB+ in flight per CU, partials ~ WGs x 8 KiB

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct SP {
  const float* A;
  long lda, sA;
  const float* W;
  long ldw, sW;
  float* out;
  long ldo, sO;
  const float* add;
  long ldadd, sAdd;
  float* part;
  int M, N, K, kc, splits, Z;
};

// weights are touched once per launch: streaming (non-temporal) loads keep them from evicting A / partials
template <bool NT>
__device__ __forceinline__ float4 ldw4(const float* p) {
  if (NT) {
    const floatx4 v = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  return *reinterpret_cast<const float4*>(p);
}

__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

template <bool NT>
__global__ __launch_bounds__(NTH) void skinny_nt_kernel(SP p) {
  extern __shared__ float As[];  // [16][kc + 4]
  const int nb = blockIdx.x, s = blockIdx.y, z = blockIdx.z;
  const int k0 = s * p.kc;
  const int kc = min(p.kc, p.K - k0);
  const int lds = p.kc + 4;
  const float* A = p.A + (long)z * p.sA;
  const float* W = p.W + (long)z * p.sW;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
  const int n0 = nb * WG_ROWS + wave * 32;
  const float* w0 = W + (long)(n0 + j) * p.ldw + k0 + 4 * q;
  const float* w1 = w0 + 16 * p.ldw;
  const float* ar = As + j * lds + 4 * q;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  // 128-wide K steps: 16 float4 per lane in flight (16 KiB per wave) while the previous step computes.
  // The first step's weights are requested before the A chunk is staged (they do not depend on it).
  float4 wa[8], wb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    wa[i] = ldw4<NT>(w0 + 16 * i);
    wb[i] = ldw4<NT>(w1 + 16 * i);
  }
  const int c4n = kc >> 2;
  for (int idx = threadIdx.x; idx < 16 * c4n; idx += NTH) {
    const int r = idx / c4n, c = idx - r * c4n;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < p.M) v = *reinterpret_cast<const float4*>(A + (long)r * p.lda + k0 + 4 * c);
    *reinterpret_cast<float4*>(As + r * lds + 4 * c) = v;
  }
  __syncthreads();
  for (int kb = 0; kb < kc; kb += KSTEP) {
    // next step's weights first (clamped on the last step: a harmless re-read, keeps the loads unconditional)
    const int kn = min(kb + KSTEP, kc - KSTEP);
    float4 na[8], nb4[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      na[i] = ldw4<NT>(w0 + kn + 16 * i);
      nb4[i] = ldw4<NT>(w1 + kn + 16 * i);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 a4 = *reinterpret_cast<const float4*>(ar + kb + 16 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a4, e), comp(wa[i], e), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a4, e), comp(wb[i], e), acc1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      wa[i] = na[i];
      wb[i] = nb4[i];
    }
  }
  // D layout: col = lane & 15 (weight row), row = 4 * (lane >> 4) + e (activation row)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = 4 * q + e;
    if (m >= p.M) continue;
    const int na_ = n0 + j, nb_ = n0 + 16 + j;
    if (p.splits == 1) {
      float* o = p.out + (long)z * p.sO + (long)m * p.ldo;
      const float* ad = p.add ? p.add + (long)z * p.sAdd + (long)m * p.ldadd : nullptr;
      o[na_] = acc0[e] + (ad ? ad[na_] : 0.f);
      o[nb_] = acc1[e] + (ad ? ad[nb_] : 0.f);
    } else {
      float* pr = p.part + (((long)s * p.Z + z) * 16 + m) * p.N;
      pr[na_] = acc0[e];
      pr[nb_] = acc1[e];
    }
  }
}

// out[z][m][n] = add[z][m][n] + sum_s part[s][z][m][n].  One workgroup per (z, m, 64 float4 columns):
// wave w sums the chunks s = w, w+4, ... and the four wave sums combine in LDS in a fixed order
// (deterministic), so the split count does not serialise one thread.
__global__ __launch_bounds__(NTH) void skinny_reduce_kernel(SP p) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n4 = p.N >> 2;
  const int c = blockIdx.x * 64 + lane, m = blockIdx.y, z = blockIdx.z;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < n4) {
    for (int s = w; s < p.splits; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p.part + (((long)s * p.Z + z) * 16 + m) * p.N + 4 * c);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < n4) {
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.add) r = *reinterpret_cast<const float4*>(p.add + (long)z * p.sAdd + (long)m * p.ldadd + 4 * c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r.x += red[i][lane].x;
      r.y += red[i][lane].y;
      r.z += red[i][lane].z;
      r.w += red[i][lane].w;
    }
    *reinterpret_cast<float4*>(p.out + (long)z * p.sO + (long)m * p.ldo + 4 * c) = r;
  }
}

}  // namespace skinny
}  // namespace srl

// Split plan: returns the number of K chunks (and the chunk width in *kc).
int skinny_plan(int N, int K, int Z, int* kc) {
  constexpr int target = srl::skinny::TARGET_WGS;
  const int nblk = std::max(1, N / srl::skinny::WG_ROWS * Z);
  int splits = std::max(1, std::min(K / srl::skinny::KSTEP, (target + nblk - 1) / nblk));
  int c = (K + splits - 1) / splits;
  c = (c + srl::skinny::KSTEP - 1) / srl::skinny::KSTEP * srl::skinny::KSTEP;
  c = std::min(c, 2048);
  *kc = c;
  return (K + c - 1) / c;
}

void launch_skinny_nt(const float* A, long lda, long sA, const float* W, long ldw, long sW, float* out, long ldo, long sO,
                      const float* add, long ldadd, long sAdd, float* part, int M, int N, int K, int Z,
                      hipStream_t st) {
  srl::skinny::SP p;
  p.A = A;
  p.lda = lda;
  p.sA = sA;
  p.W = W;
  p.ldw = ldw;
  p.sW = sW;
  p.out = out;
  p.ldo = ldo;
  p.sO = sO;
  p.add = add;
  p.ldadd = ldadd;
  p.sAdd = sAdd;
  p.part = part;
  p.M = M;
  p.N = N;
  p.K = K;
  p.Z = Z;
  p.splits = skinny_plan(N, K, Z, &p.kc);
  const size_t lds = sizeof(float) * 16 * (size_t)(p.kc + 4);
  // weight loads use the default cache policy: the non-temporal variant measured no better (round 2)
  static bool attr = false;  // > 64 KiB dynamic LDS needs the opt-in once per process
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(srl::skinny::skinny_nt_kernel<false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(float) * 16 * (2048 + 4)));
    attr = true;
  }
  const dim3 grid(N / srl::skinny::WG_ROWS, p.splits, Z);
  hipLaunchKernelGGL(srl::skinny::skinny_nt_kernel<false>, grid, dim3(srl::skinny::NTH), lds, st, p);
  if (p.splits > 1)
    hipLaunchKernelGGL(srl::skinny::skinny_reduce_kernel, dim3((N / 4 + 63) / 64, M, Z), dim3(srl::skinny::NTH), 0, st, p);
}
