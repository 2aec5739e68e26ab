// DreamerV3 return-normalisation Moments (reference: dreamer_v3/utils.py:16-41): the 5% / 95%
// percentiles of the lambda returns (torch.quantile, linear interpolation) feeding an EMA, as ONE
// single-workgroup launch instead of a full sort plus ~10 small kernels.
//
// Exact order statistics by radix select: every float maps to an order-preserving 32-bit key; four
// 8-bit passes narrow the four wanted ranks (floor / ceil of q_low * (n-1) and of q_high * (n-1))
// at once, each pass one sweep over the data building four 256-bin LDS histograms (lane-strided
// copies against same-bin atomic serialisation) and one parallel scan per rank to pick the bin.  The
// interpolation and the EMA use the reference's operation order (fp contraction off), so the result
// equals the sort-based path bit for bit.
#include "common.h"

namespace srl {
namespace moments {

constexpr int NTH = 1024;

__device__ __forceinline__ unsigned key_of(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float float_of(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

constexpr int COP = 8;  // lane-strided histogram copies: lanes that hit the same bin land on COP addresses

// ranks[0..3]: wanted 0-based order statistics.  low/high: EMA buffers (in place); inv: max(high - low, 1/max)
__global__ __launch_bounds__(NTH) void moments_kernel(const float* __restrict__ x, int n, int4 ranks, float frac_lo,
                                                      float frac_hi, float decay, float om, float inv_max, float* low, float* high,
                                                      float* inv) {
  // Lambda returns cluster in a few exponent bins, so a plain shared histogram serialises on one
  // address per pass; COP copies per bin (indexed by lane) spread those atomics.
  __shared__ unsigned hist[4][256 * COP];
  __shared__ unsigned wsum[NTH / 64];
  __shared__ unsigned prefix[4], remain[4];
  const int tid = threadIdx.x, lane = tid & 63, cop = tid & (COP - 1);
  const int j = tid >> 8, bin = tid & 255;  // scan role: rank j, bin b (4 x 256 = NTH threads)
  static_assert(NTH == 4 * 256, "one scan thread per (rank, bin)");
  if (tid < 4) {
    prefix[tid] = 0u;
    remain[tid] = (unsigned)(tid == 0 ? ranks.x : tid == 1 ? ranks.y : tid == 2 ? ranks.z : ranks.w);
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const unsigned mask = pass == 0 ? 0u : ~((1u << (shift + 8)) - 1u);  // bits already decided
    for (int i = tid; i < 4 * 256 * COP; i += NTH) (&hist[0][0])[i] = 0u;
    __syncthreads();
    const unsigned p0 = prefix[0], p1 = prefix[1], p2 = prefix[2], p3 = prefix[3];
    const unsigned r = remain[j];
    for (int i = tid; i < n; i += NTH) {
      const unsigned k = key_of(x[i]);
      const unsigned b = ((k >> shift) & 255u) * COP + cop, hk = k & mask;
      if (hk == p0) atomicAdd(&hist[0][b], 1u);
      if (hk == p1) atomicAdd(&hist[1][b], 1u);
      if (hk == p2) atomicAdd(&hist[2][b], 1u);
      if (hk == p3) atomicAdd(&hist[3][b], 1u);
    }
    __syncthreads();
    // bin totals, then an inclusive scan over the 256 bins of rank j (4 waves per rank)
    unsigned tot = 0u;
#pragma unroll
    for (int c = 0; c < COP; ++c) tot += hist[j][bin * COP + c];
    unsigned incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[tid >> 6] = incl;
    __syncthreads();
    for (int w = (j << 2); w < (tid >> 6); ++w) incl += wsum[w];
    const unsigned excl = incl - tot;
    if (excl <= r && r < incl) {  // exactly one bin per rank holds it
      prefix[j] |= (unsigned)bin << shift;
      remain[j] = r - excl;
    }
    __syncthreads();
  }
  if (tid == 0) {
#pragma clang fp contract(off)  // hipcc contracts a*b + c into an fma by default; the torch path rounds twice
    const float v0 = float_of(prefix[0]), v1 = float_of(prefix[1]), v2 = float_of(prefix[2]), v3 = float_of(prefix[3]);
    // quantile(): s[lo] + (s[hi] - s[lo]) * frac
    // plain operators under contract(off): the __f*_rn helpers are inlined from a header compiled
    // with contraction on, so they fuse into an fma anyway
    const float ql = v0 + (v1 - v0) * frac_lo;
    const float qh = v2 + (v3 - v2) * frac_hi;
    // low.mul_(decay).add_((1 - decay) * q); om = (float)(1 - decay) rounded from double on the host
    const float nl = *low * decay + om * ql;
    const float nh = *high * decay + om * qh;
    *low = nl;
    *high = nh;
    *inv = fmaxf(nh - nl, inv_max);
  }
}

}  // namespace moments
}  // namespace srl

void launch_moments(const float* x, int n, int r0, int r1, int r2, int r3, float frac_lo, float frac_hi, float decay,
                    float om, float inv_max, float* low, float* high, float* inv, hipStream_t st) {
  hipLaunchKernelGGL(srl::moments::moments_kernel, dim3(1), dim3(srl::moments::NTH), 0, st, x, n, make_int4(r0, r1, r2, r3),
                     frac_lo, frac_hi, decay, om, inv_max, low, high, inv);
}
