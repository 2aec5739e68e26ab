// Small-batch CNN encoder (the env-interaction player: one frame per env, N < 64) - reference: the DreamerV3
// player's encoder call on every env step (dreamer_v3/agent.py:572-599 -> CNNEncoder, agent.py:48-80: k4 s2 p1
// convs, each followed by LayerNormChannelLast + SiLU, flattened in (C, H, W) order).
//
// The batched implicit-GEMM stack (conv.hip) tiles 64-256 output pixels per workgroup and walks the whole
// K = 16 Cin in one workgroup: at one 64x64 frame the deepest stage has 16 output pixels and K = 2048, i.e. one
// workgroup doing 17 MFLOP (~27 us at a CU's 256 f32 FLOP/clk).  Here every stage is split over K instead:
//
//  * pe_conv_kernel: workgroup = 16 output pixels x (16 x waves) output channels x one slice of input channels;
//    enough slices that the launch has >= ~256 workgroups.  Each wave owns one 16 x 16 tile: per input channel
//    four v_mfma_f32_16x16x4f32 with A[i = pixel][k] read straight from the NCHW input (lane (i, g) reads the
//    4 contiguous input pixels of kernel row g: one float2 + two edge floats, the padding handled by masks fixed
//    per lane, so every load is unconditional) and B[k][j] = W[co0 + j][16 ci + 4 g + e] as one float4.
//    Partials go to part[slice][pixel][co].
//  * pe_ln_kernel: one wave per output pixel sums the slices, LayerNorm over the channels (DPP wave sums) +
//    activation, written as NCHW (the next stage's input and the flatten order of the last one).
#include "common.h"

namespace srl {
namespace pe {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int PE_KS_MAX = 16;  // K slices per stage (the slice-sum loads of pe_ln_kernel are unrolled over them)

struct CP {
  const void* x;  // [N, Cin, Hi, Wi] float, or uint8 (first stage of raw frames; scaled by `scale`)
  const float* w;  // [Cout, Cin, 4, 4]
  float* part;     // [KS, M, Cout]
  int N, Cin, Hi, Wi, Cout, Ho, Wo, M, KS, cper;
  float scale;
};

template <bool U8>
__device__ __forceinline__ float4 ld4(const CP& p, long b, float ml, float mr, float mrow) {
  // input pixels b-1 .. b+2 of one row (b even); ml / mr: the edge pixels exist; mrow: the row exists
  if (U8) {
    const unsigned char* x = static_cast<const unsigned char*>(p.x);
    const float s = p.scale * mrow;
    return make_float4(ml * s * (float)x[b - 1 + (ml == 0.f)], s * (float)x[b], s * (float)x[b + 1],
                       mr * s * (float)x[b + 2 - 2 * (mr == 0.f)]);
  } else {
    const float* x = static_cast<const float*>(p.x);
    const float2 c = *reinterpret_cast<const float2*>(x + b);
    const float s = p.scale * mrow;
    return make_float4(ml * s * x[b - 1 + (ml == 0.f)], s * c.x, s * c.y, mr * s * x[b + 2 - 2 * (mr == 0.f)]);
  }
}

template <bool U8>
__global__ void __launch_bounds__(256) pe_conv_kernel(CP p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 16;
  const int co0 = (blockIdx.y * (blockDim.x >> 6) + wave) * 16;
  if (co0 >= p.Cout) return;  // whole wave; no barrier in this kernel
  const int ks = blockIdx.z;
  const int c0 = ks * p.cper, c1 = min(p.Cin, c0 + p.cper);
  // this lane's A pixel (clamped when past M: its rows are never stored) and kernel row g
  const int m = min(m0 + i, p.M - 1);
  const int HoWo = p.Ho * p.Wo;
  const int n = m / HoWo, rem = m - n * HoWo, oy = rem / p.Wo, ox = rem - oy * p.Wo;
  const int iy = 2 * oy - 1 + g;
  const float mrow = (iy >= 0 && iy < p.Hi) ? 1.f : 0.f;
  const float ml = ox > 0 ? 1.f : 0.f, mr = ox < p.Wo - 1 ? 1.f : 0.f;
  const long plane = (long)p.Hi * p.Wi;
  long b = (long)n * p.Cin * plane + (long)min(max(iy, 0), p.Hi - 1) * p.Wi + 2 * ox;
  b += (long)c0 * plane;
  const int K = 16 * p.Cin;
  const float4* wr = reinterpret_cast<const float4*>(p.w + (long)(co0 + i) * K + 16 * c0 + 4 * g);
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  int c = c0;
#pragma unroll 4
  for (; c + 1 < c1; c += 2) {  // two independent accumulator chains (40-cycle dependent MFMA latency)
    const float4 a0 = ld4<U8>(p, b, ml, mr, mrow), a1 = ld4<U8>(p, b + plane, ml, mr, mrow);
    const float4 w0 = wr[0], w1 = wr[4];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, w0.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, w1.x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, w0.y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, w1.y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, w0.z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, w1.z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, w0.w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, w1.w, acc1, 0, 0, 0);
    b += 2 * plane;
    wr += 8;
  }
  if (c < c1) {
    const float4 a0 = ld4<U8>(p, b, ml, mr, mrow);
    const float4 w0 = wr[0];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, w0.x, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, w0.y, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, w0.z, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, w0.w, acc0, 0, 0, 0);
  }
  // C/D: lane (i, g) holds pixel m0 + 4 g + r, channel co0 + i
  float* out = p.part + (long)ks * p.M * p.Cout + co0 + i;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mm = m0 + 4 * g + r;
    if (mm < p.M) out[(long)mm * p.Cout] = acc0[r] + acc1[r];
  }
}

// one wave per output pixel: sum of the KS slices, LayerNorm over Cout (<= 64 * 16) + activation -> NCHW
template <int CV>
__global__ void __launch_bounds__(256) pe_ln_kernel(const float* __restrict__ part, int KS, int M, int Cout, int HoWo,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float eps, int act, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float v[CV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CV; ++j) {
    const int co = lane + 64 * j;
    // every slice's load in flight at once (KS <= PE_KS_MAX; a sequential loop here was one round trip per
    // slice: 75 us at 64 slices)
    const float* pp = part + (long)m * Cout + min(co, Cout - 1);
    float t[PE_KS_MAX];
#pragma unroll
    for (int k = 0; k < PE_KS_MAX; ++k) t[k] = pp[(long)min(k, KS - 1) * M * Cout];
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < PE_KS_MAX; ++k) a += k < KS ? t[k] : 0.f;
    if (co >= Cout) a = 0.f;
    v[j] = a;
    s += a;
  }
  const float mu = wave_sum_dpp(s) / Cout;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CV; ++j)
    if (lane + 64 * j < Cout) q += (v[j] - mu) * (v[j] - mu);
  const float rs = rsqrtf(wave_sum_dpp(q) / Cout + eps);
  const int n = m / HoWo, pix = m - n * HoWo;
  float* yo = y + (long)n * Cout * HoWo + pix;
#pragma unroll
  for (int j = 0; j < CV; ++j) {
    const int co = lane + 64 * j;
    if (co < Cout) yo[(long)co * HoWo] = act_fwd((v[j] - mu) * rs * gamma[co] + beta[co], act);
  }
}

}  // namespace pe
}  // namespace srl

using namespace srl;

// workgroups per stage the K split aims for (a 256-CU chip)
static int pe_slices(int M, int Cout, int Cin) {
  const int waves = min(4, Cout / 16);
  const int blocks = cdiv(M, 16) * cdiv(Cout, 16 * waves);
  int ks = cdiv(256, blocks);
  if (ks > pe::PE_KS_MAX) ks = pe::PE_KS_MAX;
  if (ks > Cin) ks = Cin;
  if (ks < 1) ks = 1;
  const int cper = cdiv(Cin, ks);
  return cdiv(Cin, cper);
}

int small_conv_slices(int M, int Cout, int Cin) { return pe_slices(M, Cout, Cin); }

// false: unsupported (Cout % 16, Cout > 1024, odd input size)
bool launch_small_conv_stage(const void* x, bool u8, float scale, const float* w, const float* gamma, const float* beta,
                             float eps, int act, float* part, float* y, int N, int Cin, int Hi, int Wi, int Cout,
                             hipStream_t st) {
  if ((Cout & 15) || Cout > 1024 || (Hi & 1) || (Wi & 1) || Hi < 2 || Wi < 2 || ((uintptr_t)w & 15) ||
      (!u8 && ((uintptr_t)x & 7)))
    return false;
  pe::CP p;
  p.x = x;
  p.w = w;
  p.part = part;
  p.N = N;
  p.Cin = Cin;
  p.Hi = Hi;
  p.Wi = Wi;
  p.Cout = Cout;
  p.Ho = Hi / 2;
  p.Wo = Wi / 2;
  p.M = N * p.Ho * p.Wo;
  p.KS = pe_slices(p.M, Cout, Cin);
  p.cper = cdiv(Cin, p.KS);
  p.scale = scale;
  const int waves = min(4, Cout / 16);
  const dim3 grid(cdiv(p.M, 16), cdiv(Cout, 16 * waves), p.KS);
  if (u8)
    hipLaunchKernelGGL(pe::pe_conv_kernel<true>, grid, dim3(64 * waves), 0, st, p);
  else
    hipLaunchKernelGGL(pe::pe_conv_kernel<false>, grid, dim3(64 * waves), 0, st, p);
  const int cv = cdiv(Cout, 64);
  const dim3 lg(cdiv(p.M, 4));
  const int HoWo = p.Ho * p.Wo;
#define PE_LN(CVN) hipLaunchKernelGGL(pe::pe_ln_kernel<CVN>, lg, dim3(256), 0, st, part, p.KS, p.M, Cout, HoWo, gamma, beta, eps, act, y)
  if (cv <= 1)
    PE_LN(1);
  else if (cv <= 2)
    PE_LN(2);
  else if (cv <= 4)
    PE_LN(4);
  else if (cv <= 8)
    PE_LN(8);
  else
    PE_LN(16);
#undef PE_LN
  return true;
}
