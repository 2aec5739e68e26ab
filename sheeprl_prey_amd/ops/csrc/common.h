// Shared helpers for the CDNA4 (gfx950) kernels of sheeprl_prey_amd.
// Wave64 everywhere: reductions use 64-lane xor shuffles, blocks are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SRL_WAVE 64

namespace srl {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, SRL_WAVE);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, SRL_WAVE));
  return v;
}

// Reduction inside aligned segments of `width` lanes (width = power of two <= 64).
__device__ __forceinline__ float seg_sum(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, SRL_WAVE);
  return v;
}
__device__ __forceinline__ float seg_max(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, SRL_WAVE));
  return v;
}

// ---------------------------------------------------------------- DPP reductions
// Cross-lane reductions on latency-critical paths (persistent scan, samplers), without the LDS crossbar: __shfl_xor
// lowers to ds_bpermute_b32 (an LDS-pipe round trip per level, 6 dependent ones per 64-lane sum); these use
// DPP row ops (quad butterflies, row rotations / shifts / broadcasts: plain VALU operand modifiers) and
// v_readlane for the cross-row step.  Summation order differs from the butterfly: fp32 rounding only.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// every lane of each 16-lane row gets the row's sum / max
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x128>(v));
  return v;
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = row16_sum(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
// segments of 32 lanes (lanes 0-31, 32-63): every lane gets its segment's sum / max
__device__ __forceinline__ float seg32_sum(float v) {
  v = row16_sum(v);
  const float a = lane_f(v, 0) + lane_f(v, 16), b = lane_f(v, 32) + lane_f(v, 48);
  return (threadIdx.x & 32) ? b : a;
}
__device__ __forceinline__ float seg32_max(float v) {
  v = row16_max(v);
  const float a = fmaxf(lane_f(v, 0), lane_f(v, 16)), b = fmaxf(lane_f(v, 32), lane_f(v, 48));
  return (threadIdx.x & 32) ? b : a;
}
// inclusive prefix sum inside each 32-lane segment (Hillis-Steele row shifts, then row 1 / 3 add row 0 / 2's total)
__device__ __forceinline__ float seg32_scan(float v) {
  v += dpp_f<0x111>(v);       // row_shr:1
  v += dpp_f<0x112>(v);       // row_shr:2
  v += dpp_f<0x114>(v);       // row_shr:4
  v += dpp_f<0x118>(v);       // row_shr:8
  v += dpp_f<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  return v;
}
// inclusive prefix sum inside each 16-lane row
__device__ __forceinline__ float row16_scan(float v) {
  v += dpp_f<0x111>(v);
  v += dpp_f<0x112>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  return v;
}
// width-generic forms: DPP for the widths above, the xor-shuffle butterfly otherwise
__device__ __forceinline__ float seg_sum_f(float v, int width) {
  if (width == 32) return seg32_sum(v);
  if (width == 16) return row16_sum(v);
  if (width == 64) return wave_sum_dpp(v);
  return seg_sum(v, width);
}
__device__ __forceinline__ float seg_max_f(float v, int width) {
  if (width == 32) return seg32_max(v);
  if (width == 16) return row16_max(v);
  return seg_max(v, width);
}

// Block-wide sum for blockDim.x = 64 * NW. `red` must hold NW floats (LDS).
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (NW == 1) return v;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------- activations
enum Act : int { ACT_NONE = 0, ACT_SILU = 1, ACT_ELU = 2, ACT_RELU = 3, ACT_TANH = 4 };

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ float act_fwd(float z, int act) {
  switch (act) {
    case ACT_SILU: return z * sigmoidf_(z);
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_TANH: return tanhf(z);
    default: return z;
  }
}

// d act / d z evaluated at z
__device__ __forceinline__ float act_grad(float z, int act) {
  switch (act) {
    case ACT_SILU: {
      float s = sigmoidf_(z);
      return s * (1.f + z * (1.f - s));
    }
    case ACT_ELU: return z > 0.f ? 1.f : __expf(z);
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_TANH: {
      float t = tanhf(z);
      return 1.f - t * t;
    }
    default: return 1.f;
  }
}

// Activation with a compile-time code (ACTC >= 0) or the runtime code `act` (ACTC < 0).  Hot loops branch
// ONCE on the (wave-uniform) runtime code and instantiate the SiLU body on its own (SRL_ACT_SPECIALIZE): a
// runtime switch inside an unrolled per-element loop is if-converted into selects that evaluate every
// activation's transcendentals for every element (5 v_exp/v_rcp per element where SiLU needs 2; measured in
// the persistent scan's LayerNorm prologues: ~850 instructions for an 8-element row chunk).
template <int ACTC>
__device__ __forceinline__ float act_fwd_c(float z, int act) {
  if constexpr (ACTC == ACT_SILU) return z * sigmoidf_(z);
  else if constexpr (ACTC == ACT_NONE) return z;
  else return act_fwd(z, act);
}
template <int ACTC>
__device__ __forceinline__ float act_grad_c(float z, int act) {
  if constexpr (ACTC == ACT_SILU) {
    const float s = sigmoidf_(z);
    return s * (1.f + z * (1.f - s));
  } else if constexpr (ACTC == ACT_NONE) {
    return 1.f;
  } else {
    return act_grad(z, act);
  }
}
// Runs the statement(s) with `constexpr int ACTC` = ACT_SILU when act is SiLU, -1 (runtime switch) otherwise.
#define SRL_ACT_SPECIALIZE(act, ...)      \
  do {                                    \
    if ((act) == ACT_SILU) {              \
      constexpr int ACTC = ACT_SILU;      \
      __VA_ARGS__;                        \
    } else {                              \
      constexpr int ACTC = -1;            \
      __VA_ARGS__;                        \
    }                                     \
  } while (0)

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace srl
