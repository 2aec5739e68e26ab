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
