// Persistent single-layer LSTM over a whole sequence (recurrent PPO, reference
// ppo_recurrent/agent.py:60-73 nn.LSTM), forward and backward each ONE launch:
//
//   gates_t = xg_t + h_{t-1} W_hh^T        (xg = x W_ih^T + b_ih + b_hh, one library GEMM for all t)
//   i, f, o = sigmoid, g = tanh;  c_t = f c_{t-1} + i g;  h_t = o tanh(c_t)
//
// One workgroup per 16 batch rows keeps W_hh [4H, H] in LDS for all T steps; wave w owns hidden
// units [16w, 16w+16) and computes the four gate tiles of those units with v_mfma_f32_16x16x4_f32,
// so i, f, g, o of a unit land in the same lane and the cell state c stays in registers across the
// sequence.  h_t goes through a double-buffered LDS row block (one barrier per step).
// The backward walks t = T-1..0 with dh / dc in registers: the cell adjoint writes the pre-activation
// gate gradients (global, for the weight-gradient GEMMs after the launch, and LDS) and the recurrent
// adjoint dh_{t-1} = dgates_t W_hh is the same MFMA tiling over K = 4H.
#include "common.h"

namespace srl {
namespace lstm {

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct LP {
  const float* xg;   // [T, B, 4H]
  const float* Whh;  // [4H, H]
  const float* h0;   // [B, H]
  const float* c0;   // [B, H]
  float* out;        // [T, B, H]
  float* gates;      // [T, B, 4H] activated i, f, g, o
  float* cs;         // [T, B, H] cell states
  float* hT;         // [B, H]
  float* cT;         // [B, H]
  // backward
  const float* dout;  // [T, B, H]
  const float* dhT;   // [B, H] or null
  const float* dcT;   // [B, H] or null
  float* dgates;      // [T, B, 4H] pre-activation gradients
  float* dh0;         // [B, H]
  float* dc0;         // [B, H]
  int T, B, H;
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }

__global__ void lstm_fwd_kernel(LP p) {
  extern __shared__ float sm[];
  const int H = p.H, G = 4 * H, ldw = H + 4, ldh = H + 4;
  float* Ws = sm;                   // [4H][H+4]
  float* hs = Ws + G * ldw;         // [2][16][H+4]
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, w = tid >> 6;
  const int j = lane & 15, q = lane >> 4, u = 16 * w + j;
  const int r0 = blockIdx.x * 16;
  for (int i = tid; i < G * H; i += nth) Ws[(i / H) * ldw + i % H] = p.Whh[i];
  for (int i = tid; i < 16 * H; i += nth) {
    const int r = i / H, c = i % H;
    hs[r * ldh + c] = (r0 + r < p.B) ? p.h0[(size_t)(r0 + r) * H + c] : 0.f;
  }
  float c[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = r0 + 4 * q + e;
    c[e] = row < p.B ? p.c0[(size_t)row * H + u] : 0.f;
  }
  __syncthreads();
  for (int t = 0; t < p.T; ++t) {
    const float* hcur = hs + (t & 1) * 16 * ldh;
    float* hnxt = hs + ((t + 1) & 1) * 16 * ldh;
    floatx4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = r0 + 4 * q + e;
        acc[g][e] = row < p.B ? p.xg[((size_t)t * p.B + row) * G + g * H + u] : 0.f;
      }
    }
    for (int k0 = 0; k0 < H; k0 += 16) {
      const float4 a = *reinterpret_cast<const float4*>(hcur + j * ldh + k0 + 4 * q);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = *reinterpret_cast<const float4*>(Ws + (g * H + 16 * w + j) * ldw + k0 + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), comp(b, e), acc[g], 0, 0, 0);
      }
    }
    // D layout: lane holds rows 4q+e of column (unit) 16w + j for each gate tile
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rl = 4 * q + e, row = r0 + rl;
      const float ig = sigm(acc[0][e]), fg = sigm(acc[1][e]), gg = tanhf(acc[2][e]), og = sigm(acc[3][e]);
      c[e] = fg * c[e] + ig * gg;
      const float h = og * tanhf(c[e]);
      hnxt[rl * ldh + u] = h;
      if (row < p.B) {
        const size_t o = (size_t)t * p.B + row;
        p.out[o * H + u] = h;
        p.cs[o * H + u] = c[e];
        float* gp = p.gates + o * G;
        gp[u] = ig;
        gp[H + u] = fg;
        gp[2 * H + u] = gg;
        gp[3 * H + u] = og;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int rl = 4 * q + e, row = r0 + rl;
    if (row < p.B) {
      p.hT[(size_t)row * H + u] = hs[(p.T & 1) * 16 * ldh + rl * ldh + u];
      p.cT[(size_t)row * H + u] = c[e];
    }
  }
}

__global__ void lstm_bwd_kernel(LP p) {
  extern __shared__ float sm[];
  const int H = p.H, G = 4 * H, ldw = H + 4, ldg = G + 4;
  float* Ws = sm;               // [4H][H+4]
  float* dgs = Ws + G * ldw;    // [2][16][4H+4]
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, w = tid >> 6;
  const int j = lane & 15, q = lane >> 4, u = 16 * w + j;
  const int r0 = blockIdx.x * 16;
  for (int i = tid; i < G * H; i += nth) Ws[(i / H) * ldw + i % H] = p.Whh[i];
  float dh[4], dc[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = r0 + 4 * q + e;
    dh[e] = (row < p.B && p.dhT) ? p.dhT[(size_t)row * H + u] : 0.f;
    dc[e] = (row < p.B && p.dcT) ? p.dcT[(size_t)row * H + u] : 0.f;
  }
  __syncthreads();
  for (int t = p.T - 1; t >= 0; --t) {
    float* dg = dgs + (t & 1) * 16 * ldg;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rl = 4 * q + e, row = r0 + rl;
      float di = 0.f, df = 0.f, dgg = 0.f, dov = 0.f;
      if (row < p.B) {
        const size_t o = (size_t)t * p.B + row;
        const float* gp = p.gates + o * G;
        const float ig = gp[u], fg = gp[H + u], gg = gp[2 * H + u], og = gp[3 * H + u];
        const float c = p.cs[o * H + u];
        const float cp = t > 0 ? p.cs[(o - p.B) * H + u] : p.c0[(size_t)row * H + u];
        const float tc = tanhf(c);
        const float dht = p.dout[o * H + u] + dh[e];
        const float dct = dc[e] + dht * og * (1.f - tc * tc);
        dov = dht * tc * og * (1.f - og);
        di = dct * gg * ig * (1.f - ig);
        dgg = dct * ig * (1.f - gg * gg);
        df = dct * cp * fg * (1.f - fg);
        dc[e] = dct * fg;
        float* dgp = p.dgates + o * G;
        dgp[u] = di;
        dgp[H + u] = df;
        dgp[2 * H + u] = dgg;
        dgp[3 * H + u] = dov;
      }
      dg[rl * ldg + u] = di;
      dg[rl * ldg + H + u] = df;
      dg[rl * ldg + 2 * H + u] = dgg;
      dg[rl * ldg + 3 * H + u] = dov;
    }
    __syncthreads();
    // dh_{t-1}[rows, unit u] = sum_k dg[rows][k] W_hh[k][u]
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < G; k0 += 16) {
      const float4 a = *reinterpret_cast<const float4*>(dg + j * ldg + k0 + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a, e), Ws[(k0 + 4 * q + e) * ldw + u], acc, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) dh[e] = acc[e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = r0 + 4 * q + e;
    if (row < p.B) {
      p.dh0[(size_t)row * H + u] = dh[e];
      p.dc0[(size_t)row * H + u] = dc[e];
    }
  }
}

}  // namespace lstm
}  // namespace srl

static size_t lstm_lds(int H, bool bwd) {
  const int G = 4 * H;
  return sizeof(float) * ((size_t)G * (H + 4) + (bwd ? 2 * 16 * (size_t)(G + 4) : 2 * 16 * (size_t)(H + 4)));
}

static void lstm_attr() {
  static bool done = false;
  if (!done) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(srl::lstm::lstm_fwd_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lstm_lds(64, false));
    hipFuncSetAttribute(reinterpret_cast<const void*>(srl::lstm::lstm_bwd_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lstm_lds(64, true));
    done = true;
  }
}

void launch_lstm_fwd(const float* xg, const float* Whh, const float* h0, const float* c0, float* out, float* gates, float* cs,
                     float* hT, float* cT, int T, int B, int H, hipStream_t st) {
  srl::lstm::LP p{};
  p.xg = xg;
  p.Whh = Whh;
  p.h0 = h0;
  p.c0 = c0;
  p.out = out;
  p.gates = gates;
  p.cs = cs;
  p.hT = hT;
  p.cT = cT;
  p.T = T;
  p.B = B;
  p.H = H;
  lstm_attr();
  hipLaunchKernelGGL(srl::lstm::lstm_fwd_kernel, dim3((B + 15) / 16), dim3(64 * (H / 16)), lstm_lds(H, false), st, p);
}

void launch_lstm_bwd(const float* Whh, const float* c0, const float* gates, const float* cs, const float* dout, const float* dhT,
                     const float* dcT, float* dgates, float* dh0, float* dc0, int T, int B, int H, hipStream_t st) {
  srl::lstm::LP p{};
  p.Whh = Whh;
  p.c0 = c0;
  p.gates = const_cast<float*>(gates);  // read-only in the backward
  p.cs = const_cast<float*>(cs);
  p.dout = dout;
  p.dhT = dhT;
  p.dcT = dcT;
  p.dgates = dgates;
  p.dh0 = dh0;
  p.dc0 = dc0;
  p.T = T;
  p.B = B;
  p.H = H;
  lstm_attr();
  hipLaunchKernelGGL(srl::lstm::lstm_bwd_kernel, dim3((B + 15) / 16), dim3(64 * (H / 16)), lstm_lds(H, true), st, p);
}
