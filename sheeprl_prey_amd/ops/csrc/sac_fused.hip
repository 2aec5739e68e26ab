// Fused SAC update (reference sac/sac.py:34-78 `train`, sac/agent.py:53-152 actor, sac/agent.py:256-275 critics,
// sac/loss.py:10-26 losses).  One SAC gradient step is seven launches instead of ~110 (r4_trace_sac.md: 125
// dispatches per env step, 85 of them ATen elementwise / copy kernels):
//
//   tgt_kernel   next actions sampled from the actor in-kernel (MLP, heads, tanh-squashed Gaussian) and the
//                target ensemble's entropy-regularised Bellman target                          (row blocks)
//   critic fwd / critic wgrad (sac_critic.hip; the wgrad launch also sums the loss)
//   adam_multi   critic Adam with the step-count advance folded in + the target EMA           (one launch)
//   upd_kernel   actor forward + sample, every critic's Q(s, a) and dQ/da (one workgroup per row block and
//                critic), the last critic workgroup of a row block reduces min/mean over critics and runs the
//                policy-loss backward through the squashed Gaussian, the heads and both hidden layers
//   wg_kernel    actor weight gradients (fp32 MFMA over the batch), the alpha gradient, both losses, the
//                metric sums and the random-stream advance
//   adam_multi   actor + alpha Adam                                                          (one launch)
//
// The Gaussian noise is Philox-4x32-10 keyed by (seed, per-trainer device counter, element, stream salt): the
// launches have no per-step host arguments, so the whole update replays from one hipGraph.
// All activations stay in LDS; 16 batch rows per workgroup (the MFMA row tile), 8 waves, fp32 MFMA 16x16x4.
#include "common.h"
#include "sac_fused.h"
#include "sac_tiles.h"

namespace srl {
namespace sacf {

using namespace sactile;

constexpr int NTH = 512;
constexpr int NW = NTH / 64;
constexpr int ROWS = 16;
constexpr float HALF_LOG_2PI_F = 0.91893853320467274f;
constexpr unsigned SALT_PLAYER = 0x9E3779B1u, SALT_TARGET = 0x85EBCA77u, SALT_ACTOR = 0xC2B2AE3Du;

__device__ __forceinline__ uint4 philox10(uint4 c, unsigned k0, unsigned k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const unsigned hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// standard normal number `idx` of draw `ctr` of stream `salt` (Box-Muller on two 24-bit uniforms)
__device__ __forceinline__ float gauss(unsigned long long seed, unsigned long long ctr, unsigned idx, unsigned salt) {
  const uint4 r = philox10(make_uint4(idx, (unsigned)ctr, (unsigned)(ctr >> 32), salt), (unsigned)seed,
                           (unsigned)(seed >> 32));
  const float u1 = (float)((r.x >> 8) + 1u) * (1.f / 16777216.f);  // (0, 1]
  const float u2 = (float)(r.y >> 8) * (1.f / 16777216.f);         // [0, 1)
  return sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// phase timestamp i (s_memrealtime, 100 MHz) from thread 0 of a chosen workgroup: kernel-internal profiling
__device__ __forceinline__ void stamp(long long* ts, bool who, int i) {
  if (ts && who && threadIdx.x == 0) {
    long long c;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
    ts[i] = c;
  }
}

__device__ __forceinline__ int zp_dev(int A) { return (2 * A + 15) / 16 * 16; }
__device__ __forceinline__ int pad16(int v) { return (v + 15) / 16 * 16; }

// LDS views of one 16-row actor evaluation
struct ALds {
  float *h1, *h2;  // [16][ldh]
  float* z;        // [16][ldz]: mean | raw log-std (| zero padding)
  float *e, *y, *om, *lpe;  // [16][A]: noise, tanh(x), 1 - tanh^2(x), per-element log-prob terms
  float* lp;       // [16] row log-probs
  int ldh, ldz;
};

__device__ __forceinline__ float* carve(float* base, const ActorW& a, ALds& L) {
  L.ldh = a.H + 4;
  L.ldz = zp_dev(a.A) + 4;
  L.h1 = base;
  L.h2 = L.h1 + ROWS * L.ldh;
  L.z = L.h2 + ROWS * L.ldh;
  L.e = L.z + ROWS * L.ldz;
  L.y = L.e + ROWS * a.A;
  L.om = L.y + ROWS * a.A;
  L.lpe = L.om + ROWS * a.A;
  L.lp = L.lpe + ROWS * a.A;
  return L.lp + ROWS;
}

__host__ __device__ inline size_t actor_lds_floats(const ActorW& a) {
  return (size_t)2 * ROWS * (a.H + 4) + ROWS * ((2 * a.A + 15) / 16 * 16 + 4) + 4 * ROWS * a.A + ROWS;
}

// rows r0.. of src [M][OD] into xs [16][ldx], zero padded to `width` columns
__device__ __forceinline__ void load_rows(float* xs, int ldx, int width, const float* src, int OD, int r0, int M) {
  for (int i = threadIdx.x; i < ROWS * width; i += NTH) {
    const int r = i / width, k = i - r * width, row = r0 + r;
    xs[r * ldx + k] = (row < M && k < OD) ? src[(long)row * OD + k] : 0.f;
  }
}

// h1 = relu(x W1^T + b1), h2 = relu(h1 W2^T + b2), z = h2 [Wm; Ws]^T + [bm; bs] for the 16 rows in xs (columns < OD
// are read).  H1g / H2g: optional global copies of the hidden rows (the weight-gradient operands).
template <int FIRST = 2>  // wave_tiles form of the first layer (3 in kernels at their register limit)
__device__ void actor_fwd(const ActorW& a, const float* xs, int ldx, const ALds& L, float* H1g, float* H2g, int r0, int M) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, q = lane >> 4;
  const int H = a.H;
  wave_tiles<FIRST, NW>(xs, ldx, a.W1, a.OD, H, a.OD, lane, wave, [&](int n0, const floatx4& acc) {
    const float bb = a.b1[n0 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float h = fmaxf(acc[e] + bb, 0.f);
      L.h1[(4 * q + e) * L.ldh + n0 + j] = h;
      if (H1g && r0 + 4 * q + e < M) H1g[(long)(r0 + 4 * q + e) * H + n0 + j] = h;
    }
  });
  __syncthreads();
  wave_tiles<0, NW>(L.h1, L.ldh, a.W2, H, H, H, lane, wave, [&](int n0, const floatx4& acc) {
    const float bb = a.b2[n0 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float h = fmaxf(acc[e] + bb, 0.f);
      L.h2[(4 * q + e) * L.ldh + n0 + j] = h;
      if (H2g && r0 + 4 * q + e < M) H2g[(long)(r0 + 4 * q + e) * H + n0 + j] = h;
    }
  });
  __syncthreads();
  const int A = a.A, nz = zp_dev(A) / 16;
  for (int t = wave; t < nz; t += NW) {  // head tiles: columns [mean 0..A) | [log-std A..2A) | zero padding
    const int col = 16 * t + j;
    const float* wr = col < A ? a.Wm + (long)col * H : (col < 2 * A ? a.Ws + (long)(col - A) * H : nullptr);
    const floatx4 acc = tile_gemm_rows(L.h2, L.ldh, wr, H, lane);
    const float bb = col < A ? a.bm[col] : (col < 2 * A ? a.bs[col - A] : 0.f);
#pragma unroll
    for (int e = 0; e < 4; ++e) L.z[(4 * q + e) * L.ldz + col] = acc[e] + bb;
  }
  __syncthreads();
}

// tanh-squashed reparameterised sample (reference sac/agent.py:100-138): actions to dst[r * ldd + k], noise / tanh /
// log-prob terms to LDS, row log-probs to L.lp; optional global copies for rows < M.  1 - tanh^2(x) is evaluated
// as sech^2(x) = 4 t / (1 + t)^2, t = exp(-2|x|): no cancellation for saturated actions, where the reference's
// fp32 1 - y^2 loses every significant digit (the log-prob term then follows the fp64 value, not fp32 noise).
__device__ void actor_sample(const ActorW& a, const ALds& L, float* dst, int ldd, unsigned long long seed,
                             unsigned long long ctr, unsigned salt, int r0, int M, float* Ag, float* Lg, float* Eg) {
  const int tid = threadIdx.x, A = a.A;
  if (tid < ROWS * A) {
    const int r = tid / A, k = tid - r * A, row = r0 + r;
    const float ls = fminf(fmaxf(L.z[r * L.ldz + A + k], a.lo), a.hi);
    const float e = gauss(seed, ctr, (unsigned)(row * A + k), salt);
    const float s = a.scale[k];
    const float x = L.z[r * L.ldz + k] + expf(ls) * e;
    const float y = tanhf(x), t = expf(-2.f * fabsf(x)), om = 4.f * t / ((1.f + t) * (1.f + t));
    const float act = y * s + a.bias[k];
    L.e[tid] = e;
    L.y[tid] = y;
    L.om[tid] = om;
    L.lpe[tid] = -0.5f * e * e - ls - HALF_LOG_2PI_F - logf(s * om + 1e-6f);
    dst[r * ldd + k] = act;
    if (row < M) {
      if (Ag) Ag[(long)row * A + k] = act;
      if (Eg) Eg[(long)row * A + k] = e;
    }
  }
  __syncthreads();
  if (tid < ROWS) {
    float s = 0.f;
    for (int k = 0; k < A; ++k) s += L.lpe[tid * A + k];
    L.lp[tid] = s;
    if (Lg && r0 + tid < M) Lg[r0 + tid] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- player
__global__ __launch_bounds__(NTH) void act_kernel(ActP p) {
  extern __shared__ float sm[];
  const ActorW& a = p.a;
  const int ODp = pad16(a.OD), ldx = ODp + 4;
  float* xs = sm;
  ALds L;
  float* acts = carve(xs + ROWS * ldx, a, L);  // [16][A]
  const int r0 = blockIdx.x * ROWS;
  const unsigned long long ctr = *p.ctr;
  load_rows(xs, ldx, ODp, p.obs, a.OD, r0, p.M);
  __syncthreads();
  actor_fwd(a, xs, ldx, L, nullptr, nullptr, r0, p.M);
  actor_sample(a, L, acts, a.A, p.seed, ctr, SALT_PLAYER, r0, p.M, p.act, p.logp, p.eps);
  if (threadIdx.x == 0 && atomicAdd(p.ticket, 1) == (int)gridDim.x - 1) {  // every block has read the counter
    *p.ticket = 0;
    *p.ctr = ctr + 1;
  }
}

// ---------------------------------------------------------------- Bellman target
__global__ __launch_bounds__(NTH) void tgt_kernel(TgtP p) {
  extern __shared__ float sm[];
  const ActorW& a = p.a;
  const CriticW& c = p.c;
  const int IN = a.OD + a.A, INp = pad16(IN), ldx = INp + 4, ldc = c.H + 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, q = lane >> 4;
  float* xs = sm;  // [obs | next action | 0]
  ALds L;
  float* hc = carve(xs + ROWS * ldx, a, L);  // [16][ldc]
  float* qp = hc + ROWS * ldc;               // [NW][16]
  float* qmin = qp + NW * ROWS;              // [16]
  const int r0 = blockIdx.x * ROWS;
  const bool b0 = blockIdx.x == 0;
  stamp(p.ts, b0, 0);
  const unsigned long long ctr = *p.ctr;
  load_rows(xs, ldx, INp, p.obs, a.OD, r0, p.M);
  if (tid < ROWS) qmin[tid] = INFINITY;
  __syncthreads();
  stamp(p.ts, b0, 1);
  actor_fwd(a, xs, ldx, L, nullptr, nullptr, r0, p.M);
  stamp(p.ts, b0, 2);
  actor_sample(a, L, xs + a.OD, ldx, p.seed, ctr, SALT_TARGET, r0, p.M, p.act, p.logp, p.eps);
  stamp(p.ts, b0, 3);
  for (int ci = 0; ci < c.n; ++ci) {
    const float* W1 = c.W1 + (long)ci * c.H * IN;
    wave_tiles<2, NW>(xs, ldx, W1, IN, c.H, IN, lane, wave, [&](int n0, const floatx4& acc) {
      const float bb = c.b1[ci * c.H + n0 + j];
#pragma unroll
      for (int e = 0; e < 4; ++e) hc[(4 * q + e) * ldc + n0 + j] = fmaxf(acc[e] + bb, 0.f);
    });
    __syncthreads();
    stamp(p.ts, b0 && ci < 2, 4 + 2 * ci);
    const float* W2 = c.W2 + (long)ci * c.H * c.H;
    float part[4] = {0.f, 0.f, 0.f, 0.f};
    wave_tiles<0, NW>(hc, ldc, W2, c.H, c.H, c.H, lane, wave, [&](int n0, const floatx4& acc) {
      const float bb = c.b2[ci * c.H + n0 + j], w3 = c.W3[ci * c.H + n0 + j];
#pragma unroll
      for (int e = 0; e < 4; ++e) part[e] += fmaxf(acc[e] + bb, 0.f) * w3;
    });
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = part[e];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (j == 0) qp[wave * ROWS + 4 * q + e] = v;
    }
    __syncthreads();
    if (tid < ROWS) {
      float s = c.b3[ci];
      for (int w = 0; w < NW; ++w) s += qp[w * ROWS + tid];
      qmin[tid] = fminf(qmin[tid], s);
    }
    __syncthreads();
    stamp(p.ts, b0 && ci < 2, 5 + 2 * ci);
  }
  if (tid < ROWS && r0 + tid < p.M) {
    const int row = r0 + tid;
    const float alpha = expf(*p.log_alpha);
    p.y[row] = p.rew[row] + (1.f - p.done[row]) * p.gamma * (qmin[tid] - alpha * L.lp[tid]);
  }
  stamp(p.ts, b0, 8);
}

// ---------------------------------------------------------------- actor / alpha objective, forward + data backward
__global__ __launch_bounds__(NTH) void upd_kernel(UpdP p) {
  extern __shared__ float sm[];
  __shared__ int last;
  const ActorW& a = p.a;
  const CriticW& c = p.c;
  const int A = a.A, H = a.H, OD = a.OD, ODp = pad16(OD), IN = OD + A, INp = pad16(IN), ldx = INp + 4;
  const int ZP = zp_dev(A), Hc = c.H, ldc = Hc + 4, M = p.M, n = c.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, q = lane >> 4;
  float* xs = sm;  // [obs | action | 0]
  ALds L;
  float* h1c = carve(xs + ROWS * ldx, a, L);  // [16][ldc]  h1, then dh1 in place
  float* h2c = h1c + ROWS * ldc;              // [16][ldc]  h2, then dh2 in place
  float* qp = h2c + ROWS * ldc;               // [NW][16]
  float* qv = qp + NW * ROWS;                 // [16]
  float* qred = qv + ROWS;                    // [16]
  int* sel = reinterpret_cast<int*>(qred + ROWS);  // [16]
  const int rb = blockIdx.x, ci = blockIdx.y, r0 = rb * ROWS;
  const bool lead = ci == 0;  // writes the actor's weight-gradient operands
  const bool b0 = rb == 0 && ci == 0;
  stamp(p.ts, b0, 0);
  const unsigned long long ctr = *p.ctr;
  load_rows(xs, ldx, INp, p.obs, OD, r0, M);
  if (lead)
    for (int i = tid; i < ROWS * ODp; i += NTH) {
      const int r = i / ODp, k = i - r * ODp, row = r0 + r;
      if (row < M) p.Xa[(long)row * ODp + k] = k < OD ? p.obs[(long)row * OD + k] : 0.f;
    }
  __syncthreads();
  stamp(p.ts, b0, 1);
  actor_fwd<3>(a, xs, ldx, L, lead ? p.H1a : nullptr, lead ? p.H2a : nullptr, r0, M);
  stamp(p.ts, b0, 2);
  actor_sample(a, L, xs + OD, ldx, p.seed, ctr, SALT_ACTOR, r0, M, lead ? p.act : nullptr, lead ? p.logp : nullptr,
               lead ? p.eps : nullptr);

  // critic ci: q = w3 . relu(W2 relu(W1 [obs, a] + b1) + b2) + b3
  const float* W1 = c.W1 + (long)ci * Hc * IN;
  const float* W2 = c.W2 + (long)ci * Hc * Hc;
  const float* w3 = c.W3 + (long)ci * Hc;
  wave_tiles<3, NW>(xs, ldx, W1, IN, Hc, IN, lane, wave, [&](int n0, const floatx4& acc) {
    const float bb = c.b1[ci * Hc + n0 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e) h1c[(4 * q + e) * ldc + n0 + j] = fmaxf(acc[e] + bb, 0.f);
  });
  __syncthreads();
  stamp(p.ts, b0, 3);
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  wave_tiles<0, NW>(h1c, ldc, W2, Hc, Hc, Hc, lane, wave, [&](int n0, const floatx4& acc) {
    const float bb = c.b2[ci * Hc + n0 + j], wv = w3[n0 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float h = fmaxf(acc[e] + bb, 0.f);
      part[e] += h * wv;
      h2c[(4 * q + e) * ldc + n0 + j] = h;
    }
  });
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v = part[e];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (j == 0) qp[wave * ROWS + 4 * q + e] = v;
  }
  __syncthreads();
  if (tid < ROWS) {
    float s = c.b3[ci];
    for (int w = 0; w < NW; ++w) s += qp[w * ROWS + tid];
    qv[tid] = s;
  }
  stamp(p.ts, b0, 4);
  // dq/da with a unit output gradient: dh2 = w3 [h2 > 0] (in place), dh1 = (dh2 W2) [h1 > 0] (in place: each lane
  // masks and overwrites only its own output elements), da = dh1 W1[:, OD:OD+A]
  for (int i = tid; i < ROWS * Hc; i += NTH) {
    const int r = i / Hc, k = i - r * Hc;
    float* hp = h2c + r * ldc + k;
    *hp = *hp > 0.f ? w3[k] : 0.f;
  }
  __syncthreads();
  wave_tiles<1, NW>(h2c, ldc, W2, Hc, Hc, Hc, lane, wave, [&](int n0, const floatx4& acc) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* hp = h1c + (4 * q + e) * ldc + n0 + j;
      *hp = *hp > 0.f ? acc[e] : 0.f;
    }
  });
  __syncthreads();
  // hand-off to the row block's finishing workgroup: write-through stores, drained before the ticket
  const int na = (A + 15) / 16;
  for (int t = wave; t < na; t += NW) {
    const int nc = A - 16 * t < 16 ? A - 16 * t : 16;
    const floatx4 acc = tile_gemm_nn_cols(h1c, ldc, W1 + OD + 16 * t, IN, nc, Hc, lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 4 * q + e, col = 16 * t + j;
      if (row < M && col < A)
        __hip_atomic_store(p.DAX + ((long)ci * M + row) * A + col, acc[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (tid < ROWS && r0 + tid < M) {
    __hip_atomic_store(p.QX + (long)ci * M + r0 + tid, qv[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p.q) p.q[(long)(r0 + tid) * n + ci] = qv[tid];
  }
  stamp(p.ts, b0, 5);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) last = __hip_atomic_fetch_add(p.cnt + rb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1;
  __syncthreads();
  stamp(p.ts, b0, 6);
  if (!last) return;
  const bool bl = rb == 0;
  stamp(p.ts, bl, 7);
  if (tid == 0) __hip_atomic_store(p.cnt + rb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the hand-off reads are sc1

  // ---- finishing workgroup: reduce over critics (min: the first minimal critic takes the gradient, as torch.min)
  if (tid < ROWS) {
    const int row = r0 + tid;
    float qr = 0.f;
    int s = 0;
    if (row < M) {
      for (int cc = 0; cc < n; ++cc) {
        const float v = __hip_atomic_load(p.QX + (long)cc * M + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p.reduce_min) {
          if (cc == 0 || v < qr) qr = v, s = cc;
        } else {
          qr += v;
        }
      }
      if (!p.reduce_min) qr /= (float)n;
    }
    qred[tid] = qr;
    sel[tid] = s;
  }
  __syncthreads();
  // policy loss mean_b(alpha logp - q_red): dL/dlogp = alpha / M, dL/da = -dq_red/da / M; squashed-Gaussian backward
  // into the head pre-activations (mean | raw log-std), in place of z
  const float alpha = expf(*p.log_alpha), invM = 1.f / (float)M;
  if (tid < ROWS * A) {
    const int r = tid / A, k = tid - r * A, row = r0 + r;
    const bool ok = row < M;
    float ga = 0.f;
    if (ok) {
      if (p.reduce_min) {
        ga = __hip_atomic_load(p.DAX + ((long)sel[r] * M + row) * A + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (int cc = 0; cc < n; ++cc)
          ga += __hip_atomic_load(p.DAX + ((long)cc * M + row) * A + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ga /= (float)n;
      }
    }
    const float gact = ok ? -ga * invM : 0.f, glp = ok ? alpha * invM : 0.f;
    const float raw = L.z[r * L.ldz + A + k];
    const float ls = fminf(fmaxf(raw, a.lo), a.hi), dls = (raw >= a.lo && raw <= a.hi) ? 1.f : 0.f;
    const float e = L.e[tid], y = L.y[tid], s = a.scale[k], omy2 = L.om[tid];
    const float dy = gact * s + glp * (2.f * s * y / (s * omy2 + 1e-6f));
    const float dx = dy * omy2;
    L.z[r * L.ldz + k] = dx;
    L.z[r * L.ldz + A + k] = (dx * expf(ls) * e - glp) * dls;
  }
  for (int i = tid; i < ROWS * (ZP - 2 * A); i += NTH) {
    const int r = i / (ZP - 2 * A), col = 2 * A + i - r * (ZP - 2 * A);
    L.z[r * L.ldz + col] = 0.f;
  }
  __syncthreads();
  stamp(p.ts, bl, 8);
  for (int i = tid; i < ROWS * ZP; i += NTH) {
    const int r = i / ZP, col = i - r * ZP;
    if (r0 + r < M) p.DZ[(long)(r0 + r) * ZP + col] = L.z[r * L.ldz + col];
  }
  // dh2 = (dz_mean Wm + dz_logstd Ws) [h2 > 0], in place of h2
  for (int i = tid; i < ROWS * H; i += NTH) {
    const int r = i / H, h = i - r * H;
    float s = 0.f;
    for (int k = 0; k < A; ++k) s += L.z[r * L.ldz + k] * a.Wm[(long)k * H + h] + L.z[r * L.ldz + A + k] * a.Ws[(long)k * H + h];
    float* hp = L.h2 + r * L.ldh + h;
    const float v = *hp > 0.f ? s : 0.f;
    *hp = v;
    if (r0 + r < M) p.DH2a[(long)(r0 + r) * H + h] = v;
  }
  __syncthreads();
  stamp(p.ts, bl, 9);
  // dh1 = (dh2 W2) [h1 > 0]
  wave_tiles<1, NW>(L.h2, L.ldh, a.W2, H, H, H, lane, wave, [&](int n0, const floatx4& acc) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * q + e;
      if (r0 + r < M) p.DH1a[(long)(r0 + r) * H + n0 + j] = L.h1[r * L.ldh + n0 + j] > 0.f ? acc[e] : 0.f;
    }
  });
  if (wave == 0) {  // loss partials: sum_b (alpha logp - q_red), sum_b logp
    const bool ok = lane < ROWS && r0 + lane < M;
    float v1 = ok ? alpha * L.lp[lane] - qred[lane] : 0.f, v2 = ok ? L.lp[lane] : 0.f;
    v1 = wave_sum(v1);
    v2 = wave_sum(v2);
    if (lane == 0) {
      p.part[2 * rb] = v1;
      p.part[2 * rb + 1] = v2;
    }
  }
  stamp(p.ts, bl, 10);
}

// ---------------------------------------------------------------- actor weight gradients, alpha gradient, losses
__global__ __launch_bounds__(NTH) void wg_kernel(WgP p) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, q = lane >> 4;
  const int H = p.H, M = p.M, A = p.A, ZP = zp_dev(A), ODp = pad16(p.OD), nt = H / 16;
  const int nb2 = (nt * nt + NW - 1) / NW, nb1 = (nt * (ODp / 16) + NW - 1) / NW;
  const int nbh = ((ZP / 16) * nt + NW - 1) / NW, nbb = H / 64;
  int b = blockIdx.x;
  if (b < nb2) {  // dW2 = dh2^T h1
    const int tile = b * NW + wave;
    if (tile >= nt * nt) return;
    const int i0 = (tile / nt) * 16, j0 = (tile % nt) * 16;
    const floatx4 acc = tile_wgrad(p.DH2a, H, p.H1a, H, i0, j0, M, lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) p.dW2[(long)(i0 + 4 * q + e) * H + j0 + j] = acc[e];
    return;
  }
  b -= nb2;
  if (b < nb1) {  // dW1 = dh1^T obs
    const int nj = ODp / 16, tile = b * NW + wave;
    if (tile >= nt * nj) return;
    const int i0 = (tile / nj) * 16, j0 = (tile % nj) * 16;
    const floatx4 acc = tile_wgrad(p.DH1a, H, p.Xa, ODp, i0, j0, M, lane);
    if (j0 + j < p.OD) {
#pragma unroll
      for (int e = 0; e < 4; ++e) p.dW1[(long)(i0 + 4 * q + e) * p.OD + j0 + j] = acc[e];
    }
    return;
  }
  b -= nb1;
  if (b < nbh) {  // heads: [dWm; dWs] = dz^T h2
    const int tile = b * NW + wave;
    if (tile >= (ZP / 16) * nt) return;
    const int i0 = (tile / nt) * 16, j0 = (tile % nt) * 16;
    const floatx4 acc = tile_wgrad(p.DZ, ZP, p.H2a, H, i0, j0, M, lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = i0 + 4 * q + e;
      if (i < A) p.dWm[(long)i * H + j0 + j] = acc[e];
      else if (i < 2 * A) p.dWs[(long)(i - A) * H + j0 + j] = acc[e];
    }
    return;
  }
  b -= nbh;
  __shared__ float red[NW][2][64];
  if (b < nbb) {  // hidden biases: column sums of dh1 / dh2, rows split over waves
    const int k = b * 64 + lane;
    float s1 = 0.f, s2 = 0.f;
    for (int r = wave; r < M; r += NW) {
      s1 += p.DH1a[(long)r * H + k];
      s2 += p.DH2a[(long)r * H + k];
    }
    red[wave][0][lane] = s1;
    red[wave][1][lane] = s2;
    __syncthreads();
    if (wave == 0) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        t1 += red[w][0][lane];
        t2 += red[w][1][lane];
      }
      p.db1[k] = t1;
      p.db2[k] = t2;
    }
    return;
  }
  // last workgroup: head biases (ZP <= 64 columns, one per lane), losses, alpha gradient, metric sums, counter
  float s = 0.f;
  if (lane < ZP)
    for (int r = wave; r < M; r += NW) s += p.DZ[(long)r * ZP + lane];
  red[wave][0][lane] = s;
  __syncthreads();
  if (wave == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w][0][lane];
    if (lane < A) p.dbm[lane] = t;
    else if (lane < 2 * A) p.dbs[lane - A] = t;
  }
  if (wave == 1) {
    float s1 = 0.f, s2 = 0.f;
    for (int i = lane; i < p.nblk; i += 64) {
      s1 += p.part[2 * i];
      s2 += p.part[2 * i + 1];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      const float la = *p.log_alpha, te = *p.target_entropy;
      const float pl = s1 / (float)M, lm = s2 / (float)M;
      const float al = -la * (lm + te);  // entropy loss mean_b(-log_alpha (logp + target_entropy))
      p.losses[0] = pl;
      p.losses[1] = al;
      *p.dlog_alpha = -(lm + te);
      if (p.acc) {
        const float v[3] = {p.qf_loss ? *p.qf_loss : NAN, pl, al};
        for (int i = 0; i < 3; ++i)
          if (isfinite(v[i])) {
            p.acc[2 * i] += (double)v[i];
            p.acc[2 * i + 1] += 1.0;
          }
      }
      if (p.ctr) *p.ctr += 1ull;
    }
  }
}

// ---------------------------------------------------------------- multi-slab Adam (+ step advance, + target EMA)
struct AMP {
  AdamSlab s[MAX_SLABS];
  int blocks[MAX_SLABS];
  int ns;
  int* guard;
  int* tickets;
};

__global__ __launch_bounds__(256) void adam_multi_kernel(AMP p) {
  int b = blockIdx.x, si = 0;
  while (si + 1 < p.ns && b >= p.blocks[si]) b -= p.blocks[si++];
  AdamSlab s = p.s[0];
  int nbl = p.blocks[0];
#pragma unroll
  for (int k = 1; k < MAX_SLABS; ++k)
    if (k == si) s = p.s[k], nbl = p.blocks[k];
  // the step count advance of flat_advance folded in: every block reads the count, the slab's last block to finish
  // (ticket) stores it; a fault recorded earlier in the step (guard) skips the update, as adam_kernel does
  const bool trip = p.guard && (p.guard[0] | p.guard[1]) != 0;
  const float t = s.scalars[0] + 1.f;
  const float bc1 = 1.f - powf(s.b1, t), bc2s = sqrtf(1.f - powf(s.b2, t));
  const float step = s.lr / bc1, decay = s.decoupled ? 1.f - s.lr * s.wd : 1.f, l2 = s.decoupled ? 0.f : s.wd;
  const float ew = s.ema ? *s.ema_w : 0.f;
  float4* P = reinterpret_cast<float4*>(s.p);
  const float4* G = reinterpret_cast<const float4*>(s.g);
  float4* Mo = reinterpret_cast<float4*>(s.m);
  float4* V = reinterpret_cast<float4*>(s.v);
  float4* E = reinterpret_cast<float4*>(s.ema);
  const long long n4 = s.n / 4;
  for (long long i = (long long)b * 256 + threadIdx.x; i < n4; i += (long long)nbl * 256) {
    float4 pp = P[i];
    if (!trip) {
      float4 gg = G[i], mm = Mo[i], vv = V[i];
      float* pf = reinterpret_cast<float*>(&pp);
      float* gf = reinterpret_cast<float*>(&gg);
      float* mf = reinterpret_cast<float*>(&mm);
      float* vf = reinterpret_cast<float*>(&vv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gr = gf[k] + l2 * pf[k];
        const float w = pf[k] * decay;
        const float mk = mf[k] + (1.f - s.b1) * (gr - mf[k]);
        const float vk = vf[k] * s.b2 + (1.f - s.b2) * gr * gr;
        pf[k] = w - step * mk / (sqrtf(vk) / bc2s + s.eps);
        mf[k] = mk;
        vf[k] = vk;
      }
      P[i] = pp;
      Mo[i] = mm;
      V[i] = vv;
    }
    if (E) {
      float4 tg = E[i];
      tg.x += ew * (pp.x - tg.x);
      tg.y += ew * (pp.y - tg.y);
      tg.z += ew * (pp.z - tg.z);
      tg.w += ew * (pp.w - tg.w);
      E[i] = tg;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(p.tickets + si, 1) == nbl - 1) {
    p.tickets[si] = 0;
    if (trip) {
      s.scalars[3] = 1.f;
      atomicAdd(p.guard + 2, 1);
    } else {
      s.scalars[0] = t;
      s.scalars[1] = 1.f;
      s.scalars[3] = 0.f;
    }
  }
}

// ---------------------------------------------------------------- host side
int zp_of(int A) { return (2 * A + 15) / 16 * 16; }

size_t act_lds(const ActorW& a) {
  return sizeof(float) * ((size_t)ROWS * ((a.OD + 15) / 16 * 16 + 4) + actor_lds_floats(a) + (size_t)ROWS * a.A);
}

size_t tgt_lds(const ActorW& a, const CriticW& c) {
  const int INp = (a.OD + a.A + 15) / 16 * 16;
  return sizeof(float) * ((size_t)ROWS * (INp + 4) + actor_lds_floats(a) + (size_t)ROWS * (c.H + 4) + NW * ROWS + ROWS);
}

size_t upd_lds(const ActorW& a, const CriticW& c) {
  const int INp = (a.OD + a.A + 15) / 16 * 16;
  return sizeof(float) *
         ((size_t)ROWS * (INp + 4) + actor_lds_floats(a) + (size_t)2 * ROWS * (c.H + 4) + NW * ROWS + 3 * ROWS);
}

int upd_blocks(int M) { return (M + ROWS - 1) / ROWS; }

template <typename K>
static void big_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

void launch_act(const ActP& p, hipStream_t st) {
  const size_t lds = act_lds(p.a);
  big_lds(act_kernel, lds);
  hipLaunchKernelGGL(act_kernel, dim3(upd_blocks(p.M)), dim3(NTH), lds, st, p);
}

void launch_tgt(const TgtP& p, hipStream_t st) {
  const size_t lds = tgt_lds(p.a, p.c);
  big_lds(tgt_kernel, lds);
  hipLaunchKernelGGL(tgt_kernel, dim3(upd_blocks(p.M)), dim3(NTH), lds, st, p);
}

void launch_upd(const UpdP& p, hipStream_t st) {
  const size_t lds = upd_lds(p.a, p.c);
  big_lds(upd_kernel, lds);
  hipLaunchKernelGGL(upd_kernel, dim3(upd_blocks(p.M), p.c.n), dim3(NTH), lds, st, p);
}

void launch_wg(const WgP& p, hipStream_t st) {
  const int nt = p.H / 16, ODp = (p.OD + 15) / 16 * 16, ZP = zp_of(p.A);
  const int blocks = (nt * nt + NW - 1) / NW + (nt * (ODp / 16) + NW - 1) / NW + ((ZP / 16) * nt + NW - 1) / NW + p.H / 64 + 1;
  hipLaunchKernelGGL(wg_kernel, dim3(blocks), dim3(NTH), 0, st, p);
}

void launch_adam_multi(const AdamSlab* s, int ns, int* guard, int* tickets, hipStream_t st) {
  AMP p;
  int total = 0;
  for (int i = 0; i < MAX_SLABS; ++i) {
    p.s[i] = s[i < ns ? i : 0];
    const long long n4 = s[i < ns ? i : 0].n / 4;
    long long nb = (n4 + 255) / 256;
    nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
    p.blocks[i] = (int)nb;
    if (i < ns) total += (int)nb;
  }
  p.ns = ns;
  p.guard = guard;
  p.tickets = tickets;
  hipLaunchKernelGGL(adam_multi_kernel, dim3(total), dim3(256), 0, st, p);
}

}  // namespace sacf
}  // namespace srl
