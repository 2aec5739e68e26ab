// DreamerV3 discrete-actor objective (reference: dreamer_v3/dreamer_v3.py:258-301):
//
//   adv[t,m]   = (lambda[t,m] - offset) / invscale - (baseline[t,m] - offset) / invscale
//   obj[t,m]   = sum_h log_softmax(z_h[t,m])[a_h[t,m]] * adv[t,m]
//   ent[t,m]   = ent_coef * sum_h H(softmax(z_h[t,m]))
//   loss       = -mean_{t < T-1, m} discount[t,m] * (obj[t,m] + ent[t,m])
//
// z = the unimix-mixed logits of every action head [T, M, A]; offset / invscale are the Moments
// scalars (device pointers, so the launch stays inside a captured graph).  The forward writes
// d loss / d z as well (the loss is linear in the upstream scalar gradient, the backward only scales
// it): d/dz_k of log_softmax[a] = a_k - p_k, of H = -p_k (log p_k + H).  One thread per (t, m) row;
// per-workgroup partial sums, then a fixed-order final reduction (deterministic).
#include "common.h"

#include <algorithm>

namespace srl {
namespace aloss {

constexpr int NTH = 256;
constexpr int MAXH = 8;

struct Heads {
  int n, size[MAXH];
};

__global__ __launch_bounds__(NTH) void actor_loss_kernel(const float* __restrict__ z, const float* __restrict__ act,
                                                         const float* __restrict__ lam, const float* __restrict__ base,
                                                         const float* __restrict__ disc, const float* __restrict__ offp,
                                                         const float* __restrict__ invp, Heads hd, int A, int T, int M,
                                                         float ent_coef, float* __restrict__ dz, float* __restrict__ partial) {
  __shared__ float red[NTH / 64];
  const int rows = T * M, last = (T - 1) * M;
  const float off = *offp, inv = *invp;
  const float scale = -1.f / (float)last;  // d loss / d (disc * (obj + ent)) per row
  float acc = 0.f;
  for (int r = blockIdx.x * NTH + threadIdx.x; r < rows; r += gridDim.x * NTH) {
    const float* zr = z + (size_t)r * A;
    const float* ar = act + (size_t)r * A;
    float* gr = dz + (size_t)r * A;
    if (r >= last) {  // the last imagined step enters neither the objective nor the entropy term
      for (int k = 0; k < A; ++k) gr[k] = 0.f;
      continue;
    }
    const float adv = (lam[r] - off) / inv - (base[r] - off) / inv;
    const float d = disc[r];
    float lp_sum = 0.f, h_sum = 0.f;
    int c0 = 0;
    for (int h = 0; h < hd.n; ++h) {
      const int C = hd.size[h];
      float mx = -INFINITY;
      for (int k = 0; k < C; ++k) mx = fmaxf(mx, zr[c0 + k]);
      float se = 0.f;
      for (int k = 0; k < C; ++k) se += __expf(zr[c0 + k] - mx);
      const float lse = mx + __logf(se);
      float lp = 0.f, H = 0.f;
      for (int k = 0; k < C; ++k) {
        const float l = zr[c0 + k] - lse, p = __expf(l);
        lp += ar[c0 + k] * l;
        H -= p * l;
      }
      lp_sum += lp;
      h_sum += H;
      // gradient of this row's term  scale * d * (lp * adv + ent_coef * H)
      const float ga = scale * d * adv, ge = scale * d * ent_coef;
      for (int k = 0; k < C; ++k) {
        const float l = zr[c0 + k] - lse, p = __expf(l);
        gr[c0 + k] = ga * (ar[c0 + k] - p) - ge * p * (l + H);
      }
      c0 += C;
    }
    acc += d * (lp_sum * adv + ent_coef * h_sum);
  }
  acc = block_sum<NTH / 64>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Continuous (truncated-normal) actor objective (reference dreamer_v3.py:258-301 with agent.py:685-700):
//
//   loc = tanh(p_mean), std = 2 sigmoid((p_std + init_std) / 2) + min_std             (the actor head transform)
//   H_k = log(sqrt(2 pi e)) + log Z - (b phi(b) - a phi(a)) / (2 Z) + log std,  a = (lo - loc) / std,
//         b = (hi - loc) / std, Z = max(Phi(b) - Phi(a), eps)                        (truncated-normal entropy)
//   loss = -mean_{t < T-1, m} disc[t,m] ((lam - off) / inv - (base - off) / inv + ent_coef sum_k H_k)
//
// One thread per (t, m) row; the gradients w.r.t. the head outputs (through the closed-form entropy derivative),
// the lambda returns and the baseline are written with the loss partials (unscaled: the backward multiplies by the
// upstream scalar).  Z's clamp passes no gradient where it is active, as torch's clamp_min.
__global__ __launch_bounds__(NTH) void actor_loss_cont_kernel(const float* __restrict__ pre, const float* __restrict__ lam,
                                                              const float* __restrict__ base, const float* __restrict__ disc,
                                                              const float* __restrict__ offp, const float* __restrict__ invp,
                                                              int A, int T, int M, float ent_coef, float init_std,
                                                              float min_std, float lo, float hi, float* __restrict__ dpre,
                                                              float* __restrict__ dlam, float* __restrict__ dbase,
                                                              float* __restrict__ partial) {
  __shared__ float red[NTH / 64];
  const int rows = T * M, last = (T - 1) * M;
  const float off = *offp, inv = *invp;
  const float scale = -1.f / (float)last;
  const float EPS = 1.1920928955078125e-07f, INV_SQRT2 = 0.70710678118654752f, INV_SQRT_2PI = 0.3989422804014327f;
  const float LOG_SQRT_2PI_E = 1.4189385332046727f;
  float acc = 0.f;
  for (int r = blockIdx.x * NTH + threadIdx.x; r < rows; r += gridDim.x * NTH) {
    const float* pr = pre + (size_t)r * 2 * A;
    float* gr = dpre + (size_t)r * 2 * A;
    if (r >= last) {  // the last imagined step enters neither the objective nor the entropy term
      for (int k = 0; k < 2 * A; ++k) gr[k] = 0.f;
      continue;
    }
    const float d = disc[r];
    const float adv = (lam[r] - off) / inv - (base[r] - off) / inv;
    dlam[r] = scale * d / inv;
    dbase[r] = -scale * d / inv;
    const float ge = scale * d * ent_coef;  // d loss / d H_k
    float hs = 0.f;
    for (int k = 0; k < A; ++k) {
      const float loc = tanhf(pr[k]);
      const float sg = 1.f / (1.f + expf(-0.5f * (pr[A + k] + init_std)));
      const float sd = 2.f * sg + min_std;
      const float a = (lo - loc) / sd, b = (hi - loc) / sd;
      const float pa = expf(-0.5f * a * a) * INV_SQRT_2PI, pb = expf(-0.5f * b * b) * INV_SQRT_2PI;
      const float zr = 0.5f * (1.f + erff(b * INV_SQRT2)) - 0.5f * (1.f + erff(a * INV_SQRT2));
      const bool clamped = zr < EPS;
      const float Z = clamped ? EPS : zr;
      const float N = b * pb - a * pa;
      hs += LOG_SQRT_2PI_E + logf(Z) - 0.5f * N / Z + logf(sd);
      // dH/da, dH/db (Z held constant where its clamp is active)
      const float dZa = clamped ? 0.f : -pa, dZb = clamped ? 0.f : pb;
      const float dNa = -pa * (1.f - a * a), dNb = pb * (1.f - b * b);
      const float dHa = dZa / Z - 0.5f * (dNa / Z - N * dZa / (Z * Z));
      const float dHb = dZb / Z - 0.5f * (dNb / Z - N * dZb / (Z * Z));
      const float dloc = -(dHa + dHb) / sd;
      const float dsd = -(a * dHa + b * dHb) / sd + 1.f / sd;
      gr[k] = ge * dloc * (1.f - loc * loc);
      gr[A + k] = ge * dsd * sg * (1.f - sg);
    }
    acc += d * (adv + ent_coef * hs);
  }
  acc = block_sum<NTH / 64>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// fixed-order tree over the block partials (lane-strided in index order, butterfly wave sum, 4 wave totals in order):
// bitwise reproducible, n/256 dependent adds per lane instead of n in one lane
__global__ void __launch_bounds__(256) actor_loss_final(const float* __restrict__ partial, int n, float scale,
                                                        float* __restrict__ loss) {
  __shared__ float wsum[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *loss = ((wsum[0] + wsum[1]) + (wsum[2] + wsum[3])) * scale;
}

// Imagined continuation flags and discounts (reference dreamer_v3.py:680-700): c_0 = 1 - done,
// c_t = [continue_logit_t > 0]; cont_g[t-1] = c_t * gamma (the lambda-return discount) and
// discount[t] = cumprod(c * gamma)[t] / gamma, one thread per imagined row, same fp32 operation
// order as the torch form (bitwise equal).
// clog holds rows t0 .. T1-1 of the continue logits (t0 = 1: row 0 - replaced by 1 - done - was never computed)
__global__ __launch_bounds__(256) void imag_discount_kernel(const float* __restrict__ clog, const float* __restrict__ dones,
                                                            int T1, int M, float gamma, float* __restrict__ cont_g,
                                                            float* __restrict__ discount, int t0) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const float inv = 1.f / gamma;  // torch divides by a scalar as a multiply by its fp32 reciprocal
  float acc = (1.f - dones[m]) * gamma;
  discount[m] = acc * inv;
  for (int t = 1; t < T1; ++t) {
    const float cg = (clog[(size_t)(t - t0) * M + m] > 0.f ? 1.f : 0.f) * gamma;
    cont_g[(size_t)(t - 1) * M + m] = cg;
    acc = acc * cg;
    discount[(size_t)t * M + m] = acc * inv;
  }
}

}  // namespace aloss
}  // namespace srl

void launch_imag_discount(const float* clog, const float* dones, int T1, int M, float gamma, float* cont_g, float* discount,
                          hipStream_t st, int t0) {
  hipLaunchKernelGGL(srl::aloss::imag_discount_kernel, dim3((M + 255) / 256), dim3(256), 0, st, clog, dones, T1, M, gamma,
                     cont_g, discount, t0);
}

int actor_loss_blocks(int rows) { return std::min(256, std::max(1, (rows + srl::aloss::NTH - 1) / srl::aloss::NTH)); }

void launch_actor_loss_cont(const float* pre, const float* lam, const float* base, const float* disc, const float* offp,
                            const float* invp, int A, int T, int M, float ent_coef, float init_std, float min_std, float lo,
                            float hi, float* dpre, float* dlam, float* dbase, float* partial, float* loss, hipStream_t st) {
  const int nb = actor_loss_blocks(T * M);
  hipLaunchKernelGGL(srl::aloss::actor_loss_cont_kernel, dim3(nb), dim3(srl::aloss::NTH), 0, st, pre, lam, base, disc, offp,
                     invp, A, T, M, ent_coef, init_std, min_std, lo, hi, dpre, dlam, dbase, partial);
  hipLaunchKernelGGL(srl::aloss::actor_loss_final, dim3(1), dim3(256), 0, st, partial, nb, -1.f / (float)((T - 1) * M), loss);
}

void launch_actor_loss(const float* z, const float* act, const float* lam, const float* base, const float* disc,
                       const float* offp, const float* invp, const int* heads, int nh, int A, int T, int M, float ent_coef,
                       float* dz, float* partial, float* loss, hipStream_t st) {
  srl::aloss::Heads hd{};
  hd.n = nh;
  for (int h = 0; h < nh; ++h) hd.size[h] = heads[h];
  const int nb = actor_loss_blocks(T * M);
  hipLaunchKernelGGL(srl::aloss::actor_loss_kernel, dim3(nb), dim3(srl::aloss::NTH), 0, st, z, act, lam, base, disc, offp,
                     invp, hd, A, T, M, ent_coef, dz, partial);
  hipLaunchKernelGGL(srl::aloss::actor_loss_final, dim3(1), dim3(256), 0, st, partial, nb, -1.f / (float)((T - 1) * M), loss);
}
