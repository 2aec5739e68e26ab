// One-launch PPO rollout for MLP policies on the device CartPole (reference loop: ppo/ppo.py:281-356,
// policy head ppo/agent.py:134-178, env gymnasium CartPole-v1 + TimeLimit + autoreset).
//
// Every environment is independent over the rollout and the weights are constant during it, so ONE
// WAVE per env runs all T steps back to back with no grid- or block-wide synchronisation.  The
// rollout is a chain of T dependent policy evaluations, i.e. latency-bound, so the design minimises
// the per-step critical path:
//   * all MLP weights are staged ONCE per launch into LDS, transposed to [din, dout]: lane j reads
//     W^T[k][j] (consecutive lanes -> consecutive banks, conflict-free) while the input x[k] is a
//     broadcast float4 read; 4 independent accumulators hide the FMA latency;
//   * layer boundaries are wave-local barriers (no s_barrier across waves), the env step and the
//     Gumbel-max categorical sample run on lane 0, scalars are broadcast with readfirstlane;
//   * up to RO_ENVS_PER_BLOCK envs (waves) share one staged copy of the weights.
// Per step: encoder / actor / head / critic chains, sample + log-prob, the CartPole step with
// autoreset, the truncation bootstrap r += V(final_obs) and the [T, N] rollout-buffer writes.
// This replaces ~50 kernel launches per env step (~6k per rollout) with one launch.
#include "common.h"
#include "ppo_rollout.h"

namespace srl {

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float ro_act(float z, int act) {
  switch (act) {
    case ACT_TANH: return tanhf(z);
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_SILU: return z / (1.f + __expf(-z));
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    default: return z;
  }
}

// counter-based uniform in (0, 1): splitmix64 of (seed, stream id)
__device__ __forceinline__ float ro_uniform(uint64_t seed, uint64_t id) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (id + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// y = chain(x) for one env, evaluated by one wave; x is not overwritten; returns the buffer (a or b)
// holding the result.  LW: weights staged in LDS (transposed) vs read from global (row-major).
template <bool LW>
__device__ const float* wave_chain(const Chain& c, const float* __restrict__ sw, const float* x, float* a, float* b,
                                   int lane) {
  const float* in = x;
  float* out = a;
  for (int l = 0; l < c.n; ++l) {
    const int din = c.din[l], dout = c.dout[l], act = c.act[l];
    for (int j = lane; j < dout; j += 64) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      int k = 0;
      if (LW) {
        const float* wt = sw + c.woff[l] + j;
        if ((din & 3) == 0) {
          for (; k < din; k += 4) {
            const float4 xv = *reinterpret_cast<const float4*>(in + k);
            s0 = fmaf(wt[(k + 0) * dout], xv.x, s0);
            s1 = fmaf(wt[(k + 1) * dout], xv.y, s1);
            s2 = fmaf(wt[(k + 2) * dout], xv.z, s2);
            s3 = fmaf(wt[(k + 3) * dout], xv.w, s3);
          }
        }
        for (; k < din; ++k) s0 = fmaf(wt[k * dout], in[k], s0);
        s0 += sw[c.boff[l] + j];
      } else {
        const float* w = c.W[l] + (size_t)j * din;
        for (; k + 4 <= din; k += 4) {
          s0 = fmaf(w[k], in[k], s0);
          s1 = fmaf(w[k + 1], in[k + 1], s1);
          s2 = fmaf(w[k + 2], in[k + 2], s2);
          s3 = fmaf(w[k + 3], in[k + 3], s3);
        }
        for (; k < din; ++k) s0 = fmaf(w[k], in[k], s0);
        if (c.b[l]) s0 += c.b[l][j];
      }
      out[j] = ro_act((s0 + s1) + (s2 + s3), act);
    }
    wave_lds_sync();
    in = out;
    out = (out == a) ? b : a;
  }
  return in;
}

__device__ void stage_chain(const Chain& c, float* sw) {
  for (int l = 0; l < c.n; ++l) {
    const int din = c.din[l], dout = c.dout[l];
    const float* W = c.W[l];
    for (int i = threadIdx.x; i < din * dout; i += blockDim.x) {
      const int j = i / din, k = i - j * din;
      sw[c.woff[l] + k * dout + j] = W[i];
    }
    for (int j = threadIdx.x; j < dout; j += blockDim.x) sw[c.boff[l] + j] = c.b[l] ? c.b[l][j] : 0.f;
  }
}

// per-wave scratch (floats): obs 4 | fin 4 | logits 8 | feat 256 | a 256 | b 256 | c 256
constexpr int RO_SCR = 16 + 4 * RO_MAXW;

template <bool LW>
__global__ void __launch_bounds__(64 * RO_ENVS_PER_BLOCK) ppo_cartpole_rollout_kernel(RolloutArgs p) {
  __shared__ __attribute__((aligned(16))) float s_w[LW ? RO_LDSW : 4];
  __shared__ __attribute__((aligned(16))) float s_scr[RO_ENVS_PER_BLOCK][RO_SCR];
  if (LW) {
    stage_chain(p.enc, s_w);
    stage_chain(p.actor, s_w);
    stage_chain(p.head, s_w);
    stage_chain(p.critic, s_w);
    __syncthreads();  // the only block-wide barrier: from here on every wave (env) runs on its own
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * RO_ENVS_PER_BLOCK + wave;
  if (n >= p.N) return;
  float* scr = s_scr[wave];
  float *s_obs = scr, *s_fin = scr + 4, *s_logit = scr + 8, *s_feat = scr + 16;
  float *s_a = s_feat + RO_MAXW, *s_b = s_a + RO_MAXW, *s_c = s_b + RO_MAXW;
  const float gravity = 9.8f, masscart = 1.0f, masspole = 0.1f, total_mass = masspole + masscart, length = 0.5f;
  const float pml = masspole * length, force_mag = 10.0f, tau = 0.02f;
  const float theta_thr = 12.f * 2.f * 3.14159265358979323846f / 360.f, x_thr = 2.4f;
  const int F = p.enc.dout[p.enc.n - 1];
  if (lane < 4) s_obs[lane] = p.state[4 * n + lane];
  int steps = p.steps[n];
  float ep_ret = p.ep_ret[n];
  wave_lds_sync();
  for (int t = 0; t < p.T; ++t) {
    const size_t tn = (size_t)t * p.N + n;
    if (lane < 4) p.b_state[4 * tn + lane] = s_obs[lane];
    // policy: features -> (actor -> head logits), (critic -> value)
    const float* f = wave_chain<LW>(p.enc, s_w, s_obs, s_a, s_b, lane);
    for (int j = lane; j < F; j += 64) s_feat[j] = f[j];
    wave_lds_sync();
    const float* h = wave_chain<LW>(p.actor, s_w, s_feat, s_a, s_b, lane);
    const float* lg = wave_chain<LW>(p.head, s_w, h, h == s_a ? s_b : s_a, s_c, lane);
    if (lane < p.A) s_logit[lane] = lg[lane];
    wave_lds_sync();
    const float value = wave_chain<LW>(p.critic, s_w, s_feat, s_a, s_b, lane)[0];
    int trunc_flag = 0;
    if (lane == 0) {
      // Gumbel-max sample and log-prob of a categorical over A logits
      float mx = -INFINITY;
      for (int a = 0; a < p.A; ++a) mx = fmaxf(mx, s_logit[a]);
      float se = 0.f;
      for (int a = 0; a < p.A; ++a) se += __expf(s_logit[a] - mx);
      const float lse = mx + __logf(se);
      int pick = 0;
      float best = -INFINITY;
      for (int a = 0; a < p.A; ++a) {
        const float u = ro_uniform(p.seed, ((uint64_t)tn << 8) + a);
        const float g = s_logit[a] - __logf(-__logf(u));
        if (g > best) {
          best = g;
          pick = a;
        }
      }
      for (int a = 0; a < p.A; ++a) p.b_actions[tn * p.A + a] = a == pick ? 1.f : 0.f;
      p.b_logp[tn] = s_logit[pick] - lse;
      p.b_values[tn] = value;
      // CartPole-v1 step (dynamics of envs/classic.py) with autoreset
      float x = s_obs[0], x_dot = s_obs[1], th = s_obs[2], th_dot = s_obs[3];
      const float force = pick == 1 ? force_mag : -force_mag;
      const float c = cosf(th), s = sinf(th);
      const float temp = (force + pml * th_dot * th_dot * s) / total_mass;
      const float thacc = (gravity * s - c * temp) / (length * (4.f / 3.f - masspole * c * c / total_mass));
      const float xacc = temp - pml * thacc * c / total_mass;
      x += tau * x_dot;
      x_dot += tau * xacc;
      th += tau * th_dot;
      th_dot += tau * thacc;
      const bool term = x < -x_thr || x > x_thr || th < -theta_thr || th > theta_thr;
      steps += 1;
      const bool trunc = !term && steps >= p.max_steps;
      ep_ret += 1.f;
      s_fin[0] = x;
      s_fin[1] = x_dot;
      s_fin[2] = th;
      s_fin[3] = th_dot;
      p.b_dones[tn] = (term || trunc) ? 1.f : 0.f;
      p.b_rewards[tn] = 1.f;
      if (term || trunc) {
        p.b_done_ret[tn] = ep_ret;
        p.b_done_len[tn] = (float)steps;
        for (int k = 0; k < 4; ++k) s_obs[k] = ro_uniform(p.seed, ((uint64_t)tn << 8) + 128 + k) * 0.1f - 0.05f;
        steps = 0;
        ep_ret = 0.f;
      } else {
        p.b_done_ret[tn] = 0.f;
        p.b_done_len[tn] = 0.f;
        s_obs[0] = x;
        s_obs[1] = x_dot;
        s_obs[2] = th;
        s_obs[3] = th_dot;
      }
      trunc_flag = trunc ? 1 : 0;
    }
    trunc_flag = __builtin_amdgcn_readfirstlane(trunc_flag);
    wave_lds_sync();
    if (trunc_flag) {  // truncation bootstrap: r += V(final_obs)  (wave-uniform branch)
      const float* ff = wave_chain<LW>(p.enc, s_w, s_fin, s_a, s_b, lane);
      for (int j = lane; j < F; j += 64) s_c[j] = ff[j];
      wave_lds_sync();
      const float vf = wave_chain<LW>(p.critic, s_w, s_c, s_a, s_b, lane)[0];
      if (lane == 0) p.b_rewards[tn] += vf;
    }
  }
  if (lane < 4) {
    p.state[4 * n + lane] = s_obs[lane];
    p.obs_out[4 * n + lane] = s_obs[lane];
  }
  if (lane == 0) {
    p.steps[n] = steps;
    p.ep_ret[n] = ep_ret;
  }
}

// ---------------------------------------------------------------------------------------------
// Register variant (every layer width <= 64): activations live in VGPRs, lane j holding unit j.
// A layer is y_j = act(b_j + sum_k x_k W^T[k][j]) with x_k broadcast by v_readlane (a VALU op, no
// LDS round trip) and W^T[k][j] read from LDS by consecutive lanes; no barriers, no LDS writes.
// Every lane runs the (scalar) env step redundantly, so the state stays uniform in registers.
__device__ __forceinline__ float lane_bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

__device__ __forceinline__ float reg_chain(const Chain& c, const float* __restrict__ sw, float x, int lane) {
  for (int l = 0; l < c.n; ++l) {
    const int din = c.din[l], dout = c.dout[l];
    const int jj = lane < dout ? lane : dout - 1;
    const float* wt = sw + c.woff[l] + jj;
    float a0 = sw[c.boff[l] + jj], a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (din == 64) {
#pragma unroll
      for (int k = 0; k < 64; k += 4) {
        a0 = fmaf(lane_bcast(x, k), wt[k * dout], a0);
        a1 = fmaf(lane_bcast(x, k + 1), wt[(k + 1) * dout], a1);
        a2 = fmaf(lane_bcast(x, k + 2), wt[(k + 2) * dout], a2);
        a3 = fmaf(lane_bcast(x, k + 3), wt[(k + 3) * dout], a3);
      }
    } else {
      for (int k = 0; k < din; ++k) a0 = fmaf(lane_bcast(x, k), wt[k * dout], a0);
    }
    const float y = ro_act((a0 + a1) + (a2 + a3), c.act[l]);
    x = lane < dout ? y : 0.f;
  }
  return x;
}

__global__ void __launch_bounds__(64 * RO_ENVS_PER_BLOCK) ppo_cartpole_rollout_reg_kernel(RolloutArgs p) {
  __shared__ __attribute__((aligned(16))) float s_w[RO_LDSW];
  stage_chain(p.enc, s_w);
  stage_chain(p.actor, s_w);
  stage_chain(p.head, s_w);
  stage_chain(p.critic, s_w);
  __syncthreads();  // the only barrier: from here on every wave (env) runs on its own
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * RO_ENVS_PER_BLOCK + wave;
  if (n >= p.N) return;
  const float gravity = 9.8f, masscart = 1.0f, masspole = 0.1f, total_mass = masspole + masscart, length = 0.5f;
  const float pml = masspole * length, force_mag = 10.0f, tau = 0.02f;
  const float theta_thr = 12.f * 2.f * 3.14159265358979323846f / 360.f, x_thr = 2.4f;
  float x = p.state[4 * n], x_dot = p.state[4 * n + 1], th = p.state[4 * n + 2], th_dot = p.state[4 * n + 3];
  int steps = p.steps[n];
  float ep_ret = p.ep_ret[n];
  for (int t = 0; t < p.T; ++t) {
    const size_t tn = (size_t)t * p.N + n;
    const float ob = lane == 0 ? x : lane == 1 ? x_dot : lane == 2 ? th : lane == 3 ? th_dot : 0.f;
    if (lane < 4) p.b_state[4 * tn + lane] = ob;
    const float feat = reg_chain(p.enc, s_w, ob, lane);
    const float logit = reg_chain(p.head, s_w, reg_chain(p.actor, s_w, feat, lane), lane);
    const float value = lane_bcast(reg_chain(p.critic, s_w, feat, lane), 0);
    // Gumbel-max sample and log-prob over the A logits (uniform over the wave)
    float mx = -INFINITY;
    for (int a = 0; a < p.A; ++a) mx = fmaxf(mx, lane_bcast(logit, a));
    float se = 0.f;
    for (int a = 0; a < p.A; ++a) se += __expf(lane_bcast(logit, a) - mx);
    const float lse = mx + __logf(se);
    int pick = 0;
    float best = -INFINITY, lpick = 0.f;
    for (int a = 0; a < p.A; ++a) {
      const float la = lane_bcast(logit, a);
      const float g = la - __logf(-__logf(ro_uniform(p.seed, ((uint64_t)tn << 8) + a)));
      if (g > best) {
        best = g;
        pick = a;
        lpick = la;
      }
    }
    if (lane < p.A) p.b_actions[tn * p.A + lane] = lane == pick ? 1.f : 0.f;
    // CartPole-v1 step (dynamics of envs/classic.py) with autoreset
    const float force = pick == 1 ? force_mag : -force_mag;
    const float c = cosf(th), s = sinf(th);
    const float temp = (force + pml * th_dot * th_dot * s) / total_mass;
    const float thacc = (gravity * s - c * temp) / (length * (4.f / 3.f - masspole * c * c / total_mass));
    const float xacc = temp - pml * thacc * c / total_mass;
    const float fx = x + tau * x_dot, fxd = x_dot + tau * xacc, fth = th + tau * th_dot, fthd = th_dot + tau * thacc;
    const bool term = fx < -x_thr || fx > x_thr || fth < -theta_thr || fth > theta_thr;
    steps += 1;
    const bool trunc = !term && steps >= p.max_steps;
    ep_ret += 1.f;
    float reward = 1.f;
    if (trunc) {  // truncation bootstrap: r += V(final_obs)  (wave-uniform branch)
      const float fo = lane == 0 ? fx : lane == 1 ? fxd : lane == 2 ? fth : lane == 3 ? fthd : 0.f;
      reward += lane_bcast(reg_chain(p.critic, s_w, reg_chain(p.enc, s_w, fo, lane), lane), 0);
    }
    if (lane == 0) {
      p.b_logp[tn] = lpick - lse;
      p.b_values[tn] = value;
      p.b_rewards[tn] = reward;
      p.b_dones[tn] = (term || trunc) ? 1.f : 0.f;
      p.b_done_ret[tn] = (term || trunc) ? ep_ret : 0.f;
      p.b_done_len[tn] = (term || trunc) ? (float)steps : 0.f;
    }
    if (term || trunc) {
      x = ro_uniform(p.seed, ((uint64_t)tn << 8) + 128) * 0.1f - 0.05f;
      x_dot = ro_uniform(p.seed, ((uint64_t)tn << 8) + 129) * 0.1f - 0.05f;
      th = ro_uniform(p.seed, ((uint64_t)tn << 8) + 130) * 0.1f - 0.05f;
      th_dot = ro_uniform(p.seed, ((uint64_t)tn << 8) + 131) * 0.1f - 0.05f;
      steps = 0;
      ep_ret = 0.f;
    } else {
      x = fx;
      x_dot = fxd;
      th = fth;
      th_dot = fthd;
    }
  }
  if (lane == 0) {
    p.state[4 * n] = p.obs_out[4 * n] = x;
    p.state[4 * n + 1] = p.obs_out[4 * n + 1] = x_dot;
    p.state[4 * n + 2] = p.obs_out[4 * n + 2] = th;
    p.state[4 * n + 3] = p.obs_out[4 * n + 3] = th_dot;
    p.steps[n] = steps;
    p.ep_ret[n] = ep_ret;
  }
}

}  // namespace srl

static bool ro_narrow(const srl::Chain& c) {
  for (int l = 0; l < c.n; ++l)
    if (c.din[l] > 64 || c.dout[l] > 64) return false;
  return true;
}

void launch_ppo_cartpole_rollout(const srl::RolloutArgs& p, hipStream_t st) {
  const int nb = srl::cdiv(p.N, srl::RO_ENVS_PER_BLOCK);
  const int threads = 64 * (p.N < srl::RO_ENVS_PER_BLOCK ? p.N : srl::RO_ENVS_PER_BLOCK);
  if (p.lds_weights && p.A <= 64 && ro_narrow(p.enc) && ro_narrow(p.actor) && ro_narrow(p.head) && ro_narrow(p.critic))
    hipLaunchKernelGGL(srl::ppo_cartpole_rollout_reg_kernel, dim3(nb), dim3(threads), 0, st, p);
  else if (p.lds_weights)
    hipLaunchKernelGGL(srl::ppo_cartpole_rollout_kernel<true>, dim3(nb), dim3(threads), 0, st, p);
  else
    hipLaunchKernelGGL(srl::ppo_cartpole_rollout_kernel<false>, dim3(nb), dim3(threads), 0, st, p);
}
