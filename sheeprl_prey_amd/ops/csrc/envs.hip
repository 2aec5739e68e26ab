// Device-resident classic-control environments: one thread per env, auto-reset inside the step, so
// a whole PPO rollout (policy forward + env step, T times) can be captured in ONE hipGraph with no
// host round trip (reference env: gymnasium CartPole-v1 behind SyncVectorEnv + TimeLimit(500) +
// RecordEpisodeStatistics; dynamics identical to envs/classic.py CartPoleEnv.step).
#include "common.h"

namespace srl {

// state [N,4] (x, x_dot, theta, theta_dot), steps [N] (int), ep_ret [N]; action [N] (index 0/1);
// uniform [N,4] U(0,1) draws for resets.  Outputs: obs [N,4] (post-reset observation, what the agent
// sees next), reward [N], terminated [N], truncated [N], final_obs [N,4] (pre-reset observation),
// done_ret / done_len [N] (episode return / length where an episode ended this step, else 0).
__global__ void cartpole_step_kernel(float* __restrict__ state, int* __restrict__ steps, float* __restrict__ ep_ret,
                                     const int64_t* __restrict__ action, const float* __restrict__ uniform,
                                     float* __restrict__ obs, float* __restrict__ reward, float* __restrict__ terminated,
                                     float* __restrict__ truncated, float* __restrict__ final_obs,
                                     float* __restrict__ done_ret, float* __restrict__ done_len, int N, int max_steps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const float gravity = 9.8f, masscart = 1.0f, masspole = 0.1f, total_mass = masspole + masscart, length = 0.5f;
  const float polemass_length = masspole * length, force_mag = 10.0f, tau = 0.02f;
  const float theta_thr = 12.f * 2.f * 3.14159265358979323846f / 360.f, x_thr = 2.4f;
  float x = state[4 * i], x_dot = state[4 * i + 1], th = state[4 * i + 2], th_dot = state[4 * i + 3];
  const float force = action[i] == 1 ? force_mag : -force_mag;
  const float c = cosf(th), s = sinf(th);
  const float temp = (force + polemass_length * th_dot * th_dot * s) / total_mass;
  const float thacc = (gravity * s - c * temp) / (length * (4.f / 3.f - masspole * c * c / total_mass));
  const float xacc = temp - polemass_length * thacc * c / total_mass;
  x += tau * x_dot;
  x_dot += tau * xacc;
  th += tau * th_dot;
  th_dot += tau * thacc;
  const bool term = x < -x_thr || x > x_thr || th < -theta_thr || th > theta_thr;
  const int n = steps[i] + 1;
  const bool trunc = !term && n >= max_steps;
  const float r = 1.f;
  const float ret = ep_ret[i] + r;
  final_obs[4 * i] = x;
  final_obs[4 * i + 1] = x_dot;
  final_obs[4 * i + 2] = th;
  final_obs[4 * i + 3] = th_dot;
  reward[i] = r;
  terminated[i] = term ? 1.f : 0.f;
  truncated[i] = trunc ? 1.f : 0.f;
  if (term || trunc) {
    done_ret[i] = ret;
    done_len[i] = (float)n;
    x = uniform[4 * i] * 0.1f - 0.05f;
    x_dot = uniform[4 * i + 1] * 0.1f - 0.05f;
    th = uniform[4 * i + 2] * 0.1f - 0.05f;
    th_dot = uniform[4 * i + 3] * 0.1f - 0.05f;
    steps[i] = 0;
    ep_ret[i] = 0.f;
  } else {
    done_ret[i] = 0.f;
    done_len[i] = 0.f;
    steps[i] = n;
    ep_ret[i] = ret;
  }
  state[4 * i] = x;
  state[4 * i + 1] = x_dot;
  state[4 * i + 2] = th;
  state[4 * i + 3] = th_dot;
  obs[4 * i] = x;
  obs[4 * i + 1] = x_dot;
  obs[4 * i + 2] = th;
  obs[4 * i + 3] = th_dot;
}

}  // namespace srl

void launch_cartpole_step(float* state, int* steps, float* ep_ret, const int64_t* action, const float* uniform, float* obs,
                          float* reward, float* terminated, float* truncated, float* final_obs, float* done_ret,
                          float* done_len, int N, int max_steps, hipStream_t st) {
  hipLaunchKernelGGL(srl::cartpole_step_kernel, dim3(srl::cdiv(N, 256)), dim3(256), 0, st, state, steps, ep_ret, action,
                     uniform, obs, reward, terminated, truncated, final_obs, done_ret, done_len, N, max_steps);
}
