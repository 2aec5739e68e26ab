// Argument block of the one-launch PPO rollout kernel (ppo_rollout.hip), shared by the host binding
// (bindings.cpp) so both sides agree on the layout.
#pragma once
#include <stdint.h>

namespace srl {

constexpr int RO_MAXL = 8;         // layers per MLP chain
constexpr int RO_MAXW = 256;       // max layer width
constexpr int RO_LDSW = 32 * 1024; // floats of LDS for the staged (transposed) weights + biases: 128 KB
constexpr int RO_ENVS_PER_BLOCK = 4;

// y = act_n(W_n ... act_1(W_1 x + b_1) ... + b_n); W_l row-major [dout, din] in global memory.
// woff / boff: where the kernel stages W_l^T [din, dout] and b_l inside its LDS weight block.
struct Chain {
  int n;
  int din[RO_MAXL], dout[RO_MAXL], act[RO_MAXL];
  int woff[RO_MAXL], boff[RO_MAXL];
  const float* W[RO_MAXL];
  const float* b[RO_MAXL];
};

struct RolloutArgs {
  Chain enc, actor, head, critic;
  int N, T, A, max_steps;
  int lds_weights;  // 1: all chains fit in RO_LDSW floats and are staged once per launch
  uint64_t seed;
  float *state, *ep_ret, *obs_out;
  int* steps;
  float *b_state, *b_actions, *b_logp, *b_values, *b_rewards, *b_dones, *b_done_ret, *b_done_len;
};

}  // namespace srl
