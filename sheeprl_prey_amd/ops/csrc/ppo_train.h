// Argument block of the one-launch PPO update kernel for MLP agents (ppo_train.hip), shared with the
// host binding (bindings.cpp), which also computes the LDS plan.
#pragma once
#include <stdint.h>

namespace srl {

constexpr int PT_MAXL = 16;       // layers over all chains
constexpr int PT_THREADS = 512;   // 8 waves, one workgroup
constexpr int PT_MAXT = 4;        // 4x4 weight-gradient tiles owned per thread (registers)
constexpr int PT_LDS = 40928;     // floats of the LDS arena (~160 KB: the whole CU LDS minus a reduction scratch)
constexpr int PT_R = 16;          // minibatch rows per chunk (2 per wave)
constexpr int PT_MAXD0 = 8;       // observation width held in registers per minibatch row
constexpr int PT_MAXA = 8;        // actions held in registers per minibatch row

// One Linear(+activation).  W^T augmented with the bias as row `din` lives in LDS at `wt`
// ([k4][ldw], zero padded); the activation buffers are row-major [PT_R][ld] with a constant-1
// column at `width` (the bias input of the consumer) and zeros after it.
struct PTLayer {
  int din, dout, act;
  int wt, ldw, k4;
  int pw, pb;             // flat-slab offsets of W [dout, din] and b [dout] (pb < 0: no bias)
  int tile0, tj, tk;      // first 4x4 gradient tile id, tiles along dout and along k4
  int in_node, in_ld;     // LDS activation buffer feeding this layer
  int out_node, out_ld;   // LDS buffer this layer writes
  int in_act;             // activation that produced the input (for act'), -1: raw observation
};

struct PTArgs {
  PTLayer L[PT_MAXL];
  int ne, na, nh, nc;     // encoder, actor backbone, head, critic layers (in this order in L)
  int ntiles;
  int node_lo, node_hi;   // LDS range of activation buffers + temps (zeroed at start)
  int tmpA, tmpB, tmpD, tmp_ld;
  const float *obs, *actions, *logp_old, *val_old, *ret, *adv;
  const int64_t* perm;    // [epochs, n] minibatch order
  int n, bs, epochs, D0, A;
  const float *clip_p, *ent_p;
  float vf_coef, max_grad_norm;
  int clip_vloss, norm_adv;
  float *param, *grad, *m, *v, *scalars;
  float lr, b1, b2, eps, wd;
  int decoupled;
  float* out_sums;        // [3] mean policy / value / entropy loss over the minibatch steps (zeroed by the launcher)
  // workgroup w runs chunks w, w + nwg, ... of every minibatch and publishes its gradient tiles into
  // partial[w] (flat-slab order); after a grid barrier every workgroup reduces + Adam-updates its
  // 1/nwg share of each parameter region (coalesced, straight into the slabs) and, after a second
  // barrier, re-reads the other shares into its LDS weights.  `bar` is a monotonic grid-barrier
  // counter (zeroed by the launcher), `err` > 0 if a barrier wait timed out.
  int nwg;
  int nparam;             // flat-slab length (partial holds nwg copies)
  float* partial;
  float* sq;              // [nwg] per-workgroup squared gradient norms (global-norm clip)
  int* bar;
  float* err;
  long long* prof;        // optional [4] s_memtime cycle totals of workgroup 0 (chunk / publish+barrier /
                          // reduce+Adam / barrier+reload), diagnostics only
};

}  // namespace srl
