// Parameter block of the persistent DreamerV3 imagination rollout (imagine.hip); plain C layout
// shared with the bindings (ext_bindings.cpp).
#pragma once

namespace srl {
namespace imag {

constexpr int MAXL = 8;  // actor MLP layers
constexpr int MAXH = 8;  // discrete action heads

struct IP {
  int M, horizon;              // rows (B*T start states), imagined steps
  int S, Hd, D, Da, La, Ht;    // stochastic (G*disc), recurrent, recurrent-MLP, actor dense, actor layers, transition hidden
  int A, nh, disc, G;          // total action width, heads, classes per prior categorical, prior categoricals
  int NB, RB, nslots;          // column splits per row block, 64-row blocks, row-block slots (grid = nslots * NB)
  int head[MAXH];              // classes per action head
  float alpha_a, alpha_s;      // unimix of the actor heads / of the prior
  float eps_a, eps_r, eps_g, eps_t;
  int act_a, act_r, act_t;
  // actor: Wa[l] [Da, in_l] (in_0 = S + Hd, columns (prior | h)); WaT = Wa[0][:, :S]^T [S, Da]
  const float* Wa[MAXL];
  const float* ba[MAXL];
  const float* lnaw[MAXL];
  const float* lnab[MAXL];
  const float* WaT;
  const float *Wh, *bh;                      // heads stacked [A, Da], [A]
  const float *WrT, *br, *lnrw, *lnrb;       // recurrent input layer, transposed [S + A, D] (rows (prior | action))
  const float *Wg, *bg, *lngw, *lngb;        // GRU projection [3Hd, Hd + D] (columns (h | feat)), LN over 3Hd
  const float *Wt1, *bt1, *lntw, *lntb;      // transition hidden layer [Ht, Hd]
  const float *Wt2, *bt2;                    // transition logits [S, Ht], [S]
  const float* U;                            // uniforms [horizon + 1][M * (nh + G)]
  float* buf;                                // trajectories [horizon + 1][M][A + S + Hd] = (action | prior | h)
  float* Y;                                  // pre-activation hand-off buffers [2][M][max(Da, D, Ht)]
  float* part;                               // row partial (mean, M2) per column split [2][M][NB][2]
  int* idx;                                  // sampled prior class per (row, categorical) [M][G]; holds step 0 on entry
  unsigned* sync;                            // arrival counter per slot (32-word stride) + error word
  long long* prof;                           // optional: block 0 timestamps, [arrival][2] (work done, wait done)
};

}  // namespace imag
}  // namespace srl
