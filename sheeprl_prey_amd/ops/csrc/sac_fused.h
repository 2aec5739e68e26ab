// Parameter blocks of the fused SAC update kernels (sac_fused.hip), shared with their torch bindings
// (sac_bindings.cpp).  Plain pointers and sizes: every launch is graph-capturable (the per-step random
// stream comes from device counters, not from kernel arguments).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace srl {
namespace sacf {

// SACActor: obs -> relu(W1) -> relu(W2) -> (mean = Wm h2 + bm, raw log-std = Ws h2 + bs), log-std clamped to [lo, hi]
struct ActorW {
  const float *W1, *b1, *W2, *b2, *Wm, *bm, *Ws, *bs, *scale, *bias;
  int OD, H, A;
  float lo, hi;
};

// EnsembleMLP critic (stacked [n, out, in]): q_c = w3_c . relu(W2_c relu(W1_c [obs, act] + b1_c) + b2_c) + b3_c
struct CriticW {
  const float *W1, *b1, *W2, *b2, *W3, *b3;
  int n, H;
};

// player: actions (+ log-probs) for M observation rows; counter ctr[0] advanced once per launch
struct ActP {
  ActorW a;
  const float* obs;
  float* act;   // [M, A]
  float* logp;  // [M] or null
  float* eps;   // [M, A] or null (the noise drawn)
  unsigned long long* ctr;
  int* ticket;
  unsigned long long seed;
  int M;
};

// Bellman target with the next actions sampled in-kernel: y = r + (1 - d) gamma (min_c Q'_c(s', a') - alpha logp')
struct TgtP {
  ActorW a;
  CriticW c;  // the TARGET ensemble
  const float *obs, *rew, *done, *log_alpha;
  const unsigned long long* ctr;
  unsigned long long seed;
  float* y;     // [M]
  float* act;   // [M, A] or null
  float* logp;  // [M] or null
  float* eps;   // [M, A] or null
  long long* ts;  // phase timestamps of workgroup 0 (s_memrealtime, 100 MHz) or null
  int M;
  float gamma;
};

// actor + alpha objective, forward and data backward (grid: row blocks x critics; the last critic workgroup of a
// row block finishes the actor backward)
struct UpdP {
  ActorW a;
  CriticW c;
  const float *obs, *log_alpha;
  const unsigned long long* ctr;
  unsigned long long seed;
  float *Xa, *H1a, *H2a, *DZ, *DH1a, *DH2a;  // weight-gradient operands [M, ODp] [M, H] [M, H] [M, ZP] [M, H] [M, H]
  float *QX, *DAX;                           // critic hand-off [n, M], [n, M, A]
  float* part;                               // [blocks, 2] loss partials
  float *act, *logp, *eps, *q;               // [M, A] [M] [M, A] [M, n]: optional (tests / metrics)
  int* cnt;                                  // [blocks] tickets, zero at rest
  long long* ts;                             // phase timestamps of row block 0 (s_memrealtime) or null
  int M, reduce_min;
};

// actor weight gradients + the alpha gradient + losses / metric sums
struct WgP {
  const float *Xa, *H1a, *H2a, *DZ, *DH1a, *DH2a, *part;
  float *dW1, *db1, *dW2, *db2, *dWm, *dbm, *dWs, *dbs, *dlog_alpha;
  const float *log_alpha, *target_entropy, *qf_loss;
  float* losses;                // [2] policy loss, alpha loss
  double* acc;                  // [3][2] (sum, count) of value / policy / alpha loss, or null
  unsigned long long* ctr;      // ++ctr[0] (the update's random stream) when set
  int M, OD, H, A, nblk;
};

// one flat Adam slab of a multi-slab update (the step count advance folded in; optional EMA target)
struct AdamSlab {
  float* p;
  const float* g;
  float *m, *v, *scalars;
  float* ema;          // target slab (lerp towards the updated parameters) or null
  const float* ema_w;  // device scalar weight of the EMA
  long long n;         // floats, multiple of 4
  float lr, b1, b2, eps, wd;
  int decoupled;
};
constexpr int MAX_SLABS = 4;

int zp_of(int A);  // head columns (mean | log-std) padded to 16
size_t act_lds(const ActorW& a);
size_t tgt_lds(const ActorW& a, const CriticW& c);
size_t upd_lds(const ActorW& a, const CriticW& c);
int upd_blocks(int M);
void launch_act(const ActP& p, hipStream_t st);
void launch_tgt(const TgtP& p, hipStream_t st);
void launch_upd(const UpdP& p, hipStream_t st);
void launch_wg(const WgP& p, hipStream_t st);
void launch_adam_multi(const AdamSlab* s, int ns, int* guard, int* tickets, hipStream_t st);

}  // namespace sacf
}  // namespace srl
