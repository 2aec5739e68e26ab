// Torch bindings of the fused SAC update (sac_fused.hip, sac_critic.hip).  Every operand's shape is checked
// here, before a launch: the kernels assume contiguous fp32 GPU tensors, hidden widths that are multiples of
// 128 (8 waves x 16-column tiles), A <= 32 action dimensions and the LDS budget computed by sac_fused.hip.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>

#include "sac_fused.h"

void launch_sac_critic_wgrad(const float* X, const float* H1, const float* H2, const float* DH1, const float* DH2,
                             const float* DQ, const float* g, float* dW1, float* db1, float* dW2, float* db2, float* dW3,
                             float* db3, int M, int IN, int H, int n, const float* lossp, int nlp, float* loss,
                             hipStream_t st);

namespace {

using namespace srl::sacf;

constexpr size_t LDS_MAX = 160 * 1024;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void f32(const torch::Tensor& t, const char* name, int64_t numel = -1) {
  TORCH_CHECK(t.defined() && t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), "sac_fused: ", name,
              " must be a contiguous float32 GPU tensor");
  TORCH_CHECK(numel < 0 || t.numel() == numel, "sac_fused: ", name, " holds ", t.numel(), " values, expected ", numel);
}

float* optf(const c10::optional<torch::Tensor>& t, const char* name, int64_t numel) {
  if (!t.has_value() || !t->defined()) return nullptr;
  f32(*t, name, numel);
  return t->data_ptr<float>();
}

unsigned long long* ctr_ptr(const torch::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kInt64 && t.is_contiguous() && t.numel() >= 1,
              "sac_fused: counter must be a contiguous int64 GPU tensor");
  return reinterpret_cast<unsigned long long*>(t.data_ptr<int64_t>());
}

long long* ts_ptr(const c10::optional<torch::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64 && t->is_contiguous() && t->numel() >= 16,
              "sac_fused: timestamps must be a contiguous int64 GPU tensor of >= 16 values");
  return reinterpret_cast<long long*>(t->data_ptr<int64_t>());
}

int* int_ptr(const torch::Tensor& t, int64_t numel, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kInt32 && t.is_contiguous() && t.numel() >= numel, "sac_fused: ",
              name, " must be a contiguous int32 GPU tensor of >= ", numel, " values");
  return t.data_ptr<int>();
}

// actor = [W1 [H, OD], b1, W2 [H, H], b2, Wm [A, H], bm, Ws [A, H], bs, scale [A], bias [A]]
ActorW actor_w(const std::vector<torch::Tensor>& w, double lo, double hi) {
  TORCH_CHECK(w.size() == 10, "sac_fused: actor = [W1, b1, W2, b2, Wm, bm, Ws, bs, scale, bias]");
  TORCH_CHECK(w[0].dim() == 2 && w[4].dim() == 2, "sac_fused: actor weights are 2-D");
  const int64_t H = w[0].size(0), OD = w[0].size(1), A = w[4].size(0);
  TORCH_CHECK(H % 128 == 0 && H <= 512 && OD >= 1 && OD <= 1024 && A >= 1 && A <= 32,
              "sac_fused: actor H % 128 == 0, H <= 512, obs dim <= 1024, 1 <= A <= 32");
  const int64_t numel[10] = {H * OD, H, H * H, H, A * H, A, A * H, A, A, A};
  const char* names[10] = {"W1", "b1", "W2", "b2", "Wm", "bm", "Ws", "bs", "scale", "bias"};
  for (int i = 0; i < 10; ++i) f32(w[i], names[i], numel[i]);
  ActorW a;
  a.W1 = w[0].data_ptr<float>();
  a.b1 = w[1].data_ptr<float>();
  a.W2 = w[2].data_ptr<float>();
  a.b2 = w[3].data_ptr<float>();
  a.Wm = w[4].data_ptr<float>();
  a.bm = w[5].data_ptr<float>();
  a.Ws = w[6].data_ptr<float>();
  a.bs = w[7].data_ptr<float>();
  a.scale = w[8].data_ptr<float>();
  a.bias = w[9].data_ptr<float>();
  a.OD = (int)OD;
  a.H = (int)H;
  a.A = (int)A;
  a.lo = (float)lo;
  a.hi = (float)hi;
  return a;
}

// critic = [W1 [n, H, OD + A], b1 [n, H], W2 [n, H, H], b2 [n, H], W3 [n, 1, H], b3 [n, 1]]
CriticW critic_w(const std::vector<torch::Tensor>& w, const ActorW& a) {
  TORCH_CHECK(w.size() == 6 && w[0].dim() == 3, "sac_fused: critic = [W1, b1, W2, b2, W3, b3] (stacked ensemble)");
  const int64_t n = w[0].size(0), H = w[0].size(1), IN = w[0].size(2);
  TORCH_CHECK(IN == a.OD + a.A, "sac_fused: critic input width must be obs + action dims");
  TORCH_CHECK(n >= 1 && n <= 8 && H % 128 == 0 && H <= 512, "sac_fused: critic n <= 8, H % 128 == 0, H <= 512");
  const int64_t numel[6] = {n * H * IN, n * H, n * H * H, n * H, n * H, n};
  const char* names[6] = {"critic W1", "critic b1", "critic W2", "critic b2", "critic W3", "critic b3"};
  for (int i = 0; i < 6; ++i) f32(w[i], names[i], numel[i]);
  CriticW c;
  c.W1 = w[0].data_ptr<float>();
  c.b1 = w[1].data_ptr<float>();
  c.W2 = w[2].data_ptr<float>();
  c.b2 = w[3].data_ptr<float>();
  c.W3 = w[4].data_ptr<float>();
  c.b3 = w[5].data_ptr<float>();
  c.n = (int)n;
  c.H = (int)H;
  return c;
}

int64_t rows_of(const torch::Tensor& obs, const ActorW& a) {
  f32(obs, "obs");
  TORCH_CHECK(obs.dim() == 2 && obs.size(1) == a.OD && obs.size(0) >= 1, "sac_fused: obs [M, obs dim]");
  return obs.size(0);
}

// ---- player: actions (+ logp, + the noise) for the observation rows; ctr[0] advanced once
void sac_fused_act(torch::Tensor obs, std::vector<torch::Tensor> actor, double lo, double hi, torch::Tensor ctr,
                   torch::Tensor ticket, int64_t seed, torch::Tensor act, c10::optional<torch::Tensor> logp,
                   c10::optional<torch::Tensor> eps) {
  ActP p;
  p.a = actor_w(actor, lo, hi);
  const int64_t M = rows_of(obs, p.a);
  TORCH_CHECK(act_lds(p.a) <= LDS_MAX, "sac_fused_act: LDS budget");
  f32(act, "act", M * p.a.A);
  p.obs = obs.data_ptr<float>();
  p.act = act.data_ptr<float>();
  p.logp = optf(logp, "logp", M);
  p.eps = optf(eps, "eps", M * p.a.A);
  p.ctr = ctr_ptr(ctr);
  p.ticket = int_ptr(ticket, 1, "ticket");
  p.seed = (unsigned long long)seed;
  p.M = (int)M;
  launch_act(p, stream());
}

// ---- Bellman target with in-kernel next actions
void sac_fused_target(torch::Tensor obs, torch::Tensor rew, torch::Tensor done, torch::Tensor log_alpha,
                      std::vector<torch::Tensor> actor, double lo, double hi, std::vector<torch::Tensor> target,
                      torch::Tensor ctr, int64_t seed, double gamma, torch::Tensor y, c10::optional<torch::Tensor> act,
                      c10::optional<torch::Tensor> logp, c10::optional<torch::Tensor> eps,
                      c10::optional<torch::Tensor> ts) {
  TgtP p;
  p.a = actor_w(actor, lo, hi);
  p.c = critic_w(target, p.a);
  const int64_t M = rows_of(obs, p.a);
  TORCH_CHECK(tgt_lds(p.a, p.c) <= LDS_MAX, "sac_fused_target: LDS budget");
  f32(rew, "rewards", M);
  f32(done, "dones", M);
  f32(log_alpha, "log_alpha", 1);
  f32(y, "y", M);
  p.obs = obs.data_ptr<float>();
  p.rew = rew.data_ptr<float>();
  p.done = done.data_ptr<float>();
  p.log_alpha = log_alpha.data_ptr<float>();
  p.ctr = ctr_ptr(ctr);
  p.seed = (unsigned long long)seed;
  p.y = y.data_ptr<float>();
  p.act = optf(act, "act", M * p.a.A);
  p.logp = optf(logp, "logp", M);
  p.eps = optf(eps, "eps", M * p.a.A);
  p.ts = ts_ptr(ts);
  p.M = (int)M;
  p.gamma = (float)gamma;
  launch_tgt(p, stream());
}

// ---- critic weight gradients written into the given tensors (the optimiser slab views) + the loss sum
void sac_fused_critic_wgrad(std::vector<torch::Tensor> saved, torch::Tensor g, int64_t IN, std::vector<torch::Tensor> grads,
                            torch::Tensor lossp, torch::Tensor loss) {
  TORCH_CHECK(saved.size() == 6 && grads.size() == 6, "sac_fused_critic_wgrad: saved = [X, H1, H2, DH1, DH2, DQ], 6 grads");
  const torch::Tensor& H1 = saved[1];
  TORCH_CHECK(H1.dim() == 3, "sac_fused_critic_wgrad: H1 [n, M, H]");
  const int64_t n = H1.size(0), M = H1.size(1), H = H1.size(2), INp = (IN + 15) / 16 * 16;
  TORCH_CHECK(H % 128 == 0 && n >= 1 && n <= 8, "sac_fused_critic_wgrad: H % 128 == 0, n <= 8");
  const int64_t sn[6] = {M * INp, n * M * H, n * M * H, n * M * H, n * M * H, n * M};
  for (int i = 0; i < 6; ++i) f32(saved[i], "saved operand", sn[i]);
  const int64_t gn[6] = {n * H * IN, n * H, n * H * H, n * H, n * H, n};
  for (int i = 0; i < 6; ++i) f32(grads[i], "critic gradient", gn[i]);
  f32(g, "loss gradient", 1);
  f32(lossp, "partial losses");
  f32(loss, "loss", 1);
  launch_sac_critic_wgrad(saved[0].data_ptr<float>(), saved[1].data_ptr<float>(), saved[2].data_ptr<float>(),
                          saved[3].data_ptr<float>(), saved[4].data_ptr<float>(), saved[5].data_ptr<float>(),
                          g.data_ptr<float>(), grads[0].data_ptr<float>(), grads[1].data_ptr<float>(),
                          grads[2].data_ptr<float>(), grads[3].data_ptr<float>(), grads[4].data_ptr<float>(),
                          grads[5].data_ptr<float>(), (int)M, (int)IN, (int)H, (int)n, lossp.data_ptr<float>(),
                          (int)lossp.numel(), loss.data_ptr<float>(), stream());
}

// ---- actor + alpha update: objective forward / backward (upd_kernel) and weight gradients (wg_kernel)
// ws = [Xa [M, ODp], H1a [M, H], H2a [M, H], DZ [M, ZP], DH1a [M, H], DH2a [M, H], QX [n, M], DAX [n, M, A],
//       part [blocks, 2]];  grads = [dW1, db1, dW2, db2, dWm, dbm, dWs, dbs, dlog_alpha]
void sac_fused_actor(torch::Tensor obs, torch::Tensor log_alpha, torch::Tensor target_entropy,
                     std::vector<torch::Tensor> actor, double lo, double hi, std::vector<torch::Tensor> critic,
                     torch::Tensor ctr, int64_t seed, bool reduce_min, std::vector<torch::Tensor> ws, torch::Tensor cnt,
                     std::vector<torch::Tensor> grads, c10::optional<torch::Tensor> qf_loss, torch::Tensor losses,
                     c10::optional<torch::Tensor> acc, c10::optional<torch::Tensor> act, c10::optional<torch::Tensor> logp,
                     c10::optional<torch::Tensor> eps, c10::optional<torch::Tensor> q,
                     c10::optional<torch::Tensor> ts) {
  UpdP u;
  u.a = actor_w(actor, lo, hi);
  u.c = critic_w(critic, u.a);
  const int64_t M = rows_of(obs, u.a);
  TORCH_CHECK(upd_lds(u.a, u.c) <= LDS_MAX, "sac_fused_actor: LDS budget");
  const int64_t H = u.a.H, A = u.a.A, n = u.c.n, ODp = (u.a.OD + 15) / 16 * 16, ZP = zp_of((int)A);
  const int64_t nblk = upd_blocks((int)M);
  TORCH_CHECK(ws.size() == 9 && grads.size() == 9, "sac_fused_actor: 9 workspaces, 9 gradients");
  const int64_t wn[9] = {M * ODp, M * H, M * H, M * ZP, M * H, M * H, n * M, n * M * A, 2 * nblk};
  for (int i = 0; i < 9; ++i) f32(ws[i], "workspace", wn[i]);
  const int64_t gn[9] = {H * u.a.OD, H, H * H, H, A * H, A, A * H, A, 1};
  for (int i = 0; i < 9; ++i) f32(grads[i], "actor gradient", gn[i]);
  f32(log_alpha, "log_alpha", 1);
  f32(target_entropy, "target_entropy", 1);
  f32(losses, "losses", 2);
  if (acc.has_value() && acc->defined())
    TORCH_CHECK(acc->is_cuda() && acc->scalar_type() == torch::kFloat64 && acc->is_contiguous() && acc->numel() == 6,
                "sac_fused_actor: acc [3, 2] float64");
  u.obs = obs.data_ptr<float>();
  u.log_alpha = log_alpha.data_ptr<float>();
  u.ctr = ctr_ptr(ctr);
  u.seed = (unsigned long long)seed;
  u.Xa = ws[0].data_ptr<float>();
  u.H1a = ws[1].data_ptr<float>();
  u.H2a = ws[2].data_ptr<float>();
  u.DZ = ws[3].data_ptr<float>();
  u.DH1a = ws[4].data_ptr<float>();
  u.DH2a = ws[5].data_ptr<float>();
  u.QX = ws[6].data_ptr<float>();
  u.DAX = ws[7].data_ptr<float>();
  u.part = ws[8].data_ptr<float>();
  u.act = optf(act, "act", M * A);
  u.logp = optf(logp, "logp", M);
  u.eps = optf(eps, "eps", M * A);
  u.q = optf(q, "q", M * n);
  u.cnt = int_ptr(cnt, nblk, "tickets");
  u.ts = ts_ptr(ts);
  u.M = (int)M;
  u.reduce_min = reduce_min ? 1 : 0;
  hipStream_t st = stream();
  launch_upd(u, st);
  WgP w;
  w.Xa = u.Xa;
  w.H1a = u.H1a;
  w.H2a = u.H2a;
  w.DZ = u.DZ;
  w.DH1a = u.DH1a;
  w.DH2a = u.DH2a;
  w.part = u.part;
  float* gp[9];
  for (int i = 0; i < 9; ++i) gp[i] = grads[i].data_ptr<float>();
  w.dW1 = gp[0];
  w.db1 = gp[1];
  w.dW2 = gp[2];
  w.db2 = gp[3];
  w.dWm = gp[4];
  w.dbm = gp[5];
  w.dWs = gp[6];
  w.dbs = gp[7];
  w.dlog_alpha = gp[8];
  w.log_alpha = u.log_alpha;
  w.target_entropy = target_entropy.data_ptr<float>();
  w.qf_loss = optf(qf_loss, "qf_loss", 1);
  w.losses = losses.data_ptr<float>();
  w.acc = acc.has_value() && acc->defined() ? acc->data_ptr<double>() : nullptr;
  w.ctr = ctr_ptr(ctr);
  w.M = (int)M;
  w.OD = u.a.OD;
  w.H = (int)H;
  w.A = (int)A;
  w.nblk = (int)nblk;
  launch_wg(w, st);
}

// ---- multi-slab Adam: slabs = [(p, g, m, v, scalars, ema or None, ema_w or None, lr, b1, b2, eps, wd, decoupled)]
void sac_adam_multi(std::vector<std::vector<torch::Tensor>> tensors, std::vector<std::vector<double>> hyper,
                    c10::optional<torch::Tensor> guard, torch::Tensor tickets) {
  const int ns = (int)tensors.size();
  TORCH_CHECK(ns >= 1 && ns <= MAX_SLABS && (int)hyper.size() == ns, "adam_multi: 1..4 slabs");
  AdamSlab s[MAX_SLABS];
  for (int i = 0; i < ns; ++i) {
    auto& t = tensors[i];
    auto& h = hyper[i];
    TORCH_CHECK(t.size() == 5 || t.size() == 7, "adam_multi: (p, g, m, v, scalars[, ema, ema_w])");
    TORCH_CHECK(h.size() == 6, "adam_multi: (lr, b1, b2, eps, wd, decoupled)");
    const int64_t n = t[0].numel();
    TORCH_CHECK(n % 4 == 0, "adam_multi: slab size must be a multiple of 4");
    f32(t[0], "param slab");
    for (int k = 1; k < 4; ++k) f32(t[k], "optimiser slab", n);
    f32(t[4], "scalars");
    TORCH_CHECK(t[4].numel() >= 4, "adam_multi: scalars [step, coef, norm, skip]");
    s[i].p = t[0].data_ptr<float>();
    s[i].g = t[1].data_ptr<float>();
    s[i].m = t[2].data_ptr<float>();
    s[i].v = t[3].data_ptr<float>();
    s[i].scalars = t[4].data_ptr<float>();
    s[i].ema = nullptr;
    s[i].ema_w = nullptr;
    if (t.size() == 7) {
      f32(t[5], "EMA target slab", n);
      f32(t[6], "EMA weight", 1);
      s[i].ema = t[5].data_ptr<float>();
      s[i].ema_w = t[6].data_ptr<float>();
    }
    s[i].n = n;
    s[i].lr = (float)h[0];
    s[i].b1 = (float)h[1];
    s[i].b2 = (float)h[2];
    s[i].eps = (float)h[3];
    s[i].wd = (float)h[4];
    s[i].decoupled = h[5] != 0.0 ? 1 : 0;
  }
  int* gp = nullptr;
  if (guard.has_value() && guard->defined()) gp = int_ptr(*guard, 3, "guard");
  launch_adam_multi(s, ns, gp, int_ptr(tickets, ns, "tickets"), stream());
}

}  // namespace

void register_sac(pybind11::module& m) {
  m.def("sac_fused_act", &sac_fused_act);
  m.def("sac_fused_target", &sac_fused_target, pybind11::arg("obs"), pybind11::arg("rew"), pybind11::arg("done"),
        pybind11::arg("log_alpha"), pybind11::arg("actor"), pybind11::arg("lo"), pybind11::arg("hi"), pybind11::arg("target"),
        pybind11::arg("ctr"), pybind11::arg("seed"), pybind11::arg("gamma"), pybind11::arg("y"), pybind11::arg("act"),
        pybind11::arg("logp"), pybind11::arg("eps"), pybind11::arg("ts") = pybind11::none());
  m.def("sac_fused_critic_wgrad", &sac_fused_critic_wgrad);
  m.def("sac_fused_actor", &sac_fused_actor, pybind11::arg("obs"), pybind11::arg("log_alpha"),
        pybind11::arg("target_entropy"), pybind11::arg("actor"), pybind11::arg("lo"), pybind11::arg("hi"),
        pybind11::arg("critic"), pybind11::arg("ctr"), pybind11::arg("seed"), pybind11::arg("reduce_min"), pybind11::arg("ws"),
        pybind11::arg("cnt"), pybind11::arg("grads"), pybind11::arg("qf_loss"), pybind11::arg("losses"), pybind11::arg("acc"),
        pybind11::arg("act"), pybind11::arg("logp"), pybind11::arg("eps"), pybind11::arg("q"),
        pybind11::arg("ts") = pybind11::none());
  m.def("sac_adam_multi", &sac_adam_multi);
  m.def("sac_fused_zp", [](int64_t A) { return (int64_t)zp_of((int)A); });
  m.def("sac_fused_blocks", [](int64_t M) { return (int64_t)upd_blocks((int)M); });
}
