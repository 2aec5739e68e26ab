// Torch bindings for the sheeprl_prey_amd HIP kernels.  Kernels live in *.hip files that only
// include <hip/hip_runtime.h>; this file owns shape checks, allocation and the current stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>

#include "scan4.h"
#include "scanp.h"

// ---- launchers (defined in the .hip translation units)
void launch_flat_grad_norm(const float*, int64_t, float*, int, float*, float*, float, int*, hipStream_t);
void launch_flat_advance(float*, int*, hipStream_t);
void launch_flat_adam(float*, const float*, float*, float*, const float*, int64_t, float, float, float, float, float, int,
                      hipStream_t);
bool launch_ln_act_fwd(const float*, int, float*, int, const float*, const float*, float*, float*, int, int, int, float, int,
                       hipStream_t);
int ln_bwd_grid(int, int, int);
bool launch_ln_act_bwd(const float*, int, const float*, int, float*, int, const float*, const float*, const float*,
                       const float*, float*, float*, float*, float*, int, int, int, int, hipStream_t);
void launch_colsum2(const float*, const float*, float*, float*, int, int, int, hipStream_t);
void launch_colsum1(const float*, int, float*, int, int, hipStream_t);
void set_colsum_workspace(float*, int64_t, int*, int64_t);
void set_colsum_side_stream(hipStream_t);
void launch_cartpole_step(float*, int*, float*, const int64_t*, const float*, float*, float*, float*, float*, float*, float*,
                          float*, int, int, hipStream_t);
void launch_rssm_mask_fwd(const float*, int, const float*, const float*, const float*, float*, int, float*, int, int, int,
                          hipStream_t);
void launch_rssm_mask_bwd(const float*, int, const float*, int, const float*, const float*, float*, float*, int, int, int,
                          hipStream_t);
void launch_ln_nchw_fwd(const float*, const float*, const float*, float*, float*, float*, int, int, int, float, int,
                        hipStream_t);
int ln_nchw_splits(int, int);
void launch_ln_nchw_bwd(const float*, const float*, const float*, const float*, const float*, const float*, float*, float*,
                        float*, float*, float*, int, int, int, int, hipStream_t);
bool launch_ln_gru_fwd(const float*, const float*, int, const float*, const float*, float*, float*, float*, int, int, float,
                       hipStream_t, int ldo = 0, const float* x2 = nullptr, int ldx2 = 0, float* xsum = nullptr);
int ln_gru_bwd_grid(int);
bool launch_ln_gru_bwd(const float*, const float*, int, const float*, const float*, const float*, const float*, const float*,
                       float*, float*, float*, float*, float*, float*, int, int, hipStream_t, const float* dadd = nullptr,
                       int ldadd = 0);
bool launch_unimix_sample_fwd(const float*, const float*, float*, float*, int, int, float, hipStream_t, int G = 0,
                              int lds = 0, int* idx = nullptr, int ldi = 0, int ioff = 0);
bool launch_unimix_sample_bwd(const float*, const float*, const float*, float*, int, int, float, hipStream_t);
bool launch_twohot_nll_fwd(const float*, const float*, const float*, float*, int, int, hipStream_t);
bool launch_twohot_nll_bwd(const float*, const float*, const float*, const float*, float*, int, int, hipStream_t);
bool launch_value_loss2(const float*, const float*, const float*, const float*, const float*, float*, float*, float*, int, int,
                        hipStream_t);
bool launch_twohot_mean_fwd(const float*, const float*, float*, float*, int, int, hipStream_t);
bool launch_twohot_mean_bwd(const float*, const float*, const float*, const float*, float*, int, int, hipStream_t);
bool launch_kl_fwd(const float*, const float*, float*, float*, float*, float*, int, int, int, float, float, float, hipStream_t);
bool launch_kl_bwd(const float*, const float*, const float*, const float*, float*, float*, int, int, int, float, float, float,
                   hipStream_t);
void launch_lambda_fwd(const float*, const float*, const float*, float*, int, int, float, hipStream_t);
void launch_lambda_bwd(const float*, const float*, const float*, const float*, float*, float*, float*, int, int, float,
                       hipStream_t);
void launch_gae(const float*, const float*, const float*, const float*, float*, float*, int, int, float, float, hipStream_t);
void launch_squashed_gaussian_fwd(const float*, const float*, const float*, const float*, const float*, float*, float*, int,
                                  int, int, float, float, hipStream_t);
void launch_squashed_gaussian_bwd(const float*, const float*, const float*, const float*, const float*, const float*, float*,
                                  float*, int, int, int, float, float, hipStream_t);

void launch_truncnorm_rsample_fwd(const float*, const float*, const float*, int, const float*, int, const float*, float*, int,
                                  hipStream_t);
void launch_truncnorm_rsample_bwd(const float*, const float*, const float*, int, const float*, int, const float*, const float*,
                                  float*, float*, int, hipStream_t);
void launch_truncnorm_logprob_fwd(const float*, const float*, const float*, const float*, int, const float*, int, float*, int,
                                  int, hipStream_t);
void launch_truncnorm_logprob_bwd(const float*, const float*, const float*, const float*, int, const float*, int, const float*,
                                  float*, float*, float*, int, int, hipStream_t);
bool launch_tn_head_linear_sample_fwd(const float*, int, const float*, const float*, const float*, float, float, float, float,
                                      float*, float*, float*, float*, int, int, int, int, hipStream_t, const float*,
                                      const float*, float, int, float*, int, float*, float*);
void launch_tn_head_sample_fwd(const float*, int, const float*, float, float, float, float, float*, float*, float*, int, int, int,
                               hipStream_t);
void launch_tn_head_sample_bwd(const float*, const float*, const float*, const float*, const float*, float, float, float, float*,
                               int, int, hipStream_t);

void launch_scan4_fwd(const srl::scan4::SP&, hipStream_t);
void launch_scan4_bwd(const srl::scan4::SP&, hipStream_t);
int scan4_fwd_lds(int, int, int, int);
int scan4_bwd_lds(int, int, int, int);
void launch_scanp_fwd(const srl::scanp::PP&, hipStream_t);
void launch_scanp_bwd(const srl::scanp::PP&, hipStream_t);
bool scanp_supported(int, int, int, int, int, int);
int scanp_sync_words();
int scanp_fwd_grid(int, int, int);
int scanp_bwd_grid(int, int, int, int);

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_f32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

const float* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}

// ------------------------------------------------------------------ optimiser
int* guard_ptr(const c10::optional<torch::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt32 && t->is_contiguous() && t->numel() >= 3,
              "optimiser guard: contiguous int32 GPU fault block [>= 3]");
  return t->data_ptr<int>();
}

torch::Tensor flat_grad_norm(torch::Tensor g, torch::Tensor scalars, double max_norm, c10::optional<torch::Tensor> guard) {
  check_f32(g, "grad");
  check_f32(scalars, "scalars");
  TORCH_CHECK(scalars.numel() >= 4, "scalars: [step, coef, norm, skip]");
  TORCH_CHECK(g.numel() % 4 == 0, "flat grad numel must be a multiple of 4");
  const int np = 2048;
  auto partial = torch::empty({np}, g.options());
  auto out = torch::empty({}, g.options());
  launch_flat_grad_norm(g.data_ptr<float>(), g.numel(), partial.data_ptr<float>(), np, scalars.data_ptr<float>(),
                        out.data_ptr<float>(), (float)max_norm, guard_ptr(guard), cur_stream());
  return out;
}

void flat_advance(torch::Tensor scalars, c10::optional<torch::Tensor> guard) {
  check_f32(scalars, "scalars");
  TORCH_CHECK(scalars.numel() >= 4, "scalars: [step, coef, norm, skip]");
  launch_flat_advance(scalars.data_ptr<float>(), guard_ptr(guard), cur_stream());
}

void flat_adam(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, torch::Tensor scalars, double lr,
               double b1, double b2, double eps, double wd, bool decoupled) {
  for (auto* t : {&p, &g, &m, &v, &scalars}) check_f32(*t, "adam buffer");
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adam: size mismatch");
  TORCH_CHECK(p.numel() % 4 == 0, "adam: numel must be a multiple of 4");
  launch_flat_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                   scalars.data_ptr<float>(), p.numel(), (float)lr, (float)b1, (float)b2, (float)eps, (float)wd,
                   decoupled ? 1 : 0, cur_stream());
}

// ------------------------------------------------------------------ LayerNorm + act
std::vector<torch::Tensor> ln_act_fwd(torch::Tensor x, c10::optional<torch::Tensor> gamma,
                                      c10::optional<torch::Tensor> beta, double eps, int64_t act) {
  check_f32(x, "x");
  const int N = x.size(-1);
  const int M = x.numel() / N;
  auto y = torch::empty_like(x);
  auto mean = torch::empty({M}, x.options());
  auto rstd = torch::empty({M}, x.options());
  bool ok = launch_ln_act_fwd(x.data_ptr<float>(), N, y.data_ptr<float>(), N, opt_ptr(gamma), opt_ptr(beta),
                              mean.data_ptr<float>(), rstd.data_ptr<float>(), M, N, 1, (float)eps, (int)act, cur_stream());
  TORCH_CHECK(ok, "ln_act_fwd: unsupported feature size ", N);
  return {y, mean, rstd};
}

std::vector<torch::Tensor> ln_act_bwd(torch::Tensor x, torch::Tensor dy, c10::optional<torch::Tensor> gamma,
                                      c10::optional<torch::Tensor> beta, torch::Tensor mean, torch::Tensor rstd,
                                      int64_t act) {
  check_f32(x, "x");
  check_f32(dy, "dy");
  const int N = x.size(-1);
  const int M = x.numel() / N;
  auto dx = torch::empty_like(x);
  bool affine = gamma.has_value() && gamma->defined();
  torch::Tensor pdg, pdb, dg, db;
  const int grid = ln_bwd_grid(M, N, 1);
  if (affine) {
    pdg = torch::empty({grid, N}, x.options());
    pdb = torch::empty({grid, N}, x.options());
    dg = torch::empty({N}, x.options());
    db = torch::empty({N}, x.options());
  }
  bool ok = launch_ln_act_bwd(x.data_ptr<float>(), N, dy.data_ptr<float>(), N, dx.data_ptr<float>(), N, opt_ptr(gamma),
                              opt_ptr(beta), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                              affine ? pdg.data_ptr<float>() : nullptr, affine ? pdb.data_ptr<float>() : nullptr,
                              affine ? dg.data_ptr<float>() : nullptr, affine ? db.data_ptr<float>() : nullptr, M, N, 1,
                              (int)act, cur_stream());
  TORCH_CHECK(ok, "ln_act_bwd: unsupported feature size ", N);
  return {dx, dg, db};
}

std::vector<torch::Tensor> ln_nchw_fwd(torch::Tensor x, c10::optional<torch::Tensor> gamma,
                                       c10::optional<torch::Tensor> beta, double eps, int64_t act) {
  check_f32(x, "x");
  TORCH_CHECK(x.dim() == 4, "ln_nchw expects NCHW");
  const int B = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  auto y = torch::empty_like(x);
  auto mean = torch::empty({B * HW}, x.options());
  auto rstd = torch::empty({B * HW}, x.options());
  launch_ln_nchw_fwd(x.data_ptr<float>(), opt_ptr(gamma), opt_ptr(beta), y.data_ptr<float>(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), B, C, HW, (float)eps, (int)act, cur_stream());
  return {y, mean, rstd};
}

std::vector<torch::Tensor> ln_nchw_bwd(torch::Tensor x, torch::Tensor dy, c10::optional<torch::Tensor> gamma,
                                       c10::optional<torch::Tensor> beta, torch::Tensor mean, torch::Tensor rstd,
                                       int64_t act) {
  check_f32(x, "x");
  check_f32(dy, "dy");
  const int B = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  auto dx = torch::empty_like(x);
  bool affine = gamma.has_value() && gamma->defined();
  torch::Tensor pdg, pdb, dg, db;
  if (affine) {
    const int S = ln_nchw_splits(B, HW);
    pdg = torch::empty({S, C}, x.options());
    pdb = torch::empty({S, C}, x.options());
    dg = torch::empty({C}, x.options());
    db = torch::empty({C}, x.options());
  }
  launch_ln_nchw_bwd(x.data_ptr<float>(), dy.data_ptr<float>(), opt_ptr(gamma), opt_ptr(beta), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), dx.data_ptr<float>(), affine ? pdg.data_ptr<float>() : nullptr,
                     affine ? pdb.data_ptr<float>() : nullptr, affine ? dg.data_ptr<float>() : nullptr,
                     affine ? db.data_ptr<float>() : nullptr, B, C, HW, (int)act, cur_stream());
  return {dx, dg, db};
}

// ------------------------------------------------------------------ LN-GRU
std::vector<torch::Tensor> ln_gru_fwd(torch::Tensor x, torch::Tensor h, torch::Tensor gamma, torch::Tensor beta,
                                      double eps) {
  check_f32(x, "x");
  check_f32(h, "h");
  check_f32(gamma, "gamma");
  check_f32(beta, "beta");
  const int H = h.size(-1);
  const int M = h.numel() / H;
  TORCH_CHECK(x.size(-1) == 3 * H && x.numel() == (int64_t)M * 3 * H, "ln_gru: x must be [M, 3H]");
  auto hn = torch::empty_like(h);
  auto mean = torch::empty({M}, x.options());
  auto rstd = torch::empty({M}, x.options());
  bool ok = launch_ln_gru_fwd(x.data_ptr<float>(), h.data_ptr<float>(), H, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                              hn.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), M, H, (float)eps,
                              cur_stream());
  TORCH_CHECK(ok, "ln_gru_fwd: unsupported hidden size ", H);
  return {hn, mean, rstd};
}

std::vector<torch::Tensor> ln_gru_bwd(torch::Tensor x, torch::Tensor h, torch::Tensor gamma, torch::Tensor beta,
                                      torch::Tensor mean, torch::Tensor rstd, torch::Tensor dhn) {
  check_f32(dhn, "dhn");
  const int H = h.size(-1);
  const int M = h.numel() / H;
  auto dx = torch::empty_like(x);
  auto dh = torch::empty_like(h);
  const int grid = ln_gru_bwd_grid(M);
  auto pdg = torch::empty({grid, 3 * H}, x.options());
  auto pdb = torch::empty({grid, 3 * H}, x.options());
  auto dg = torch::empty({3 * H}, x.options());
  auto db = torch::empty({3 * H}, x.options());
  bool ok = launch_ln_gru_bwd(x.data_ptr<float>(), h.data_ptr<float>(), H, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                              mean.data_ptr<float>(), rstd.data_ptr<float>(), dhn.data_ptr<float>(), dx.data_ptr<float>(),
                              dh.data_ptr<float>(), pdg.data_ptr<float>(), pdb.data_ptr<float>(), dg.data_ptr<float>(),
                              db.data_ptr<float>(), M, H, cur_stream());
  TORCH_CHECK(ok, "ln_gru_bwd: unsupported hidden size ", H);
  return {dx, dh, dg, db};
}

// ------------------------------------------------------------------ tanh-squashed Gaussian (SAC heads)
std::vector<torch::Tensor> squashed_gaussian_fwd(torch::Tensor mean, torch::Tensor raw, torch::Tensor eps,
                                                 torch::Tensor scale, torch::Tensor bias, int64_t mode, double lo,
                                                 double hi) {
  check_f32(mean, "mean");
  check_f32(raw, "log_std");
  check_f32(eps, "eps");
  check_f32(scale, "scale");
  check_f32(bias, "bias");
  const int A = mean.size(-1);
  TORCH_CHECK(A >= 1 && A <= 64, "squashed_gaussian: action dim must be in [1, 64], got ", A);
  TORCH_CHECK(raw.sizes() == mean.sizes() && eps.sizes() == mean.sizes(), "squashed_gaussian: shape mismatch");
  TORCH_CHECK(scale.numel() == A && bias.numel() == A, "squashed_gaussian: scale/bias must have A elements");
  const int R = mean.numel() / A;
  auto action = torch::empty_like(mean);
  auto sizes = mean.sizes().vec();
  sizes.back() = 1;
  auto logp = torch::empty(sizes, mean.options());
  launch_squashed_gaussian_fwd(mean.data_ptr<float>(), raw.data_ptr<float>(), eps.data_ptr<float>(),
                               scale.data_ptr<float>(), bias.data_ptr<float>(), action.data_ptr<float>(),
                               logp.data_ptr<float>(), R, A, (int)mode, (float)lo, (float)hi, cur_stream());
  return {action, logp};
}

std::vector<torch::Tensor> squashed_gaussian_bwd(torch::Tensor mean, torch::Tensor raw, torch::Tensor eps,
                                                 torch::Tensor scale, c10::optional<torch::Tensor> ga,
                                                 c10::optional<torch::Tensor> glp, int64_t mode, double lo, double hi) {
  const int A = mean.size(-1);
  const int R = mean.numel() / A;
  if (ga.has_value() && ga->defined()) check_f32(*ga, "grad_action");
  if (glp.has_value() && glp->defined()) {
    check_f32(*glp, "grad_logp");
    TORCH_CHECK(glp->numel() == R, "grad_logp must have one value per row");
  }
  auto dmean = torch::empty_like(mean);
  auto draw = torch::empty_like(raw);
  launch_squashed_gaussian_bwd(mean.data_ptr<float>(), raw.data_ptr<float>(), eps.data_ptr<float>(),
                               scale.data_ptr<float>(), opt_ptr(ga), opt_ptr(glp), dmean.data_ptr<float>(),
                               draw.data_ptr<float>(), R, A, (int)mode, (float)lo, (float)hi, cur_stream());
  return {dmean, draw};
}

// ------------------------------------------------------------------ distributions
std::vector<torch::Tensor> unimix_sample_fwd(torch::Tensor logits, c10::optional<torch::Tensor> uniform, int64_t C,
                                             double alpha) {
  check_f32(logits, "logits");
  const int R = logits.numel() / C;
  if (uniform.has_value() && uniform->defined()) {
    check_f32(*uniform, "uniform");
    TORCH_CHECK(uniform->numel() == R, "uniform must have one value per categorical");
  }
  auto mixed = torch::empty_like(logits);
  auto sample = torch::empty_like(logits);
  bool ok = launch_unimix_sample_fwd(logits.data_ptr<float>(), opt_ptr(uniform), mixed.data_ptr<float>(),
                                     sample.data_ptr<float>(), R, (int)C, (float)alpha, cur_stream());
  TORCH_CHECK(ok, "unimix_sample: too many classes ", C);
  return {mixed, sample};
}

torch::Tensor unimix_sample_bwd(torch::Tensor logits, c10::optional<torch::Tensor> g_mixed,
                                c10::optional<torch::Tensor> g_sample, int64_t C, double alpha) {
  const int R = logits.numel() / C;
  auto dl = torch::empty_like(logits);
  bool ok = launch_unimix_sample_bwd(logits.data_ptr<float>(), opt_ptr(g_mixed), opt_ptr(g_sample), dl.data_ptr<float>(),
                                     R, (int)C, (float)alpha, cur_stream());
  TORCH_CHECK(ok, "unimix_sample_bwd: too many classes ", C);
  return dl;
}

torch::Tensor twohot_nll_fwd(torch::Tensor logits, torch::Tensor y, torch::Tensor bins) {
  check_f32(logits, "logits");
  check_f32(y, "y");
  check_f32(bins, "bins");
  const int K = logits.size(-1);
  const int R = logits.numel() / K;
  TORCH_CHECK(y.numel() == R && bins.numel() == K, "twohot_nll: shape mismatch");
  auto loss = torch::empty({R}, logits.options());
  bool ok = launch_twohot_nll_fwd(logits.data_ptr<float>(), y.data_ptr<float>(), bins.data_ptr<float>(),
                                  loss.data_ptr<float>(), R, K, cur_stream());
  TORCH_CHECK(ok, "twohot: too many bins ", K);
  return loss;
}

// critic objective mean_r w_r (nll(l_r, y1_r) + nll(l_r, y2_r)) and its logits gradient, one pass (dist.hip)
std::vector<torch::Tensor> value_loss2(torch::Tensor logits, torch::Tensor y1, torch::Tensor y2, torch::Tensor w,
                                       torch::Tensor bins) {
  for (auto* t : {&logits, &y1, &y2, &w, &bins})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous(), "value_loss2: contiguous fp32 GPU tensors");
  const int64_t K = logits.size(-1), R = logits.numel() / K;
  TORCH_CHECK(y1.numel() == R && y2.numel() == R && w.numel() == R && bins.numel() == K, "value_loss2: shape mismatch");
  auto dl = torch::empty_like(logits);
  auto partial = torch::empty({(R + 3) / 4}, logits.options());
  auto loss = torch::empty({}, logits.options());
  bool ok = launch_value_loss2(logits.data_ptr<float>(), y1.data_ptr<float>(), y2.data_ptr<float>(), w.data_ptr<float>(),
                               bins.data_ptr<float>(), dl.data_ptr<float>(), partial.data_ptr<float>(), loss.data_ptr<float>(),
                               (int)R, (int)K, cur_stream());
  TORCH_CHECK(ok, "value_loss2: K > 512");
  return {loss, dl};
}

torch::Tensor twohot_nll_bwd(torch::Tensor logits, torch::Tensor y, torch::Tensor bins, torch::Tensor gl) {
  check_f32(gl, "grad");
  const int K = logits.size(-1);
  const int R = logits.numel() / K;
  auto dl = torch::empty_like(logits);
  bool ok = launch_twohot_nll_bwd(logits.data_ptr<float>(), y.data_ptr<float>(), bins.data_ptr<float>(),
                                  gl.data_ptr<float>(), dl.data_ptr<float>(), R, K, cur_stream());
  TORCH_CHECK(ok, "twohot: too many bins ", K);
  return dl;
}

std::vector<torch::Tensor> twohot_mean_fwd(torch::Tensor logits, torch::Tensor bins) {
  check_f32(logits, "logits");
  check_f32(bins, "bins");
  const int K = logits.size(-1);
  const int R = logits.numel() / K;
  auto out = torch::empty({R}, logits.options());
  auto s = torch::empty({R}, logits.options());
  bool ok = launch_twohot_mean_fwd(logits.data_ptr<float>(), bins.data_ptr<float>(), out.data_ptr<float>(),
                                   s.data_ptr<float>(), R, K, cur_stream());
  TORCH_CHECK(ok, "twohot: too many bins ", K);
  return {out, s};
}

torch::Tensor twohot_mean_bwd(torch::Tensor logits, torch::Tensor bins, torch::Tensor s, torch::Tensor gout) {
  check_f32(gout, "grad");
  const int K = logits.size(-1);
  const int R = logits.numel() / K;
  auto dl = torch::empty_like(logits);
  bool ok = launch_twohot_mean_bwd(logits.data_ptr<float>(), bins.data_ptr<float>(), s.data_ptr<float>(),
                                   gout.data_ptr<float>(), dl.data_ptr<float>(), R, K, cur_stream());
  TORCH_CHECK(ok, "twohot: too many bins ", K);
  return dl;
}

std::vector<torch::Tensor> kl_fwd(torch::Tensor a, torch::Tensor b, int64_t G, int64_t C, double dyn, double rep,
                                  double free_nats) {
  check_f32(a, "post_logits");
  check_f32(b, "prior_logits");
  TORCH_CHECK(a.numel() == b.numel(), "kl: shape mismatch");
  const int R = a.numel() / (G * C);
  auto kl = torch::empty({R}, a.options());
  auto loss = torch::empty({R}, a.options());
  auto ea = torch::empty({R}, a.options());  // per-row summed categorical entropies of a and b
  auto eb = torch::empty({R}, a.options());
  bool ok = launch_kl_fwd(a.data_ptr<float>(), b.data_ptr<float>(), kl.data_ptr<float>(), loss.data_ptr<float>(),
                          ea.data_ptr<float>(), eb.data_ptr<float>(), R, (int)G, (int)C, (float)dyn, (float)rep,
                          (float)free_nats, cur_stream());
  TORCH_CHECK(ok, "kl: too many classes ", C);
  return {kl, loss, ea, eb};
}

std::vector<torch::Tensor> kl_bwd(torch::Tensor a, torch::Tensor b, torch::Tensor kl, torch::Tensor gl, int64_t G,
                                  int64_t C, double dyn, double rep, double free_nats) {
  check_f32(gl, "grad");
  const int R = a.numel() / (G * C);
  auto da = torch::empty_like(a);
  auto db = torch::empty_like(b);
  bool ok = launch_kl_bwd(a.data_ptr<float>(), b.data_ptr<float>(), kl.data_ptr<float>(), gl.data_ptr<float>(),
                          da.data_ptr<float>(), db.data_ptr<float>(), R, (int)G, (int)C, (float)dyn, (float)rep,
                          (float)free_nats, cur_stream());
  TORCH_CHECK(ok, "kl: too many classes ", C);
  return {da, db};
}

// ------------------------------------------------------------------ scans
torch::Tensor lambda_fwd(torch::Tensor r, torch::Tensor v, torch::Tensor c, double lam) {
  for (auto* t : {&r, &v, &c}) check_f32(*t, "lambda input");
  const int H = r.size(0);
  const int M = r.numel() / H;
  auto out = torch::empty_like(r);
  launch_lambda_fwd(r.data_ptr<float>(), v.data_ptr<float>(), c.data_ptr<float>(), out.data_ptr<float>(), H, M, (float)lam,
                    cur_stream());
  return out;
}

std::vector<torch::Tensor> lambda_bwd(torch::Tensor v, torch::Tensor c, torch::Tensor ret, torch::Tensor g, double lam) {
  check_f32(g, "grad");
  const int H = v.size(0);
  const int M = v.numel() / H;
  auto dr = torch::empty_like(v), dv = torch::empty_like(v), dc = torch::empty_like(v);
  launch_lambda_bwd(v.data_ptr<float>(), c.data_ptr<float>(), ret.data_ptr<float>(), g.data_ptr<float>(),
                    dr.data_ptr<float>(), dv.data_ptr<float>(), dc.data_ptr<float>(), H, M, (float)lam, cur_stream());
  return {dr, dv, dc};
}

std::vector<torch::Tensor> gae(torch::Tensor rew, torch::Tensor val, torch::Tensor done, torch::Tensor next_value,
                               double gamma, double lam) {
  for (auto* t : {&rew, &val, &done, &next_value}) check_f32(*t, "gae input");
  const int T = rew.size(0);
  const int N = rew.numel() / T;
  TORCH_CHECK(next_value.numel() == N, "gae: next_value must have one value per env");
  auto ret = torch::empty_like(rew), adv = torch::empty_like(rew);
  launch_gae(rew.data_ptr<float>(), val.data_ptr<float>(), done.data_ptr<float>(), next_value.data_ptr<float>(),
             ret.data_ptr<float>(), adv.data_ptr<float>(), T, N, (float)gamma, (float)lam, cur_stream());
  return {ret, adv};
}


// ------------------------------------------------------------------ low-level entry points (RSSM scan)
// Pointers come from (possibly offset) views; strides are explicit so outputs can land in slices
// of persistent buffers.  No allocation happens here (hipGraph-friendly).
const float* fp(const torch::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }
float* mp(const torch::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }
const float* ofp(const c10::optional<torch::Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }
float* omp(const c10::optional<torch::Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

void ln_act_fwd_into(torch::Tensor x, int64_t ldx, torch::Tensor y, int64_t ldy, c10::optional<torch::Tensor> gamma,
                     c10::optional<torch::Tensor> beta, torch::Tensor mean, torch::Tensor rstd, int64_t M, int64_t N,
                     int64_t G, double eps, int64_t act) {
  TORCH_CHECK(x.is_cuda() && y.is_cuda(), "ln_act_fwd_into: GPU tensors required");
  bool ok = launch_ln_act_fwd(fp(x), ldx, mp(y), ldy, ofp(gamma), ofp(beta), mp(mean), mp(rstd), M, N, G, (float)eps,
                              (int)act, cur_stream());
  TORCH_CHECK(ok, "ln_act_fwd_into: unsupported N/G ", N, "/", G);
}

void ln_act_bwd_into(torch::Tensor x, int64_t ldx, torch::Tensor dy, int64_t lddy, torch::Tensor dx, int64_t lddx,
                     c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta, torch::Tensor mean,
                     torch::Tensor rstd, c10::optional<torch::Tensor> pdg, c10::optional<torch::Tensor> pdb,
                     c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta, int64_t M, int64_t N,
                     int64_t G, int64_t act) {
  bool ok = launch_ln_act_bwd(fp(x), ldx, fp(dy), lddy, mp(dx), lddx, ofp(gamma), ofp(beta), fp(mean), fp(rstd), omp(pdg),
                              omp(pdb), omp(dgamma), omp(dbeta), M, N, G, (int)act, cur_stream());
  TORCH_CHECK(ok, "ln_act_bwd_into: unsupported N/G ", N, "/", G);
}

// column-sum workspace (float32) + ticket counters (int32 zeros) on the current device; None, None: detach
void set_colsum_workspace_py(c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> cnt) {
  if (!ws.has_value() || !ws->defined()) {
    set_colsum_workspace(nullptr, 0, nullptr, 0);
    return;
  }
  TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == torch::kFloat32 && ws->is_contiguous(), "colsum workspace: float32 GPU");
  TORCH_CHECK(cnt.has_value() && cnt->is_cuda() && cnt->scalar_type() == torch::kInt32 && cnt->is_contiguous() &&
                  cnt->device() == ws->device(), "colsum counters: int32 zeros on the workspace's device");
  set_colsum_workspace(ws->data_ptr<float>(), ws->numel(), cnt->data_ptr<int>(), cnt->numel());
}

int64_t ln_bwd_grid_py(int64_t M, int64_t N, int64_t G) { return ln_bwd_grid(M, N, G); }
int64_t ln_gru_bwd_grid_py(int64_t M) { return ln_gru_bwd_grid(M); }

void ln_gru_fwd_into(torch::Tensor x, torch::Tensor h, int64_t ldh, torch::Tensor gamma, torch::Tensor beta,
                     torch::Tensor hn, torch::Tensor mean, torch::Tensor rstd, int64_t M, int64_t H, double eps) {
  bool ok = launch_ln_gru_fwd(fp(x), fp(h), ldh, fp(gamma), fp(beta), mp(hn), mp(mean), mp(rstd), M, H, (float)eps,
                              cur_stream());
  TORCH_CHECK(ok, "ln_gru_fwd_into: unsupported H ", H);
}

void ln_gru_bwd_into(torch::Tensor x, torch::Tensor h, int64_t ldh, torch::Tensor gamma, torch::Tensor beta,
                     torch::Tensor mean, torch::Tensor rstd, torch::Tensor dhn, torch::Tensor dx, torch::Tensor dh,
                     torch::Tensor pdg, torch::Tensor pdb, c10::optional<torch::Tensor> dgamma,
                     c10::optional<torch::Tensor> dbeta, int64_t M, int64_t H, c10::optional<torch::Tensor> dadd) {
  // dadd (optional, [M, H] row-strided): added to the dh output (a second gradient into h_{t-1})
  const float* ap = nullptr;
  int ldadd = 0;
  if (dadd.has_value() && dadd->defined()) {
    TORCH_CHECK(dadd->is_cuda() && dadd->scalar_type() == torch::kFloat32 && dadd->dim() == 2 && dadd->size(0) == M &&
                    dadd->size(1) == H && dadd->stride(1) == 1,
                "ln_gru_bwd_into: dadd must be a row-strided [M, H] float32 view");
    ap = dadd->data_ptr<float>();
    ldadd = (int)dadd->stride(0);
  }
  bool ok = launch_ln_gru_bwd(fp(x), fp(h), ldh, fp(gamma), fp(beta), fp(mean), fp(rstd), fp(dhn), mp(dx), mp(dh), mp(pdg),
                              mp(pdb), omp(dgamma), omp(dbeta), M, H, cur_stream(), ap, ldadd);
  TORCH_CHECK(ok, "ln_gru_bwd_into: unsupported H ", H);
}

void colsum2(torch::Tensor pa, torch::Tensor pb, torch::Tensor oa, torch::Tensor ob, int64_t rows, int64_t N, int64_t G) {
  launch_colsum2(fp(pa), fp(pb), mp(oa), mp(ob), rows, N, G, cur_stream());
}

void rssm_mask_fwd(c10::optional<torch::Tensor> h, int64_t ldh_in, c10::optional<torch::Tensor> z, torch::Tensor first,
                   torch::Tensor z0, torch::Tensor hout, int64_t ldh_out, torch::Tensor zout, int64_t B, int64_t H, int64_t S) {
  launch_rssm_mask_fwd(ofp(h), ldh_in, ofp(z), fp(first), fp(z0), mp(hout), ldh_out, mp(zout), B, H, S, cur_stream());
}

void rssm_mask_bwd(torch::Tensor dha, int64_t ldha, torch::Tensor dhb, int64_t ldhb, torch::Tensor dz, torch::Tensor first,
                   torch::Tensor dh_acc, torch::Tensor dz_acc, int64_t B, int64_t H, int64_t S) {
  launch_rssm_mask_bwd(fp(dha), ldha, fp(dhb), ldhb, fp(dz), fp(first), mp(dh_acc), mp(dz_acc), B, H, S, cur_stream());
}

void unimix_sample_fwd_into(torch::Tensor logits, c10::optional<torch::Tensor> uniform, torch::Tensor mixed,
                            torch::Tensor sample, int64_t C, double alpha) {
  const int R = logits.numel() / C;
  bool ok = launch_unimix_sample_fwd(fp(logits), ofp(uniform), mp(mixed), mp(sample), R, (int)C, (float)alpha, cur_stream());
  TORCH_CHECK(ok, "unimix_sample_fwd_into: too many classes ", C);
}

void unimix_sample_bwd_into(torch::Tensor logits, c10::optional<torch::Tensor> g_mixed, c10::optional<torch::Tensor> g_sample,
                            torch::Tensor dl, int64_t C, double alpha) {
  const int R = logits.numel() / C;
  bool ok = launch_unimix_sample_bwd(fp(logits), ofp(g_mixed), ofp(g_sample), mp(dl), R, (int)C, (float)alpha, cur_stream());
  TORCH_CHECK(ok, "unimix_sample_bwd_into: too many classes ", C);
}

// ------------------------------------------------------------------ 4-launch RSSM scan
// tensors (fixed order, see ops/rssm.py RSSMScan4Fn): 32 forward buffers, then 20 backward ones;
// an undefined / empty tensor is a null pointer.
srl::scan4::SP scan4_params(const std::vector<torch::Tensor>& ts, const std::vector<int64_t>& ints,
                            const std::vector<double>& fl) {
  TORCH_CHECK(ints.size() == 9 && fl.size() == 4, "scan4: bad scalar arguments");
  srl::scan4::SP p{};
  p.T = ints[0]; p.B = ints[1]; p.S = ints[2]; p.D = ints[3]; p.H = ints[4]; p.hid = ints[5]; p.C = ints[6];
  p.act1 = ints[7]; p.act2 = ints[8];
  p.alpha = fl[0]; p.eps1 = fl[1]; p.epsg = fl[2]; p.eps2 = fl[3];
  TORCH_CHECK(p.B >= 1 && p.B <= 16, "scan4: batch must be <= 16");
  TORCH_CHECK(p.H <= 512, "scan4: recurrent size must be <= 512");
  TORCH_CHECK(p.S % 32 == 0 && p.D % 16 == 0 && p.H % 16 == 0 && p.hid % 16 == 0, "scan4: dims must be multiples of 16/32");
  TORCH_CHECK(p.C >= 1 && p.C <= 32 && (32 % p.C) == 0, "scan4: classes must divide 32");
  auto P = [&](size_t i) -> float* {
    if (i >= ts.size() || !ts[i].defined() || ts[i].numel() == 0) return nullptr;
    TORCH_CHECK(ts[i].is_cuda() && ts[i].scalar_type() == torch::kFloat32 && ts[i].is_contiguous(),
                "scan4: tensor ", i, " must be a contiguous float32 GPU tensor");
    return ts[i].data_ptr<float>();
  };
  size_t k = 0;
  p.a_proj = P(k++); p.P = P(k++); p.first = P(k++); p.uni = P(k++); p.z0 = P(k++); p.Wz = P(k++); p.ln1w = P(k++);
  p.ln1b = P(k++); p.Wg = P(k++); p.lngw = P(k++); p.lngb = P(k++); p.W1 = P(k++); p.ln2w = P(k++); p.ln2b = P(k++);
  p.W2 = P(k++); p.b2 = P(k++);
  p.cat = P(k++); p.zm = P(k++); p.xr = P(k++); p.m1 = P(k++); p.r1 = P(k++); p.gx = P(k++); p.mg = P(k++); p.rg = P(k++);
  p.hs = P(k++); p.u = P(k++); p.v = P(k++); p.m2 = P(k++); p.r2 = P(k++); p.logits = P(k++); p.mixed = P(k++);
  p.samples = P(k++);
  p.WzT = P(k++); p.WgT = P(k++); p.W1T = P(k++); p.W2T = P(k++); p.dpost = P(k++); p.dmixed = P(k++);
  p.DH = P(k++); p.dlog = P(k++); p.dv = P(k++); p.du = P(k++); p.dgx = P(k++); p.dx = P(k++); p.dcat = P(k++);
  p.dhp = P(k++); p.p1g = P(k++); p.p1b = P(k++); p.pgg = P(k++); p.pgb = P(k++); p.p2g = P(k++); p.p2b = P(k++);
  p.prof = nullptr;
  return p;
}

long long* g_scan4_prof = nullptr;  // debug phase timestamps (set_scan4_prof)

void set_scan4_prof(c10::optional<torch::Tensor> buf) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->scalar_type() == torch::kInt64 && buf->numel() >= 128 && buf->is_cuda(), "prof buffer: int64[128] on GPU");
    g_scan4_prof = (long long*)buf->data_ptr<int64_t>();
  } else {
    g_scan4_prof = nullptr;
  }
}

void scan4_fwd(const std::vector<torch::Tensor>& ts, const std::vector<int64_t>& ints, const std::vector<double>& fl,
               torch::Tensor WzT, torch::Tensor c0, torch::Tensor sel) {
  TORCH_CHECK(ts.size() == 32, "scan4_fwd: expects 32 tensors");
  auto p = scan4_params(ts, ints, fl);
  p.prof = g_scan4_prof;
  TORCH_CHECK(p.uni && p.z0 && p.logits && p.samples, "scan4_fwd: missing tensors");
  check_f32(WzT, "WzT");
  check_f32(c0, "c0");
  TORCH_CHECK(WzT.size(0) == p.S && WzT.size(1) == p.D && c0.numel() == p.D, "scan4_fwd: WzT [S, D] / c0 [D]");
  p.WzT = WzT.data_ptr<float>();
  p.c0 = c0.data_ptr<float>();
  TORCH_CHECK(sel.is_cuda() && sel.scalar_type() == torch::kInt32 && sel.is_contiguous() &&
                  sel.numel() >= (int64_t)p.T * 16 * (p.S / p.C) && p.D % 4 == 0,
              "scan4_fwd: sel must be int32 [T, 16, S / C]");
  p.sel = sel.data_ptr<int>();
  launch_scan4_fwd(p, cur_stream());
}

void scan4_bwd(const std::vector<torch::Tensor>& ts, const std::vector<int64_t>& ints, const std::vector<double>& fl) {
  TORCH_CHECK(ts.size() == 52, "scan4_bwd: expects 52 tensors");
  auto p = scan4_params(ts, ints, fl);
  p.prof = g_scan4_prof;
  TORCH_CHECK(p.dmixed && p.DH && p.dlog && p.WzT, "scan4_bwd: missing tensors");
  launch_scan4_bwd(p, cur_stream());
}

int64_t scan4_lds(int64_t S, int64_t D, int64_t H, int64_t hid) {
  int a = scan4_fwd_lds(S, D, H, hid), b = scan4_bwd_lds(S, D, H, hid);
  return a > b ? a : b;
}

// ------------------------------------------------------------------ persistent RSSM posterior scan
// tensors (fixed order, see ops/rssm.py RSSMPersistFn): 33 forward buffers + the int32 sample table and hand-off
// counter block, then 20 backward ones; an undefined / empty tensor is a null pointer.
srl::scanp::PP scanp_params(const std::vector<torch::Tensor>& ts, const std::vector<int64_t>& ints,
                            const std::vector<double>& fl) {
  TORCH_CHECK(ints.size() == 9 && fl.size() == 4, "scanp: bad scalar arguments");
  srl::scanp::PP p{};
  p.T = ints[0]; p.B = ints[1]; p.S = ints[2]; p.D = ints[3]; p.H = ints[4]; p.hid = ints[5]; p.C = ints[6];
  p.act1 = ints[7]; p.act2 = ints[8];
  p.alpha = fl[0]; p.eps1 = fl[1]; p.epsg = fl[2]; p.eps2 = fl[3];
  TORCH_CHECK(scanp_supported(p.B, p.S, p.D, p.H, p.hid, p.C), "scanp: unsupported shape B=", p.B, " S=", p.S, " D=", p.D,
              " H=", p.H, " hid=", p.hid, " C=", p.C);
  auto P = [&](size_t i) -> float* {
    if (i >= ts.size() || !ts[i].defined() || ts[i].numel() == 0) return nullptr;
    TORCH_CHECK(ts[i].is_cuda() && ts[i].scalar_type() == torch::kFloat32 && ts[i].is_contiguous(),
                "scanp: tensor ", i, " must be a contiguous float32 GPU tensor");
    return ts[i].data_ptr<float>();
  };
  size_t k = 0;
  p.P = P(k++); p.first = P(k++); p.uni = P(k++); p.z0 = P(k++); p.Wz = P(k++); p.WzT = P(k++); p.ln1w = P(k++);
  p.ln1b = P(k++); p.Wg = P(k++); p.lngw = P(k++); p.lngb = P(k++); p.W1 = P(k++); p.ln2w = P(k++); p.ln2b = P(k++);
  p.W2 = P(k++); p.b2 = P(k++);
  p.xr = P(k++); p.cat = P(k++); p.zm = P(k++); p.m1 = P(k++); p.r1 = P(k++); p.gx = P(k++); p.gst = P(k++); p.mg = P(k++);
  p.rg = P(k++); p.hs = P(k++); p.u = P(k++); p.v = P(k++); p.m2 = P(k++); p.r2 = P(k++); p.logits = P(k++);
  p.mixed = P(k++); p.samples = P(k++);
  const torch::Tensor& sel = ts.at(k++);
  TORCH_CHECK(sel.is_cuda() && sel.scalar_type() == torch::kInt32 && sel.is_contiguous() && sel.numel() >= p.T * p.B * (p.S / p.C),
              "scanp: sel must be int32 [T, B, S/C] on the GPU");
  p.sel = sel.data_ptr<int32_t>();
  const torch::Tensor& sync = ts.at(k++);
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == torch::kInt32 && sync.is_contiguous() &&
                  sync.numel() >= scanp_sync_words(), "scanp: sync must be int32[", scanp_sync_words(), "] on the GPU");
  p.sync = (unsigned*)sync.data_ptr<int32_t>();
  p.W2T = P(k++); p.W1T = P(k++); p.WgT = P(k++); p.dpost = P(k++); p.dmixed = P(k++);
  p.DH = P(k++); p.dlog = P(k++); p.dv = P(k++); p.du = P(k++); p.dgx = P(k++); p.dcat = P(k++); p.dx = P(k++);
  // the LayerNorm parameter partials: [T, n] column slices (unit column stride) of one buffer, so the host
  // reduces all six with ONE column sum
  p.ldp = 0;
  auto PL = [&](size_t i, int64_t n) -> float* {
    if (i >= ts.size() || !ts[i].defined() || ts[i].numel() == 0) return nullptr;
    const torch::Tensor& t = ts[i];
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.dim() == 2 && t.size(0) == p.T && t.size(1) == n &&
                    t.stride(1) == 1, "scanp: LN partial ", i, " must be a float32 [T, ", n, "] GPU view with unit column stride");
    TORCH_CHECK(p.ldp == 0 || p.ldp == t.stride(0), "scanp: the LN partials must share one row stride");
    p.ldp = t.stride(0);
    return t.data_ptr<float>();
  };
  p.p1g = PL(k++, p.D); p.p1b = PL(k++, p.D); p.pgg = PL(k++, 3 * p.H); p.pgb = PL(k++, 3 * p.H);
  p.p2g = PL(k++, p.hid); p.p2b = PL(k++, p.hid);
  p.dZ = P(k++); p.sst = P(k++);
  return p;
}

long long* g_scanp_prof = nullptr;  // debug phase timestamps (set_scanp_prof)
unsigned* g_scanp_health = nullptr;  // sticky timeout word shared by every launch (set_scanp_health)

unsigned g_scanp_spin = 0;           // spin bound of the hand-off waits (0 = kernel default; tests force timeouts)

void set_scanp_health(c10::optional<torch::Tensor> buf, int64_t spin_max) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->scalar_type() == torch::kInt32 && buf->is_cuda() && buf->numel() >= 1, "health word: int32 [1] on GPU");
    g_scanp_health = (unsigned*)buf->data_ptr<int32_t>();
  } else {
    g_scanp_health = nullptr;
  }
  g_scanp_spin = (unsigned)std::max<int64_t>(0, spin_max);
}

void set_scanp_prof(c10::optional<torch::Tensor> buf) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->scalar_type() == torch::kInt64 && buf->is_cuda(), "prof buffer: int64 [7 * T * 8] on GPU");
    g_scanp_prof = (long long*)buf->data_ptr<int64_t>();
  } else {
    g_scanp_prof = nullptr;
  }
}

void scanp_fwd(const std::vector<torch::Tensor>& ts, const std::vector<int64_t>& ints, const std::vector<double>& fl) {
  TORCH_CHECK(ts.size() == 35, "scanp_fwd: expects 35 tensors");
  auto p = scanp_params(ts, ints, fl);
  p.prof = g_scanp_prof;
  p.health = g_scanp_health;
  p.spin_max = g_scanp_spin;
  TORCH_CHECK(p.P && p.first && p.uni && p.z0 && p.WzT && p.Wg && p.W1 && p.W2 && p.xr && p.hs && p.u && p.samples,
              "scanp_fwd: missing tensors");
  launch_scanp_fwd(p, cur_stream());
}

void scanp_bwd(const std::vector<torch::Tensor>& ts, const std::vector<int64_t>& ints, const std::vector<double>& fl) {
  TORCH_CHECK(ts.size() == 55, "scanp_bwd: expects 55 tensors");
  auto p = scanp_params(ts, ints, fl);
  p.prof = g_scanp_prof;
  p.health = g_scanp_health;
  p.spin_max = g_scanp_spin;
  TORCH_CHECK(p.W2T && p.W1T && p.WgT && p.dmixed && p.DH && p.dlog && p.dv && p.du && p.dgx && p.dcat && p.dx && p.dZ && p.sst,
              "scanp_bwd: missing tensors");
  launch_scanp_bwd(p, cur_stream());
}

// ------------------------------------------------------------------ truncated normal (ops.truncnorm_*)
void tn_check(const torch::Tensor& loc, const torch::Tensor& scale, const torch::Tensor& lo, const torch::Tensor& hi) {
  check_f32(loc, "loc");
  check_f32(scale, "scale");
  check_f32(lo, "lo");
  check_f32(hi, "hi");
  TORCH_CHECK(scale.numel() == loc.numel(), "truncnorm: loc / scale sizes differ");
  TORCH_CHECK(lo.numel() == 1 || lo.numel() == loc.numel(), "truncnorm: lo must be a scalar or loc-shaped");
  TORCH_CHECK(hi.numel() == 1 || hi.numel() == loc.numel(), "truncnorm: hi must be a scalar or loc-shaped");
}

torch::Tensor truncnorm_rsample_fwd(torch::Tensor loc, torch::Tensor scale, torch::Tensor lo, torch::Tensor hi, torch::Tensor u) {
  tn_check(loc, scale, lo, hi);
  check_f32(u, "u");
  TORCH_CHECK(u.numel() == loc.numel(), "truncnorm: u must be loc-shaped");
  auto x = torch::empty_like(loc);
  launch_truncnorm_rsample_fwd(loc.data_ptr<float>(), scale.data_ptr<float>(), lo.data_ptr<float>(), (int)lo.numel(),
                               hi.data_ptr<float>(), (int)hi.numel(), u.data_ptr<float>(), x.data_ptr<float>(), (int)loc.numel(),
                               cur_stream());
  return x;
}

std::vector<torch::Tensor> truncnorm_rsample_bwd(torch::Tensor loc, torch::Tensor scale, torch::Tensor lo, torch::Tensor hi,
                                                 torch::Tensor u, torch::Tensor gx) {
  tn_check(loc, scale, lo, hi);
  check_f32(u, "u");
  check_f32(gx, "gx");
  auto gl = torch::empty_like(loc), gs = torch::empty_like(loc);
  launch_truncnorm_rsample_bwd(loc.data_ptr<float>(), scale.data_ptr<float>(), lo.data_ptr<float>(), (int)lo.numel(),
                               hi.data_ptr<float>(), (int)hi.numel(), u.data_ptr<float>(), gx.data_ptr<float>(),
                               gl.data_ptr<float>(), gs.data_ptr<float>(), (int)loc.numel(), cur_stream());
  return {gl, gs};
}

torch::Tensor truncnorm_logprob_fwd(torch::Tensor v, torch::Tensor loc, torch::Tensor scale, torch::Tensor lo, torch::Tensor hi) {
  tn_check(loc, scale, lo, hi);
  check_f32(v, "value");
  TORCH_CHECK(v.numel() % loc.numel() == 0, "truncnorm: value must be [sample..., *loc.shape]");
  auto lp = torch::empty_like(v);
  launch_truncnorm_logprob_fwd(v.data_ptr<float>(), loc.data_ptr<float>(), scale.data_ptr<float>(), lo.data_ptr<float>(),
                               (int)lo.numel(), hi.data_ptr<float>(), (int)hi.numel(), lp.data_ptr<float>(), (int)v.numel(),
                               (int)loc.numel(), cur_stream());
  return lp;
}

std::vector<torch::Tensor> truncnorm_logprob_bwd(torch::Tensor v, torch::Tensor loc, torch::Tensor scale, torch::Tensor lo,
                                                 torch::Tensor hi, torch::Tensor g) {
  tn_check(loc, scale, lo, hi);
  check_f32(v, "value");
  check_f32(g, "grad");
  auto gv = torch::empty_like(v), gl = torch::empty_like(v), gs = torch::empty_like(v);
  launch_truncnorm_logprob_bwd(v.data_ptr<float>(), loc.data_ptr<float>(), scale.data_ptr<float>(), lo.data_ptr<float>(),
                               (int)lo.numel(), hi.data_ptr<float>(), (int)hi.numel(), g.data_ptr<float>(), gv.data_ptr<float>(),
                               gl.data_ptr<float>(), gs.data_ptr<float>(), (int)v.numel(), (int)loc.numel(), cur_stream());
  return {gv, gl, gs};
}

// DreamerV3 trunc_normal actor head: pre [M, 2A] (row-strided) -> loc, scale [M, A] and the sample into x
// (row-strided [M, A] view); uniforms u [M, A].
void tn_head_sample_fwd(torch::Tensor pre, torch::Tensor u, double init_std, double min_std, double lo, double hi,
                        torch::Tensor loc, torch::Tensor scale, torch::Tensor x) {
  check_f32(pre, "pre");
  check_f32(u, "u");
  TORCH_CHECK(pre.dim() == 2 && pre.stride(1) == 1 && x.dim() == 2 && x.stride(1) == 1, "tn_head_sample: 2-D row-strided views");
  const int M = pre.size(0), A = pre.size(1) / 2;
  TORCH_CHECK(pre.size(1) == 2 * A && x.size(0) == M && x.size(1) == A && u.numel() == (int64_t)M * A &&
                  loc.numel() == (int64_t)M * A && scale.numel() == (int64_t)M * A && loc.is_contiguous() && scale.is_contiguous() &&
                  u.is_contiguous(),
              "tn_head_sample_fwd: shapes");
  launch_tn_head_sample_fwd(fp(pre), pre.stride(0), fp(u), (float)init_std, (float)min_std, (float)lo, (float)hi, mp(loc),
                            mp(scale), mp(x), x.stride(0), M, A, cur_stream());
}

// The same with the head Linear folded in: y [M, K] (row-strided), W [2A, K], b [2A] (optional) -> pre [M, 2A]
// (contiguous), loc, scale [M, A], the sample into x.  False: shape outside the kernel (caller keeps GEMM + sample).
bool tn_head_linear_sample_fwd(torch::Tensor y, torch::Tensor W, c10::optional<torch::Tensor> b, torch::Tensor u,
                               double init_std, double min_std, double lo, double hi, torch::Tensor pre, torch::Tensor loc,
                               torch::Tensor scale, torch::Tensor x, c10::optional<torch::Tensor> ln_w,
                               c10::optional<torch::Tensor> ln_b, double ln_eps, int64_t act, c10::optional<torch::Tensor> y_out,
                               c10::optional<torch::Tensor> mean, c10::optional<torch::Tensor> rstd) {
  check_f32(W, "W");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == torch::kFloat32 && y.dim() == 2 && y.stride(1) == 1 && W.dim() == 2 &&
                  x.dim() == 2 && x.stride(1) == 1,
              "tn_head_linear_sample: 2-D row-strided float32 y / x, contiguous W");
  const int M = y.size(0), K = y.size(1), A = W.size(0) / 2;
  TORCH_CHECK(W.size(0) == 2 * A && W.size(1) == K && pre.is_contiguous() && pre.numel() == (int64_t)M * 2 * A &&
                  x.size(0) == M && x.size(1) == A && u.is_contiguous() && u.numel() == (int64_t)M * A && loc.is_contiguous() &&
                  scale.is_contiguous() && loc.numel() == (int64_t)M * A && scale.numel() == (int64_t)M * A,
              "tn_head_linear_sample_fwd: shapes");
  if (b.has_value() && b->defined()) TORCH_CHECK(b->is_contiguous() && b->numel() == 2 * A, "tn_head_linear_sample_fwd: bias");
  // optional LayerNorm + activation of y first (y = the trunk's last pre-activation): weights [K], the normalised
  // row into y_out (row-strided [M, K]), statistics into mean / rstd [M]
  const bool ln = ln_w.has_value() && ln_w->defined();
  if (ln) {
    TORCH_CHECK(ln_b.has_value() && ln_b->defined() && ln_w->numel() == K && ln_b->numel() == K && y_out.has_value() &&
                    y_out->defined() && y_out->dim() == 2 && y_out->stride(1) == 1 && y_out->size(0) == M && y_out->size(1) == K &&
                    mean.has_value() && rstd.has_value() && mean->numel() == M && rstd->numel() == M,
                "tn_head_linear_sample_fwd: LayerNorm operands");
  }
  return launch_tn_head_linear_sample_fwd(fp(y), y.stride(0), fp(W), b.has_value() && b->defined() ? fp(*b) : nullptr, fp(u),
                                          (float)init_std, (float)min_std, (float)lo, (float)hi, mp(pre), mp(loc), mp(scale),
                                          mp(x), x.stride(0), M, K, A, cur_stream(), ln ? fp(*ln_w) : nullptr,
                                          ln ? fp(*ln_b) : nullptr, (float)ln_eps, (int)act, ln ? mp(*y_out) : nullptr,
                                          ln ? y_out->stride(0) : 0, ln ? mp(*mean) : nullptr, ln ? mp(*rstd) : nullptr);
}

// d pre [M, 2A] of the head + sample above: gx = d sample (optional), dpre_in = a gradient reaching pre directly
// (optional, [M, 2A] contiguous).
torch::Tensor tn_head_sample_bwd(torch::Tensor loc, torch::Tensor scale, torch::Tensor u, c10::optional<torch::Tensor> gx,
                                 c10::optional<torch::Tensor> dpre_in, double min_std, double lo, double hi) {
  const int A = loc.size(-1);
  const int M = loc.numel() / A;
  TORCH_CHECK(loc.is_contiguous() && scale.is_contiguous() && u.is_contiguous() && scale.numel() == loc.numel() &&
                  u.numel() == loc.numel(), "tn_head_sample_bwd: loc/scale/u must be contiguous [M, A]");
  if (gx.has_value() && gx->defined()) TORCH_CHECK(gx->is_contiguous() && gx->numel() == loc.numel(), "tn_head_sample_bwd: gx");
  if (dpre_in.has_value() && dpre_in->defined())
    TORCH_CHECK(dpre_in->is_contiguous() && dpre_in->numel() == 2 * loc.numel(), "tn_head_sample_bwd: dpre_in");
  auto dpre = torch::empty({M, 2 * A}, loc.options());
  launch_tn_head_sample_bwd(fp(loc), fp(scale), fp(u), ofp(gx), ofp(dpre_in), (float)min_std, (float)lo, (float)hi, mp(dpre), M,
                            A, cur_stream());
  return dpre;
}

std::vector<int64_t> scanp_info(int64_t B, int64_t S, int64_t D, int64_t H, int64_t hid, int64_t C) {
  // [supported, sync words, error word index, forward grid, backward grid]
  const int words = scanp_sync_words();
  return {scanp_supported(B, S, D, H, hid, C) ? 1 : 0, words, words - 32, scanp_fwd_grid(S, H, hid),
          scanp_bwd_grid(S, D, H, hid)};
}

}  // namespace

// ------------------------------------------------------------------ strided-output (no-grad) forms
// Write into a caller-owned row-strided view (e.g. a slice of an imagination trajectory buffer):
// out must have unit stride in its last dim; rows may be strided.
// ``mean`` / ``rstd`` (optional [M]): keep the LayerNorm row statistics (for a later ln_gru_bwd_into).
void set_gru_vec(bool on);

void ln_gru_into(torch::Tensor x, torch::Tensor h, torch::Tensor gamma, torch::Tensor beta, double eps, torch::Tensor out,
                 c10::optional<torch::Tensor> mean_out, c10::optional<torch::Tensor> rstd_out, c10::optional<torch::Tensor> x2,
                 bool write_sum) {
  check_f32(x, "x");
  check_f32(gamma, "gamma");
  check_f32(beta, "beta");
  TORCH_CHECK(h.is_cuda() && h.dim() == 2 && h.stride(1) == 1 && out.dim() == 2 && out.stride(1) == 1,
              "ln_gru_into: h/out must be row-strided 2-D views");
  const int H = h.size(1), M = h.size(0);
  TORCH_CHECK(x.numel() == (int64_t)M * 3 * H && out.size(0) == M && out.size(1) == H, "ln_gru_into: shapes");
  const float* x2p = nullptr;
  int64_t ldx2 = 0;
  if (x2.has_value() && x2->defined()) {  // gx = x + x2: the two parts of a split GRU input GEMM
    TORCH_CHECK(x2->is_cuda() && x2->scalar_type() == torch::kFloat32 && x2->dim() == 2 && x2->size(0) == M &&
                    x2->size(1) == 3 * H && x2->stride(1) == 1,
                "ln_gru_into: x2 must be a row-strided float32 [M, 3H] view");
    x2p = x2->data_ptr<float>();
    ldx2 = x2->stride(0);
  }
  const bool keep = mean_out.has_value() && mean_out->defined() && rstd_out.has_value() && rstd_out->defined();
  if (keep) TORCH_CHECK(mean_out->numel() == M && rstd_out->numel() == M, "ln_gru_into: mean/rstd must hold M rows");
  auto mean = keep ? *mean_out : torch::empty({M}, x.options());
  auto rstd = keep ? *rstd_out : torch::empty({M}, x.options());
  bool ok = launch_ln_gru_fwd(x.data_ptr<float>(), h.data_ptr<float>(), h.stride(0), gamma.data_ptr<float>(),
                              beta.data_ptr<float>(), out.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                              M, H, (float)eps, cur_stream(), out.stride(0), x2p, (int)ldx2,
                              (write_sum && x2p) ? x.data_ptr<float>() : nullptr);
  TORCH_CHECK(ok, "ln_gru_into: unsupported hidden size ", H);
}

// ``idx`` (optional int32 [M, >= N / C] row-strided view): the hot column of each sampled categorical,
// ``idx_off + g * C + pick`` (the one-hot gather consumers of ops/csrc/onehot.hip read it).
void unimix_sample_into(torch::Tensor logits, c10::optional<torch::Tensor> uniform, int64_t classes, double alpha,
                        torch::Tensor out, c10::optional<torch::Tensor> idx, int64_t idx_off) {
  check_f32(logits, "logits");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.stride(1) == 1, "unimix_sample_into: out must be a row-strided 2-D view");
  const int C = classes, N = out.size(1), M = out.size(0);
  TORCH_CHECK(N % C == 0 && logits.numel() == (int64_t)M * N, "unimix_sample_into: shapes");
  const int R = M * (N / C);
  int* ip = nullptr;
  int ldi = 0;
  if (idx.has_value() && idx->defined()) {
    TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == torch::kInt && idx->dim() == 2 && idx->stride(1) == 1 &&
                    idx->size(0) == M && idx->size(1) >= N / C,
                "unimix_sample_into: idx must be an int32 [M, >= G] row-strided view");
    ip = idx->data_ptr<int>();
    ldi = idx->stride(0);
  }
  bool ok = launch_unimix_sample_fwd(logits.data_ptr<float>(), opt_ptr(uniform), nullptr, out.data_ptr<float>(), R, C,
                                     (float)alpha, cur_stream(), N / C, out.stride(0), ip, ldi, (int)idx_off);
  TORCH_CHECK(ok, "unimix_sample_into: classes must be <= 1024");
}

// column sums of a row-strided 2-D view [rows, N] (stride(1) == 1) -> [N]
torch::Tensor colsum(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.dim() == 2 && x.stride(1) == 1,
              "colsum: x must be a row-strided 2-D float32 GPU view");
  auto out = torch::empty({x.size(1)}, x.options());
  launch_colsum1(x.data_ptr<float>(), x.stride(0), out.data_ptr<float>(), x.size(0), x.size(1), cur_stream());
  return out;
}

// device CartPole step (envs.hip); state/steps/ep_ret are updated in place, outputs preallocated
void cartpole_step(torch::Tensor state, torch::Tensor steps, torch::Tensor ep_ret, torch::Tensor action,
                   torch::Tensor uniform, torch::Tensor obs, torch::Tensor reward, torch::Tensor terminated,
                   torch::Tensor truncated, torch::Tensor final_obs, torch::Tensor done_ret, torch::Tensor done_len,
                   int64_t max_steps) {
  const int64_t N = state.size(0);
  for (auto* t : {&state, &ep_ret, &uniform, &obs, &reward, &terminated, &truncated, &final_obs, &done_ret, &done_len})
    check_f32(*t, "cartpole buffer");
  TORCH_CHECK(state.dim() == 2 && state.size(1) == 4 && obs.numel() == 4 * N && final_obs.numel() == 4 * N &&
                  uniform.numel() == 4 * N,
              "cartpole_step: state/obs/final_obs/uniform must be [N, 4]");
  TORCH_CHECK(steps.is_cuda() && steps.scalar_type() == torch::kInt32 && steps.numel() == N, "cartpole_step: steps int32 [N]");
  TORCH_CHECK(action.is_cuda() && action.scalar_type() == torch::kInt64 && action.numel() == N && action.is_contiguous(),
              "cartpole_step: action int64 [N]");
  TORCH_CHECK(reward.numel() == N && terminated.numel() == N && truncated.numel() == N && done_ret.numel() == N &&
                  done_len.numel() == N,
              "cartpole_step: per-env outputs must have N elements");
  launch_cartpole_step(state.data_ptr<float>(), steps.data_ptr<int>(), ep_ret.data_ptr<float>(), action.data_ptr<int64_t>(),
                       uniform.data_ptr<float>(), obs.data_ptr<float>(), reward.data_ptr<float>(),
                       terminated.data_ptr<float>(), truncated.data_ptr<float>(), final_obs.data_ptr<float>(),
                       done_ret.data_ptr<float>(), done_len.data_ptr<float>(), N, max_steps, cur_stream());
}

// one-launch PPO rollout on the device CartPole (ppo_rollout.hip)
#include "ppo_rollout.h"
void launch_ppo_cartpole_rollout(const srl::RolloutArgs&, hipStream_t);

namespace {
srl::Chain make_chain(const std::vector<torch::Tensor>& W, const std::vector<c10::optional<torch::Tensor>>& b,
                      const std::vector<int64_t>& act, int64_t& lds_off) {
  TORCH_CHECK(W.size() >= 1 && W.size() <= 8 && b.size() == W.size() && act.size() == W.size(), "rollout chain: 1..8 layers");
  srl::Chain c{};
  c.n = W.size();
  for (size_t l = 0; l < W.size(); ++l) {
    check_f32(W[l], "chain weight");
    TORCH_CHECK(W[l].dim() == 2 && W[l].size(0) <= 256 && W[l].size(1) <= 256, "rollout chain: widths <= 256");
    if (l > 0) TORCH_CHECK(W[l].size(1) == W[l - 1].size(0), "rollout chain: layer widths do not chain");
    c.dout[l] = W[l].size(0);
    c.din[l] = W[l].size(1);
    c.act[l] = act[l];
    c.W[l] = W[l].data_ptr<float>();
    c.b[l] = opt_ptr(b[l]);
    c.woff[l] = (int)lds_off;
    lds_off += (int64_t)c.din[l] * c.dout[l];
    c.boff[l] = (int)lds_off;
    lds_off += (c.dout[l] + 3) & ~3;
  }
  return c;
}
}  // namespace

void ppo_cartpole_rollout(std::vector<torch::Tensor> eW, std::vector<c10::optional<torch::Tensor>> eb, std::vector<int64_t> ea,
                          std::vector<torch::Tensor> aW, std::vector<c10::optional<torch::Tensor>> ab, std::vector<int64_t> aa,
                          std::vector<torch::Tensor> hW, std::vector<c10::optional<torch::Tensor>> hb, std::vector<int64_t> ha,
                          std::vector<torch::Tensor> cW, std::vector<c10::optional<torch::Tensor>> cb, std::vector<int64_t> ca,
                          torch::Tensor state, torch::Tensor steps, torch::Tensor ep_ret, torch::Tensor obs_out,
                          std::vector<torch::Tensor> bufs, int64_t max_steps, int64_t seed, bool allow_lds) {
  srl::RolloutArgs p{};
  int64_t lds_off = 0;
  p.enc = make_chain(eW, eb, ea, lds_off);
  p.actor = make_chain(aW, ab, aa, lds_off);
  p.head = make_chain(hW, hb, ha, lds_off);
  p.critic = make_chain(cW, cb, ca, lds_off);
  p.lds_weights = allow_lds && lds_off <= srl::RO_LDSW ? 1 : 0;
  TORCH_CHECK(p.enc.din[0] == 4, "rollout: the encoder must take the 4-dim CartPole observation");
  TORCH_CHECK(p.actor.din[0] == p.enc.dout[p.enc.n - 1] && p.critic.din[0] == p.enc.dout[p.enc.n - 1] &&
                  p.head.din[0] == p.actor.dout[p.actor.n - 1] && p.critic.dout[p.critic.n - 1] == 1,
              "rollout: chain shapes");
  p.A = p.head.dout[p.head.n - 1];
  TORCH_CHECK(p.A == 2, "rollout: CartPole has 2 actions");
  check_f32(state, "state");
  check_f32(ep_ret, "ep_ret");
  check_f32(obs_out, "obs_out");
  TORCH_CHECK(steps.is_cuda() && steps.scalar_type() == torch::kInt32, "steps int32");
  p.N = state.size(0);
  TORCH_CHECK(bufs.size() == 8, "rollout: 8 buffers (state, actions, logp, values, rewards, dones, done_ret, done_len)");
  for (auto& t : bufs) check_f32(t, "rollout buffer");
  p.T = bufs[0].size(0);
  TORCH_CHECK(bufs[0].numel() == (int64_t)p.T * p.N * 4 && bufs[1].numel() == (int64_t)p.T * p.N * p.A, "rollout: buffer shapes");
  for (int i = 2; i < 8; ++i) TORCH_CHECK(bufs[i].numel() == (int64_t)p.T * p.N, "rollout: per-step buffers [T, N]");
  p.max_steps = max_steps;
  p.seed = (uint64_t)seed;
  p.state = state.data_ptr<float>();
  p.steps = steps.data_ptr<int>();
  p.ep_ret = ep_ret.data_ptr<float>();
  p.obs_out = obs_out.data_ptr<float>();
  p.b_state = bufs[0].data_ptr<float>();
  p.b_actions = bufs[1].data_ptr<float>();
  p.b_logp = bufs[2].data_ptr<float>();
  p.b_values = bufs[3].data_ptr<float>();
  p.b_rewards = bufs[4].data_ptr<float>();
  p.b_dones = bufs[5].data_ptr<float>();
  p.b_done_ret = bufs[6].data_ptr<float>();
  p.b_done_len = bufs[7].data_ptr<float>();
  launch_ppo_cartpole_rollout(p, cur_stream());
}

// one-launch PPO update for MLP agents (ppo_train.hip)
#include "ppo_train.h"
hipError_t launch_ppo_mlp_train(const srl::PTArgs&, hipStream_t);

namespace {
int r4(int x) { return (x + 3) & ~3; }

// LDS plan of the fused PPO update; false when the agent does not fit the kernel.
// layers: [din, dout, act, pw, pb] per Linear, chains in order encoder / actor / head / critic.
bool pt_plan(const std::vector<std::vector<int64_t>>& layers, const std::vector<int64_t>& counts, int D0, int A,
             srl::PTArgs& p) {
  if (counts.size() != 4) return false;
  p.ne = counts[0];
  p.na = counts[1];
  p.nh = counts[2];
  p.nc = counts[3];
  const int NL = p.ne + p.na + p.nh + p.nc;
  if (p.ne < 1 || p.na < 1 || p.nh < 1 || p.nc < 1 || NL > srl::PT_MAXL || (int)layers.size() != NL) return false;
  int off = 0, tiles = 0, wmax = D0;
  for (int l = 0; l < NL; ++l) {
    const auto& d = layers[l];
    if (d.size() != 5) return false;
    srl::PTLayer& L = p.L[l];
    L.din = d[0];
    L.dout = d[1];
    L.act = d[2];
    L.pw = d[3];
    L.pb = d[4];
    if (L.act != 0 && L.act != 2 && L.act != 3 && L.act != 4) return false;  // none, elu, relu, tanh (common.h Act)
    if (L.din < 1 || L.dout < 1 || L.din > 256 || L.dout > 256) return false;
    L.k4 = r4(L.din + 1);
    L.ldw = r4(L.dout) + 4;
    L.wt = off;
    off += L.k4 * L.ldw;
    L.tile0 = tiles;
    L.tj = (L.dout + 3) / 4;
    L.tk = L.k4 / 4;
    tiles += L.tj * L.tk;
    wmax = std::max(wmax, std::max(L.din, L.dout));
  }
  p.ntiles = tiles;
  if (tiles > srl::PT_THREADS * srl::PT_MAXT) return false;
  // activation buffers: observation, then every layer's output
  p.node_lo = off;
  const int obs_node = off, obs_ld = r4(D0 + 1);
  off += srl::PT_R * obs_ld;
  for (int l = 0; l < NL; ++l) {
    p.L[l].out_node = off;
    p.L[l].out_ld = r4(p.L[l].dout + 1);
    off += srl::PT_R * p.L[l].out_ld;
  }
  const int e_last = p.ne - 1, a0 = p.ne, h0 = p.ne + p.na, c0 = p.ne + p.na + p.nh;
  for (int l = 0; l < NL; ++l) {
    srl::PTLayer& L = p.L[l];
    int src = l - 1;
    if (l == 0) src = -1;
    else if (l == a0 || l == c0) src = e_last;
    if (src < 0) {
      L.in_node = obs_node;
      L.in_ld = obs_ld;
      L.in_act = -1;
      if (L.din != D0) return false;
    } else {
      L.in_node = p.L[src].out_node;
      L.in_ld = p.L[src].out_ld;
      L.in_act = p.L[src].act;
      if (L.din != p.L[src].dout) return false;
    }
  }
  if (p.L[h0 + p.nh - 1].dout != A || p.L[NL - 1].dout != 1 || A > srl::PT_MAXA || D0 > srl::PT_MAXD0) return false;
  p.tmp_ld = r4(wmax + 1);
  p.tmpA = off;
  off += srl::PT_R * p.tmp_ld;
  p.tmpB = off;
  off += srl::PT_R * p.tmp_ld;
  p.tmpD = off;
  off += srl::PT_R * p.tmp_ld;
  p.node_hi = off;
  p.D0 = D0;
  p.A = A;
  return off <= srl::PT_LDS;
}
}  // namespace

bool ppo_mlp_train_fits(std::vector<std::vector<int64_t>> layers, std::vector<int64_t> counts, int64_t D0, int64_t A) {
  srl::PTArgs p{};
  return pt_plan(layers, counts, D0, A, p);
}

// data: obs [n, D0], actions [n, A] (one-hot), logprobs / values / returns / advantages [n];
// perm [epochs, n] int64; slabs: flat param, flat grad, exp_avg, exp_avg_sq, scalars (FlatAdam);
// coefs: device clip / entropy coefficients; out_sums [3]
void ppo_mlp_train(std::vector<std::vector<int64_t>> layers, std::vector<int64_t> counts, std::vector<torch::Tensor> data,
                   torch::Tensor perm, std::vector<torch::Tensor> slabs, std::vector<torch::Tensor> coefs,
                   torch::Tensor out_sums, int64_t bs, double vf_coef, double max_grad_norm, bool clip_vloss,
                   bool norm_adv, double lr, double b1, double b2, double eps, double wd, bool decoupled,
                   int64_t nwg, torch::Tensor err, torch::Tensor prof) {
  TORCH_CHECK(data.size() == 6 && slabs.size() == 5 && coefs.size() == 2, "ppo_mlp_train: argument lists");
  for (auto& t : data) check_f32(t, "ppo_mlp_train data");
  for (auto& t : slabs) check_f32(t, "ppo_mlp_train slab");
  for (auto& t : coefs) check_f32(t, "ppo_mlp_train coef");
  check_f32(out_sums, "out_sums");
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == torch::kInt64 && perm.is_contiguous() && perm.dim() == 2,
              "perm: contiguous int64 [epochs, n]");
  const int64_t n = data[0].size(0);
  const int D0 = data[0].size(1), A = data[1].size(1);
  srl::PTArgs p{};
  TORCH_CHECK(pt_plan(layers, counts, D0, A, p), "ppo_mlp_train: agent does not fit the fused kernel");
  TORCH_CHECK(perm.size(1) == n && data[1].size(0) == n, "ppo_mlp_train: row counts");
  for (int i = 2; i < 6; ++i) TORCH_CHECK(data[i].numel() == n, "ppo_mlp_train: per-row vectors");
  const int64_t P = slabs[0].numel();
  for (int i = 1; i < 4; ++i) TORCH_CHECK(slabs[i].numel() == P, "ppo_mlp_train: slab sizes");
  TORCH_CHECK(slabs[4].numel() >= 3 && out_sums.numel() >= 3, "ppo_mlp_train: scalars");
  const int NL = p.ne + p.na + p.nh + p.nc;
  for (int l = 0; l < NL; ++l) {
    TORCH_CHECK(p.L[l].pw >= 0 && p.L[l].pw + (int64_t)p.L[l].din * p.L[l].dout <= P, "ppo_mlp_train: weight offset");
    TORCH_CHECK(p.L[l].pb < 0 || p.L[l].pb + p.L[l].dout <= P, "ppo_mlp_train: bias offset");
  }
  TORCH_CHECK(bs >= 1 && bs <= srl::PT_THREADS && n >= 1, "ppo_mlp_train: 1 <= batch size <= 512");
  p.obs = data[0].data_ptr<float>();
  p.actions = data[1].data_ptr<float>();
  p.logp_old = data[2].data_ptr<float>();
  p.val_old = data[3].data_ptr<float>();
  p.ret = data[4].data_ptr<float>();
  p.adv = data[5].data_ptr<float>();
  p.perm = perm.data_ptr<int64_t>();
  p.n = n;
  p.bs = bs;
  p.epochs = perm.size(0);
  p.clip_p = coefs[0].data_ptr<float>();
  p.ent_p = coefs[1].data_ptr<float>();
  p.vf_coef = vf_coef;
  p.max_grad_norm = max_grad_norm;
  p.clip_vloss = clip_vloss;
  p.norm_adv = norm_adv;
  p.param = slabs[0].data_ptr<float>();
  p.grad = slabs[1].data_ptr<float>();
  p.m = slabs[2].data_ptr<float>();
  p.v = slabs[3].data_ptr<float>();
  p.scalars = slabs[4].data_ptr<float>();
  p.lr = lr;
  p.b1 = b1;
  p.b2 = b2;
  p.eps = eps;
  p.wd = wd;
  p.decoupled = decoupled;
  p.out_sums = out_sums.data_ptr<float>();
  // workgroups per minibatch: one 16-row chunk each (a cooperative launch; 1 = single workgroup)
  p.nwg = (int)std::max<int64_t>(1, std::min<int64_t>({nwg, (bs + srl::PT_R - 1) / srl::PT_R, 16}));
  check_f32(err, "err");
  p.err = err.data_ptr<float>();
  p.prof = prof.numel() >= 4 && prof.is_cuda() && prof.scalar_type() == torch::kInt64 ? reinterpret_cast<long long*>(prof.data_ptr<int64_t>()) : nullptr;
  p.nparam = (int)P;
  // zeros: the slab's alignment padding is never written by the gradient tiles and must read as 0
  torch::Tensor scratch = torch::zeros({(int64_t)p.nwg * P + p.nwg + 4}, slabs[0].options());
  p.partial = scratch.data_ptr<float>();
  p.sq = p.partial + (int64_t)p.nwg * P;
  p.bar = reinterpret_cast<int*>(p.sq + p.nwg);
  const hipError_t e = launch_ppo_mlp_train(p, cur_stream());
  TORCH_CHECK(e == hipSuccess, "ppo_mlp_train launch failed: ", hipGetErrorString(e));
}

void register_conv(pybind11::module& m);
void register_ext(pybind11::module& m);
void register_sac(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  register_conv(m);
  register_ext(m);
  register_sac(m);
  m.def("set_gru_vec", &set_gru_vec);  // float4 wide-row LN-GRU forward on (default) / off (A/B, tests)
  m.def("ln_gru_into", &ln_gru_into, pybind11::arg("x"), pybind11::arg("h"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("eps"), pybind11::arg("out"), pybind11::arg("mean") = pybind11::none(),
        pybind11::arg("rstd") = pybind11::none(), pybind11::arg("x2") = pybind11::none(),
        pybind11::arg("write_sum") = false);  // write_sum: x <- x + x2 (the whole GRU input, for a backward)
  m.def("colsum", &colsum);
  m.def("cartpole_step", &cartpole_step);
  m.def("ppo_cartpole_rollout", &ppo_cartpole_rollout);
  m.def("ppo_mlp_train_fits", &ppo_mlp_train_fits);
  m.def("ppo_mlp_train", &ppo_mlp_train);
  m.def("unimix_sample_into", &unimix_sample_into, pybind11::arg("logits"), pybind11::arg("uniform"), pybind11::arg("classes"),
        pybind11::arg("alpha"), pybind11::arg("out"), pybind11::arg("idx") = pybind11::none(), pybind11::arg("idx_off") = 0);
  m.doc() = "sheeprl_prey_amd HIP kernels (gfx950)";
  m.def("flat_grad_norm", &flat_grad_norm, pybind11::arg("g"), pybind11::arg("scalars"), pybind11::arg("max_norm"),
        pybind11::arg("guard") = pybind11::none());
  m.def("flat_advance", &flat_advance, pybind11::arg("scalars"), pybind11::arg("guard") = pybind11::none());
  m.def("flat_adam", &flat_adam);
  m.def("ln_act_fwd", &ln_act_fwd);
  m.def("ln_act_bwd", &ln_act_bwd);
  m.def("ln_nchw_fwd", &ln_nchw_fwd);
  m.def("ln_nchw_bwd", &ln_nchw_bwd);
  m.def("ln_gru_fwd", &ln_gru_fwd);
  m.def("ln_gru_bwd", &ln_gru_bwd);
  m.def("unimix_sample_fwd", &unimix_sample_fwd);
  m.def("unimix_sample_bwd", &unimix_sample_bwd);
  m.def("twohot_nll_fwd", &twohot_nll_fwd);
  m.def("twohot_nll_bwd", &twohot_nll_bwd);
  m.def("value_loss2", &value_loss2);
  m.def("twohot_mean_fwd", &twohot_mean_fwd);
  m.def("twohot_mean_bwd", &twohot_mean_bwd);
  m.def("kl_fwd", &kl_fwd);
  m.def("kl_bwd", &kl_bwd);
  m.def("lambda_fwd", &lambda_fwd);
  m.def("lambda_bwd", &lambda_bwd);
  m.def("gae", &gae);
  m.def("squashed_gaussian_fwd", &squashed_gaussian_fwd);
  m.def("squashed_gaussian_bwd", &squashed_gaussian_bwd);
  m.def("ln_act_fwd_into", &ln_act_fwd_into);
  m.def("ln_act_bwd_into", &ln_act_bwd_into);
  m.def("ln_bwd_grid", &ln_bwd_grid_py);
  m.def("set_colsum_workspace", &set_colsum_workspace_py);
  m.def("set_colsum_side_stream", [](int64_t st) { set_colsum_side_stream(reinterpret_cast<hipStream_t>(st)); });
  m.def("ln_gru_bwd_grid", &ln_gru_bwd_grid_py);
  m.def("ln_gru_fwd_into", &ln_gru_fwd_into);
  m.def("ln_gru_bwd_into", &ln_gru_bwd_into, pybind11::arg("x"), pybind11::arg("h"), pybind11::arg("ldh"), pybind11::arg("gamma"),
        pybind11::arg("beta"), pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("dhn"), pybind11::arg("dx"),
        pybind11::arg("dh"), pybind11::arg("pdg"), pybind11::arg("pdb"), pybind11::arg("dgamma"), pybind11::arg("dbeta"),
        pybind11::arg("M"), pybind11::arg("H"), pybind11::arg("dadd") = pybind11::none());
  m.def("colsum2", &colsum2);
  m.def("rssm_mask_fwd", &rssm_mask_fwd);
  m.def("rssm_mask_bwd", &rssm_mask_bwd);
  m.def("unimix_sample_fwd_into", &unimix_sample_fwd_into);
  m.def("unimix_sample_bwd_into", &unimix_sample_bwd_into);
  m.def("scan4_fwd", &scan4_fwd);
  m.def("scan4_bwd", &scan4_bwd);
  m.def("scan4_lds", &scan4_lds);
  m.def("scanp_fwd", &scanp_fwd);
  m.def("scanp_bwd", &scanp_bwd);
  m.def("scanp_info", &scanp_info);
  m.def("truncnorm_rsample_fwd", &truncnorm_rsample_fwd);
  m.def("truncnorm_rsample_bwd", &truncnorm_rsample_bwd);
  m.def("truncnorm_logprob_fwd", &truncnorm_logprob_fwd);
  m.def("truncnorm_logprob_bwd", &truncnorm_logprob_bwd);
  m.def("tn_head_sample_fwd", &tn_head_sample_fwd);
  m.def("tn_head_linear_sample_fwd", &tn_head_linear_sample_fwd, pybind11::arg("y"), pybind11::arg("W"), pybind11::arg("b"),
        pybind11::arg("u"), pybind11::arg("init_std"), pybind11::arg("min_std"), pybind11::arg("lo"), pybind11::arg("hi"),
        pybind11::arg("pre"), pybind11::arg("loc"), pybind11::arg("scale"), pybind11::arg("x"),
        pybind11::arg("ln_w") = pybind11::none(), pybind11::arg("ln_b") = pybind11::none(), pybind11::arg("ln_eps") = 0.0,
        pybind11::arg("act") = 0, pybind11::arg("y_out") = pybind11::none(), pybind11::arg("mean") = pybind11::none(),
        pybind11::arg("rstd") = pybind11::none());
  m.def("tn_head_sample_bwd", &tn_head_sample_bwd);
  m.def("set_scanp_prof", &set_scanp_prof);
  m.def("set_scanp_health", &set_scanp_health);
  m.def("set_scan4_prof", &set_scan4_prof);
}
