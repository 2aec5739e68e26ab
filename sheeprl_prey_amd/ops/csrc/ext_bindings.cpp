// Torch bindings of the round-2+ kernels (replay gather, LSTM, GRU cell, NatureCNN, ...).  Registered into the
// same extension module as bindings.cpp (register_ext).  Every launch validates the shapes of all
// operands on the host against the dimensions the kernel indexes with.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>


void natcnn_fwd(const float* x, const float* w, const float* b, float* y, int Nb, int H, int W, int Ci, int Co, int KH,
                int KW, int S, hipStream_t st);
void natcnn_wgrad(const float* x, const float* dy, const float* y, float* dw, float* db, int Nb, int H, int W, int Ci,
                  int Co, int KH, int KW, int S, hipStream_t st);
void natcnn_dgrad(const float* dy, const float* y, const float* w, float* dcol, float* dx, int Nb, int H, int W, int Ci,
                  int Co, int KH, int KW, int S, hipStream_t st);

void launch_moments(const float* x, int n, int r0, int r1, int r2, int r3, float frac_lo, float frac_hi, float decay,
                    float om, float inv_max, float* low, float* high, float* inv, hipStream_t st);

int skinny_plan(int N, int K, int Z, int* kc);
void launch_skinny_nt(const float* A, long lda, long sA, const float* W, long ldw, long sW, float* out, long ldo, long sO,
                      const float* add, long ldadd, long sAdd, float* part, int M, int N, int K, int Z, hipStream_t st);
void launch_sac_target(const float* obs, const float* act, const float* logp, const float* rew, const float* done,
                       const float* log_alpha, const float* W1, const float* b1, const float* W2, const float* b2,
                       const float* W3, const float* b3, float* y, int M, int OD, int AD, int H, int n, float gamma,
                       hipStream_t st);
size_t sac_critic_fwd_lds(int INp, int H);
int sac_critic_blocks(int M);
void launch_sac_critic_fwd(const float* obs, const float* act, const float* y, const float* W1, const float* b1,
                           const float* W2, const float* b2, const float* W3, const float* b3, float* X, float* H1, float* H2,
                           float* DH1, float* DH2, float* DQ, float* Q, float* lossp, int M, int OD, int AD, int H, int n,
                           hipStream_t st);
void launch_sac_critic_wgrad(const float* X, const float* H1, const float* H2, const float* DH1, const float* DH2,
                             const float* DQ, const float* g, float* dW1, float* db1, float* dW2, float* db2, float* dW3,
                             float* db3, int M, int IN, int H, int n, const float* lossp, int nlp, float* loss,
                             hipStream_t st);
void launch_wm_loss_fwd(const float* kl_loss, const float* obs, const float* rew, const float* logit, const float* done,
                        const float* kl, int R, float kl_reg, float scale, float* total, float* means, hipStream_t st);
void launch_wm_loss_bwd(const float* logit, const float* done, const float* g, int R, float kl_reg, float scale, float* d_kll,
                        float* d_obs, float* d_rew, float* d_logit, hipStream_t st);
bool launch_ens_disagreement(const float* X, const float* W, const float* b, float* part, int n, int M, int O, int H,
                             hipStream_t st);
bool launch_symlog_cat(const float* const* src, const int* d, int n, float* out, int rows, hipStream_t st);
void launch_obs_mse_fwd(const float* rec, const void* tgt, bool u8, int rows, int n, float scale, int symlog, float* loss,
                        hipStream_t st);
void launch_obs_mse_bwd(const float* rec, const void* tgt, bool u8, int rows, int n, float scale, int symlog, const float* g,
                        float* drec, hipStream_t st);
void launch_imag_discount(const float* clog, const float* dones, int T1, int M, float gamma, float* cont_g, float* discount,
                          hipStream_t st, int t0);
void launch_lstm_fwd(const float* xg, const float* Whh, const float* h0, const float* c0, float* out, float* gates, float* cs,
                     float* hT, float* cT, int T, int B, int H, hipStream_t st);
void launch_lstm_bwd(const float* Whh, const float* c0, const float* gates, const float* cs, const float* dout, const float* dhT,
                     const float* dcT, float* dgates, float* dh0, float* dc0, int T, int B, int H, hipStream_t st);
void launch_gru_cell_fwd(const float* gi, const float* gh, const float* h, float* hn, float* rzn, int B, int H, hipStream_t st);
void launch_gru_cell_bwd(const float* gh, const float* h, const float* rzn, const float* dhn, float* dgi, float* dgh, float* dh,
                         int B, int H, hipStream_t st);
void launch_gather_rows(const void* const* src, void* const* dst, const long* row_bytes, int nk, int n_envs, long cap, int N,
                        const long* row, const long* env, int* err, hipStream_t st);
int actor_loss_blocks(int rows);
void launch_actor_loss_cont(const float* pre, const float* lam, const float* base, const float* disc, const float* offp,
                            const float* invp, int A, int T, int M, float ent_coef, float init_std, float min_std, float lo,
                            float hi, float* dpre, float* dlam, float* dbase, float* partial, float* loss, hipStream_t st);
void launch_actor_loss(const float* z, const float* act, const float* lam, const float* base, const float* disc,
                       const float* offp, const float* invp, const int* heads, int nh, int A, int T, int M, float ent_coef,
                       float* dz, float* partial, float* loss, hipStream_t st);

int wgrad_dense_chunks(int M, int N, int K);
void launch_wgrad_dense(const float* dz, long ldz, const float* x, long ldx, float* part, float* bpart, int M, int N, int K,
                        int S, hipStream_t st);
int wgrad_onehot_chunks(int M, int N, int G, int C);
bool launch_wgrad_onehot(const float* dz, long ldz, const int* idx, long ldi, int off, float* part, int M, int N, int G, int C,
                         int S, hipStream_t st);
void launch_wgrad_reduce(const float* part, int S, int N, int K, float* out, long ldo, int coff, bool accumulate,
                         hipStream_t st);

bool launch_actor_tail(const float* pre, long ldp, float* y, long ldy, const float* gamma, const float* beta, float* mean,
                       float* rstd, float eps, int act, const float* Wh, const float* bh, int A, const float* uniform,
                       float alpha, float* sample, long lds, int* idx, long ldi, int ioff, float* logits, int M, int N,
                       hipStream_t st);

bool launch_prior_head(const float* x, long ldx, const float* gamma, const float* beta, float eps, int act, const float* W,
                       const float* b, const float* uni, float alpha, float* sample, long lds, int* idx, long ldi, int ioff,
                       int M, int K, int N, hipStream_t st, float* logits = nullptr, long ldl = 0,
                       float* mean_out = nullptr, float* rstd_out = nullptr);

bool launch_seq_sample(const void* const* src, void* const* dst, const long* row_bytes, int nk, int n_envs, long cap, int B,
                       int L, long n1, long start2, long n2, unsigned long long seed, unsigned long long counter,
                       hipStream_t st);

void launch_onehot_index(const float* x, int ldx, int M, int G, int C, int* idx, int ldi, int off, hipStream_t st);
bool launch_onehot_gather_ln(const float* Y, int ldy, const int* idx, int ldi, int G, int off, const float* T, int K,
                             const float* bias, const float* gamma, const float* beta, float eps, int act, int ln,
                             float* z_out, int ldz, float* y_out, int ldo, float* mean, float* rstd, int M, int N, int* err,
                             hipStream_t st, const float* xa = nullptr, int ldxa = 0, int nA = 0, const float* Wa = nullptr);

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

const float* optf(const c10::optional<torch::Tensor>& t, const char* name, int64_t numel) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous() && t->numel() == numel, "onehot: ",
              name, " must be a contiguous float32 GPU tensor of ", numel, " elements");
  return t->data_ptr<float>();
}

void rowview(const torch::Tensor& t, const char* name, int64_t M, int64_t N, torch::ScalarType dt) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.dim() == 2 && t.size(0) == M && t.size(1) >= N && t.stride(1) == 1 &&
                  t.stride(0) >= t.size(1),
              "onehot: ", name, " must be a row-strided 2-D [", M, ", >=", N, "] view of the right dtype");
}

}  // namespace

// ------------------------------------------------------------------ one-hot row gathers (onehot.hip)
// x [M, G*C] one-hot rows (row-strided) -> idx [M, >= G] int32 (row-strided): off + g*C + hot class.
void onehot_index(torch::Tensor x, int64_t C, torch::Tensor idx, int64_t off) {
  TORCH_CHECK(x.dim() == 2 && x.size(1) % C == 0, "onehot_index: x [M, G*C]");
  const int64_t M = x.size(0), G = x.size(1) / C;
  rowview(x, "x", M, G * C, torch::kFloat32);
  rowview(idx, "idx", M, G, torch::kInt);
  launch_onehot_index(x.data_ptr<float>(), x.stride(0), M, G, C, idx.data_ptr<int>(), idx.stride(0), off, stream());
}

// y = act(LN(Y + sum_j table[idx_j - off] + bias)) per row (LN when gamma/beta given or ln=true); writes z (pre-norm),
// mean/rstd when given.  table [K, N] contiguous; Y / z / y row-strided [M, N]; idx row-strided [M, >= G].
bool onehot_gather_ln(c10::optional<torch::Tensor> Y, torch::Tensor idx, int64_t G, int64_t off, torch::Tensor table,
                      c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
                      double eps, int64_t act, bool ln, c10::optional<torch::Tensor> z_out, torch::Tensor y_out,
                      c10::optional<torch::Tensor> mean, c10::optional<torch::Tensor> rstd, c10::optional<torch::Tensor> err,
                      c10::optional<torch::Tensor> xa, c10::optional<torch::Tensor> Wa) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == torch::kFloat32 && table.dim() == 2 && table.is_contiguous(),
              "onehot_gather_ln: table [K, N] contiguous float32");
  const int64_t K = table.size(0), N = table.size(1), M = y_out.size(0);
  rowview(y_out, "y_out", M, N, torch::kFloat32);
  rowview(idx, "idx", M, G, torch::kInt);
  const float* yp = nullptr;
  int64_t ldy = 0;
  if (Y.has_value() && Y->defined()) {
    rowview(*Y, "Y", M, N, torch::kFloat32);
    yp = Y->data_ptr<float>();
    ldy = Y->stride(0);
  }
  float* zp = nullptr;
  int64_t ldz = 0;
  if (z_out.has_value() && z_out->defined()) {
    rowview(*z_out, "z_out", M, N, torch::kFloat32);
    zp = z_out->data_ptr<float>();
    ldz = z_out->stride(0);
  }
  int* ep = nullptr;
  if (err.has_value() && err->defined()) {
    TORCH_CHECK(err->is_cuda() && err->scalar_type() == torch::kInt && err->numel() >= 1, "onehot_gather_ln: err int32 [1]");
    ep = err->data_ptr<int>();
  }
  float* mp_ = mean.has_value() && mean->defined() ? const_cast<float*>(optf(mean, "mean", M)) : nullptr;
  float* rp_ = rstd.has_value() && rstd->defined() ? const_cast<float*>(optf(rstd, "rstd", M)) : nullptr;
  // optional dense input columns: xa [M, nA] row-strided, Wa [nA, N] contiguous (acc += xa Wa)
  const float* xap = nullptr;
  const float* wap = nullptr;
  int64_t ldxa = 0, nA = 0;
  if (xa.has_value() && xa->defined()) {
    TORCH_CHECK(Wa.has_value() && Wa->defined() && Wa->is_cuda() && Wa->scalar_type() == torch::kFloat32 && Wa->dim() == 2 &&
                    Wa->is_contiguous() && Wa->size(1) == N,
                "onehot_gather_ln: Wa [nA, N] contiguous float32");
    nA = Wa->size(0);
    rowview(*xa, "xa", M, nA, torch::kFloat32);
    xap = xa->data_ptr<float>();
    ldxa = xa->stride(0);
    wap = Wa->data_ptr<float>();
  }
  return launch_onehot_gather_ln(yp, ldy, idx.data_ptr<int>(), idx.stride(0), G, off, table.data_ptr<float>(), K,
                                 optf(bias, "bias", N), optf(gamma, "gamma", N), optf(beta, "beta", N), (float)eps, act,
                                 ln ? 1 : 0, zp, ldz, y_out.data_ptr<float>(), y_out.stride(0), mp_, rp_, M, N, ep, stream(),
                                 xap, (int)ldxa, (int)nA, wap);
}


// ------------------------------------------------------------------ NatureCNN convolutions (natcnn.hip)
namespace {
void nc_check(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.defined() && t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), "natcnn: ", name,
              " must be a contiguous float32 GPU tensor");
}
struct NcDims {
  int Nb, H, W, Ci, Co, OH, OW;
};
NcDims nc_dims(const torch::Tensor& x, const torch::Tensor& wp, int64_t KH, int64_t KW, int64_t S) {
  nc_check(x, "x");
  nc_check(wp, "w");
  TORCH_CHECK(x.dim() == 4, "natcnn: x must be NHWC [N, H, W, C]");
  NcDims d{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)wp.size(0), 0, 0};
  TORCH_CHECK(KH >= 1 && KW >= 1 && S >= 1 && d.H >= KH && d.W >= KW, "natcnn: bad kernel/stride for the input");
  TORCH_CHECK(d.Ci % 4 == 0 && d.Co % 4 == 0, "natcnn: channel counts must be multiples of 4");
  TORCH_CHECK(wp.dim() == 2 && wp.size(1) == KH * KW * d.Ci, "natcnn: packed weight must be [Co, KH*KW*Ci]");
  TORCH_CHECK((int64_t)d.Nb * d.H * d.W * d.Ci < (1LL << 31), "natcnn: input too large for 32-bit offsets");
  d.OH = (int)((d.H - KH) / S + 1);
  d.OW = (int)((d.W - KW) / S + 1);
  return d;
}
}  // namespace

torch::Tensor nc_conv_fwd(torch::Tensor x, torch::Tensor wp, c10::optional<torch::Tensor> b, int64_t KH, int64_t KW,
                          int64_t S) {
  const NcDims d = nc_dims(x, wp, KH, KW, S);
  const float* bp = nullptr;
  if (b.has_value() && b->defined()) {
    nc_check(*b, "b");
    TORCH_CHECK(b->numel() == d.Co, "natcnn: bias size");
    bp = b->data_ptr<float>();
  }
  auto y = torch::empty({d.Nb, d.OH, d.OW, d.Co}, x.options());
  natcnn_fwd(x.data_ptr<float>(), wp.data_ptr<float>(), bp, y.data_ptr<float>(), d.Nb, d.H, d.W, d.Ci, d.Co, (int)KH,
             (int)KW, (int)S, stream());
  return y;
}

// {dx (empty unless need_dx), dW packed [Co, K], db [Co]} for y = relu(conv(x) + b)
std::vector<torch::Tensor> nc_conv_bwd(torch::Tensor x, torch::Tensor y, torch::Tensor dy, torch::Tensor wp, int64_t KH,
                                       int64_t KW, int64_t S, bool need_dx) {
  const NcDims d = nc_dims(x, wp, KH, KW, S);
  nc_check(y, "y");
  nc_check(dy, "dy");
  TORCH_CHECK(y.numel() == (int64_t)d.Nb * d.OH * d.OW * d.Co && dy.numel() == y.numel(), "natcnn: y / dy shape");
  auto dw = torch::zeros_like(wp);
  auto db = torch::zeros({d.Co}, x.options());
  natcnn_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), y.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
               d.Nb, d.H, d.W, d.Ci, d.Co, (int)KH, (int)KW, (int)S, stream());
  torch::Tensor dx;
  if (need_dx) {
    dx = torch::empty_like(x);
    auto dcol = torch::empty({(int64_t)d.Nb * d.OH * d.OW, KH * KW * d.Ci}, x.options());
    natcnn_dgrad(dy.data_ptr<float>(), y.data_ptr<float>(), wp.data_ptr<float>(), dcol.data_ptr<float>(), dx.data_ptr<float>(),
                 d.Nb, d.H, d.W, d.Ci, d.Co, (int)KH, (int)KW, (int)S, stream());
  }
  return {dx, dw, db};
}

// ------------------------------------------------------------------ Moments percentile EMA (moments.hip)
// ranks = order statistics {floor, ceil} of q_low * (n - 1) and of q_high * (n - 1); low / high / inv: fp32 scalars
void moments_update(torch::Tensor x, std::vector<int64_t> ranks, std::vector<double> fracs, double decay, double max_,
                    torch::Tensor low, torch::Tensor high, torch::Tensor inv) {
  nc_check(x, "x");
  nc_check(low, "low");
  nc_check(high, "high");
  nc_check(inv, "inv");
  TORCH_CHECK(low.numel() == 1 && high.numel() == 1 && inv.numel() == 1, "moments: scalar buffers");
  TORCH_CHECK(ranks.size() == 4 && fracs.size() == 2, "moments: 4 ranks, 2 fractions");
  const int64_t n = x.numel();
  TORCH_CHECK(n >= 1 && n < (1LL << 31), "moments: size");
  for (auto r : ranks) TORCH_CHECK(r >= 0 && r < n, "moments: rank out of range");
  launch_moments(x.data_ptr<float>(), (int)n, (int)ranks[0], (int)ranks[1], (int)ranks[2], (int)ranks[3], (float)fracs[0],
                 (float)fracs[1], (float)decay, (float)(1.0 - decay), (float)(1.0 / max_), low.data_ptr<float>(),
                 high.data_ptr<float>(), inv.data_ptr<float>(), stream());
}

// ------------------------------------------------------------------ DreamerV3 discrete actor objective (actor_loss.hip)
// z, actions [T, M, A]; lam, base [T-1, M]; disc [T, M] (only the first T-1 rows read); offset / invscale
// scalars.  Returns {loss (0-dim), dloss/dz [T, M, A]}.
std::vector<torch::Tensor> actor_loss_discrete(torch::Tensor z, torch::Tensor actions, torch::Tensor lam, torch::Tensor base,
                                               torch::Tensor disc, torch::Tensor offset, torch::Tensor invscale,
                                               std::vector<int64_t> heads, double ent_coef) {
  for (auto* t : {&z, &actions, &lam, &base, &disc, &offset, &invscale}) nc_check(*t, "actor_loss operand");
  TORCH_CHECK(z.dim() == 3 && actions.sizes() == z.sizes(), "actor_loss: z / actions must be [T, M, A]");
  const int64_t T = z.size(0), M = z.size(1), A = z.size(2);
  TORCH_CHECK(T >= 2 && lam.numel() == (T - 1) * M && base.numel() == (T - 1) * M && disc.numel() >= (T - 1) * M,
              "actor_loss: lambda / baseline [T-1, M], discount [T, M]");
  TORCH_CHECK(offset.numel() == 1 && invscale.numel() == 1, "actor_loss: scalar offset / invscale");
  TORCH_CHECK(!heads.empty() && heads.size() <= 8, "actor_loss: 1..8 heads");
  int64_t sum = 0;
  std::vector<int> hs;
  for (auto h : heads) {
    TORCH_CHECK(h >= 1, "actor_loss: head size");
    sum += h;
    hs.push_back((int)h);
  }
  TORCH_CHECK(sum == A, "actor_loss: head sizes must add up to A");
  auto dz = torch::empty_like(z);
  auto loss = torch::empty({}, z.options());
  auto partial = torch::empty({actor_loss_blocks((int)(T * M))}, z.options());
  launch_actor_loss(z.data_ptr<float>(), actions.data_ptr<float>(), lam.data_ptr<float>(), base.data_ptr<float>(),
                    disc.data_ptr<float>(), offset.data_ptr<float>(), invscale.data_ptr<float>(), hs.data(), (int)hs.size(),
                    (int)A, (int)T, (int)M, (float)ent_coef, dz.data_ptr<float>(), partial.data_ptr<float>(),
                    loss.data_ptr<float>(), stream());
  return {loss, dz};
}

// ------------------------------------------------------------------ DreamerV3 continuous actor objective (actor_loss.hip)
// pre [T, M, 2A] (the trunc-normal head outputs); lam, base [T-1, M]; disc [T, M] (first T-1 rows read); offset /
// invscale scalars.  Returns {loss (0-dim), grads [T*M*2A | (T-1)M | (T-1)M] packed: d pre, d lambda, d baseline}.
std::vector<torch::Tensor> actor_loss_cont(torch::Tensor pre, torch::Tensor lam, torch::Tensor base, torch::Tensor disc,
                                           torch::Tensor offset, torch::Tensor invscale, double ent_coef, double init_std,
                                           double min_std, double lo, double hi) {
  for (auto* t : {&pre, &lam, &base, &disc, &offset, &invscale}) nc_check(*t, "actor_loss_cont operand");
  TORCH_CHECK(pre.dim() == 3 && pre.size(2) % 2 == 0, "actor_loss_cont: pre must be [T, M, 2A]");
  const int64_t T = pre.size(0), M = pre.size(1), A = pre.size(2) / 2;
  TORCH_CHECK(T >= 2 && A >= 1 && lam.numel() == (T - 1) * M && base.numel() == (T - 1) * M && disc.numel() >= (T - 1) * M,
              "actor_loss_cont: lambda / baseline [T-1, M], discount [T, M]");
  TORCH_CHECK(offset.numel() == 1 && invscale.numel() == 1, "actor_loss_cont: scalar offset / invscale");
  auto grads = torch::empty({T * M * 2 * A + 2 * (T - 1) * M}, pre.options());
  auto loss = torch::empty({}, pre.options());
  auto partial = torch::empty({actor_loss_blocks((int)(T * M))}, pre.options());
  float* g = grads.data_ptr<float>();
  launch_actor_loss_cont(pre.data_ptr<float>(), lam.data_ptr<float>(), base.data_ptr<float>(), disc.data_ptr<float>(),
                         offset.data_ptr<float>(), invscale.data_ptr<float>(), (int)A, (int)T, (int)M, (float)ent_coef,
                         (float)init_std, (float)min_std, (float)lo, (float)hi, g, g + T * M * 2 * A,
                         g + T * M * 2 * A + (T - 1) * M, partial.data_ptr<float>(), loss.data_ptr<float>(), stream());
  return {loss, grads};
}

// ------------------------------------------------------------------ skinny weight-streaming GEMM (skinny.hip)
// out[z] = A[z] . W[z]^T (+ add[z]); A [Z, M<=16, K] (row stride free), W [Z, N, K] contiguous rows,
// out [Z, M, N], add [Z, M or 1 (broadcast), N].  2-D operands are Z = 1.  Returns the workspace size
// needed (floats) when `part` is undefined and nothing was launched.
static void skinny_dims(const torch::Tensor& t, int64_t& Z, int64_t& R, int64_t& C, int64_t& ld, int64_t& sz) {
  TORCH_CHECK(t.dim() == 2 || t.dim() == 3, "skinny_nt: 2-D or 3-D operands");
  TORCH_CHECK(t.stride(-1) == 1, "skinny_nt: unit stride along the last dim");
  Z = t.dim() == 3 ? t.size(0) : 1;
  R = t.size(-2);
  C = t.size(-1);
  ld = t.stride(-2);
  sz = t.dim() == 3 ? t.stride(0) : 0;
}

int64_t skinny_nt(torch::Tensor A, torch::Tensor W, torch::Tensor out, c10::optional<torch::Tensor> add,
                  c10::optional<torch::Tensor> part) {
  int64_t Za, M, K, lda, sA, Zw, N, Kw, ldw, sW, Zo, Mo, No, ldo, sO;
  skinny_dims(A, Za, M, K, lda, sA);
  skinny_dims(W, Zw, N, Kw, ldw, sW);
  skinny_dims(out, Zo, Mo, No, ldo, sO);
  TORCH_CHECK(Za == Zw && Za == Zo && K == Kw && Mo == M && No == N, "skinny_nt: shape mismatch");
  TORCH_CHECK(M >= 1 && M <= 16 && K % 128 == 0 && N % 128 == 0, "skinny_nt: M <= 16, K % 128 == 0, N % 128 == 0");
  for (auto* t : {&A, &W, &out}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32, "skinny_nt: fp32 CUDA operands");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "skinny_nt: 16-byte aligned operands");
  }
  TORCH_CHECK(lda % 4 == 0 && ldw % 4 == 0 && ldo % 4 == 0 && sA % 4 == 0 && sW % 4 == 0 && sO % 4 == 0,
              "skinny_nt: strides must be multiples of 4 floats");
  const float* addp = nullptr;
  int64_t ldadd = 0, sAdd = 0;
  if (add.has_value() && add->defined()) {
    int64_t Zd, Md, Nd;
    skinny_dims(*add, Zd, Md, Nd, ldadd, sAdd);
    TORCH_CHECK(Nd == N && (Md == M || Md == 1) && (Zd == Za || add->dim() == 2), "skinny_nt: addend shape");
    TORCH_CHECK(add->scalar_type() == torch::kFloat32 && reinterpret_cast<uintptr_t>(add->data_ptr()) % 16 == 0 &&
                    ldadd % 4 == 0 && sAdd % 4 == 0, "skinny_nt: addend fp32, 16-byte aligned");
    if (Md == 1) ldadd = 0;
    addp = add->data_ptr<float>();
  }
  int kc = 0;
  const int splits = skinny_plan((int)N, (int)K, (int)Za, &kc);
  const int64_t need = splits > 1 ? (int64_t)splits * Za * 16 * N : 0;
  float* pp = nullptr;
  if (need) {
    if (!part.has_value() || !part->defined()) return need;
    TORCH_CHECK(part->numel() >= need && part->scalar_type() == torch::kFloat32 && part->is_contiguous(),
                "skinny_nt: workspace too small");
    pp = part->data_ptr<float>();
  }
  launch_skinny_nt(A.data_ptr<float>(), lda, sA, W.data_ptr<float>(), ldw, sW, out.data_ptr<float>(), ldo, sO, addp, ldadd,
                   sAdd, pp, (int)M, (int)N, (int)K, (int)Za, stream());
  return 0;
}

int64_t skinny_workspace(int64_t N, int64_t K, int64_t Z) {
  int kc = 0;
  const int splits = skinny_plan((int)N, (int)K, (int)Z, &kc);
  return splits > 1 ? (int64_t)splits * Z * 16 * N : 0;
}

// ------------------------------------------------------------------ SAC twin-Q target (sac_target.hip)
torch::Tensor sac_twin_q_target(torch::Tensor obs, torch::Tensor act, torch::Tensor logp, torch::Tensor rew, torch::Tensor done,
                                torch::Tensor log_alpha, torch::Tensor W1, torch::Tensor b1, torch::Tensor W2, torch::Tensor b2,
                                torch::Tensor W3, torch::Tensor b3, double gamma) {
  for (auto* t : {&obs, &act, &logp, &rew, &done, &log_alpha, &W1, &b1, &W2, &b2, &W3, &b3}) nc_check(*t, "sac_twin_q_target operand");
  TORCH_CHECK(obs.dim() == 2 && act.dim() == 2 && obs.size(0) == act.size(0), "sac_twin_q_target: obs / act [M, *]");
  const int64_t M = obs.size(0), OD = obs.size(1), AD = act.size(1);
  TORCH_CHECK(logp.numel() == M && rew.numel() == M && done.numel() == M && log_alpha.numel() >= 1, "sac_twin_q_target: [M] terms");
  TORCH_CHECK(W1.dim() == 3 && W1.size(2) == OD + AD, "sac_twin_q_target: W1 [n, H, obs+act]");
  const int64_t n = W1.size(0), H = W1.size(1);
  TORCH_CHECK(n >= 1 && n <= 4 && H % 128 == 0 && H <= 512 && OD + AD <= 1024, "sac_twin_q_target: n <= 4, H % 128 == 0, H <= 512");
  TORCH_CHECK(b1.numel() == n * H && W2.numel() == n * H * H && b2.numel() == n * H && W3.numel() == n * H && b3.numel() == n,
              "sac_twin_q_target: layer shapes");
  auto y = torch::empty({M, 1}, obs.options());
  launch_sac_target(obs.data_ptr<float>(), act.data_ptr<float>(), logp.data_ptr<float>(), rew.data_ptr<float>(),
                    done.data_ptr<float>(), log_alpha.data_ptr<float>(), W1.data_ptr<float>(), b1.data_ptr<float>(),
                    W2.data_ptr<float>(), b2.data_ptr<float>(), W3.data_ptr<float>(), b3.data_ptr<float>(), y.data_ptr<float>(),
                    (int)M, (int)OD, (int)AD, (int)H, (int)n, (float)gamma, stream());
  return y;
}

// ------------------------------------------------------------------ SAC twin-Q critic update (sac_critic.hip)
// -> {loss partials [n * blocks], q [M, n], saved: X, H1, H2, DH1, DH2, DQ}
std::vector<torch::Tensor> sac_critic_fwd(torch::Tensor obs, torch::Tensor act, torch::Tensor y, torch::Tensor W1,
                                          torch::Tensor b1, torch::Tensor W2, torch::Tensor b2, torch::Tensor W3, torch::Tensor b3) {
  for (auto* t : {&obs, &act, &y, &W1, &b1, &W2, &b2, &W3, &b3}) nc_check(*t, "sac_critic operand");
  TORCH_CHECK(obs.dim() == 2 && act.dim() == 2 && obs.size(0) == act.size(0), "sac_critic: obs / act [M, *]");
  const int64_t M = obs.size(0), OD = obs.size(1), AD = act.size(1), IN = OD + AD;
  TORCH_CHECK(M >= 1 && y.numel() == M, "sac_critic: y holds one target per row");
  TORCH_CHECK(W1.dim() == 3 && W1.size(2) == IN, "sac_critic: W1 [n, H, obs+act]");
  const int64_t n = W1.size(0), H = W1.size(1), INp = (IN + 15) / 16 * 16;
  TORCH_CHECK(n >= 1 && n <= 8 && H % 128 == 0 && H <= 512 && IN <= 1024, "sac_critic: n <= 8, H % 128 == 0, H <= 512");
  TORCH_CHECK(b1.numel() == n * H && W2.numel() == n * H * H && b2.numel() == n * H && W3.numel() == n * H && b3.numel() == n,
              "sac_critic: layer shapes");
  auto o = obs.options();
  const int64_t blocks = sac_critic_blocks((int)M);
  auto lossp = torch::empty({n * blocks}, o);
  auto q = torch::empty({M, n}, o);
  auto X = torch::empty({M, INp}, o);
  auto H1 = torch::empty({n, M, H}, o), H2 = torch::empty({n, M, H}, o);
  auto DH1 = torch::empty({n, M, H}, o), DH2 = torch::empty({n, M, H}, o);
  auto DQ = torch::empty({n, M}, o);
  launch_sac_critic_fwd(obs.data_ptr<float>(), act.data_ptr<float>(), y.data_ptr<float>(), W1.data_ptr<float>(),
                        b1.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(), W3.data_ptr<float>(), b3.data_ptr<float>(),
                        X.data_ptr<float>(), H1.data_ptr<float>(), H2.data_ptr<float>(), DH1.data_ptr<float>(), DH2.data_ptr<float>(),
                        DQ.data_ptr<float>(), q.data_ptr<float>(), lossp.data_ptr<float>(), (int)M, (int)OD, (int)AD, (int)H, (int)n,
                        stream());
  return {lossp, q, X, H1, H2, DH1, DH2, DQ};
}

// -> {dW1 [n, H, IN], db1 [n, H], dW2 [n, H, H], db2 [n, H], dW3 [n, 1, H], db3 [n, 1]}, scaled by g (device scalar)
std::vector<torch::Tensor> sac_critic_wgrad(torch::Tensor X, torch::Tensor H1, torch::Tensor H2, torch::Tensor DH1,
                                            torch::Tensor DH2, torch::Tensor DQ, torch::Tensor g, int64_t IN) {
  for (auto* t : {&X, &H1, &H2, &DH1, &DH2, &DQ, &g}) nc_check(*t, "sac_critic_wgrad operand");
  TORCH_CHECK(H1.dim() == 3, "sac_critic_wgrad: H1 [n, M, H]");
  const int64_t n = H1.size(0), M = H1.size(1), H = H1.size(2), INp = (IN + 15) / 16 * 16;
  TORCH_CHECK(X.numel() == M * INp && H2.sizes() == H1.sizes() && DH1.sizes() == H1.sizes() && DH2.sizes() == H1.sizes() &&
                  DQ.numel() == n * M && g.numel() >= 1 && H % 128 == 0,
              "sac_critic_wgrad: saved shapes");
  auto o = H1.options();
  auto dW1 = torch::empty({n, H, IN}, o), db1 = torch::empty({n, H}, o), dW2 = torch::empty({n, H, H}, o);
  auto db2 = torch::empty({n, H}, o), dW3 = torch::empty({n, 1, H}, o), db3 = torch::empty({n, 1}, o);
  launch_sac_critic_wgrad(X.data_ptr<float>(), H1.data_ptr<float>(), H2.data_ptr<float>(), DH1.data_ptr<float>(),
                          DH2.data_ptr<float>(), DQ.data_ptr<float>(), g.data_ptr<float>(), dW1.data_ptr<float>(),
                          db1.data_ptr<float>(), dW2.data_ptr<float>(), db2.data_ptr<float>(), dW3.data_ptr<float>(),
                          db3.data_ptr<float>(), (int)M, (int)IN, (int)H, (int)n, nullptr, 0, nullptr, stream());
  return {dW1, db1, dW2, db2, dW3, db3};
}

// ------------------------------------------------------------------ DV3 world-model loss assembly (wm_loss.hip)
static void row_check(const torch::Tensor& t, int64_t R, const char* name) {
  nc_check(t, name);
  TORCH_CHECK(t.numel() == R, "wm_loss: ", name, " must hold one value per row");
}

// -> {total (0-dim), [mean kl, mean kl_loss, mean reward loss, mean obs loss, mean continue loss]}
std::vector<torch::Tensor> wm_loss_fwd(torch::Tensor kl_loss, torch::Tensor obs, torch::Tensor rew, c10::optional<torch::Tensor> logit,
                          c10::optional<torch::Tensor> done, torch::Tensor kl, double kl_reg, double scale) {
  const int64_t R = kl_loss.numel();
  TORCH_CHECK(R > 0 && R < (int64_t(1) << 31), "wm_loss: rows");
  row_check(kl_loss, R, "kl_loss");
  row_check(obs, R, "obs");
  row_check(rew, R, "rew");
  row_check(kl, R, "kl");
  const bool has_c = logit.has_value() && logit->defined();
  if (has_c) {
    row_check(*logit, R, "continue logits");
    TORCH_CHECK(done.has_value() && done->defined(), "wm_loss: dones needed with continue logits");
    row_check(*done, R, "dones");
  }
  auto total = torch::empty({}, kl_loss.options());
  auto means = torch::empty({5}, kl_loss.options());
  launch_wm_loss_fwd(kl_loss.data_ptr<float>(), obs.data_ptr<float>(), rew.data_ptr<float>(),
                     has_c ? logit->data_ptr<float>() : nullptr, has_c ? done->data_ptr<float>() : nullptr,
                     kl.data_ptr<float>(), (int)R, (float)kl_reg, (float)scale, total.data_ptr<float>(), means.data_ptr<float>(),
                     stream());
  return {total, means};
}

std::vector<torch::Tensor> wm_loss_bwd(c10::optional<torch::Tensor> logit, c10::optional<torch::Tensor> done, torch::Tensor g,
                                       int64_t R, double kl_reg, double scale) {
  nc_check(g, "wm_loss grad");
  TORCH_CHECK(g.numel() == 1, "wm_loss: scalar upstream gradient");
  const bool has_c = logit.has_value() && logit->defined();
  if (has_c) {
    row_check(*logit, R, "continue logits");
    row_check(*done, R, "dones");
  }
  auto opts = g.options();
  auto d_kll = torch::empty({R}, opts), d_obs = torch::empty({R}, opts), d_rew = torch::empty({R}, opts);
  auto d_logit = has_c ? torch::empty({R}, opts) : torch::Tensor();
  launch_wm_loss_bwd(has_c ? logit->data_ptr<float>() : nullptr, has_c ? done->data_ptr<float>() : nullptr, g.data_ptr<float>(),
                     (int)R, (float)kl_reg, (float)scale, d_kll.data_ptr<float>(), d_obs.data_ptr<float>(),
                     d_rew.data_ptr<float>(), has_c ? d_logit.data_ptr<float>() : nullptr, stream());
  return {d_kll, d_obs, d_rew, d_logit};
}

// ------------------------------------------------------------------ P2E disagreement (ensemble.hip)
// X [n, M, H] last hidden layer of every member, W [n, O, H], b [n, O] -> partial feature sums of the
// member variance [ceil(O / 64), M]
torch::Tensor ens_disagreement(torch::Tensor X, torch::Tensor W, c10::optional<torch::Tensor> b) {
  nc_check(X, "disagreement X");
  nc_check(W, "disagreement W");
  TORCH_CHECK(X.dim() == 3 && W.dim() == 3 && X.size(0) == W.size(0) && X.size(2) == W.size(2),
              "disagreement: X [n, M, H] and W [n, O, H]");
  const int64_t n = X.size(0), M = X.size(1), H = X.size(2), O = W.size(1);
  TORCH_CHECK(H % 4 == 0 && n <= 64 && M < (int64_t(1) << 31) && n * M * H < (int64_t(1) << 40), "disagreement: H % 4, n <= 64");
  const float* bp = nullptr;
  if (b.has_value() && b->defined()) {
    nc_check(*b, "disagreement b");
    TORCH_CHECK(b->numel() == n * O, "disagreement: b [n, O]");
    bp = b->data_ptr<float>();
  }
  auto part = torch::empty({(O + 63) / 64, M}, X.options());
  TORCH_CHECK(launch_ens_disagreement(X.data_ptr<float>(), W.data_ptr<float>(), bp, part.data_ptr<float>(), (int)n, (int)M,
                                      (int)O, (int)H, stream()),
              "disagreement: unsupported shape");
  return part;
}

// ------------------------------------------------------------------ observation MSE (obs_loss.hip)
static void obs_check(const torch::Tensor& rec, const torch::Tensor& tgt, int64_t rows) {
  nc_check(rec, "obs_mse rec");
  TORCH_CHECK(tgt.is_cuda() && tgt.is_contiguous() && tgt.numel() == rec.numel(), "obs_mse: target like rec");
  TORCH_CHECK(tgt.scalar_type() == torch::kUInt8 || tgt.scalar_type() == torch::kFloat32, "obs_mse: uint8 or fp32 target");
  TORCH_CHECK(rows > 0 && rec.numel() % rows == 0 && (rec.numel() / rows) % 4 == 0, "obs_mse: row length % 4");
}

// cat([symlog(x) for x in xs], -1) in one launch: xs contiguous float32 [..., d_j] with equal leading shapes
torch::Tensor symlog_cat(std::vector<torch::Tensor> xs) {
  TORCH_CHECK(!xs.empty() && xs.size() <= 8, "symlog_cat: 1..8 inputs");
  std::vector<const float*> src;
  std::vector<int> d;
  const auto lead = xs[0].sizes().slice(0, xs[0].dim() - 1);
  int64_t W = 0;
  for (auto& x : xs) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.is_contiguous() && x.dim() >= 1,
                "symlog_cat: contiguous float32 GPU inputs");
    TORCH_CHECK(x.sizes().slice(0, x.dim() - 1) == lead, "symlog_cat: equal leading shapes");
    src.push_back(x.data_ptr<float>());
    d.push_back((int)x.size(-1));
    W += x.size(-1);
  }
  std::vector<int64_t> shape(lead.begin(), lead.end());
  shape.push_back(W);
  auto out = torch::empty(shape, xs[0].options());
  const int64_t rows = W > 0 ? out.numel() / W : 0;
  TORCH_CHECK(rows * W < (int64_t(1) << 31), "symlog_cat: too large");
  if (rows > 0) TORCH_CHECK(launch_symlog_cat(src.data(), d.data(), (int)xs.size(), out.data_ptr<float>(), (int)rows, stream()),
                            "symlog_cat: launch");
  return out;
}

torch::Tensor obs_mse_fwd(torch::Tensor rec, torch::Tensor tgt, int64_t rows, double scale, int64_t symlog) {
  obs_check(rec, tgt, rows);
  auto loss = torch::empty({rows}, rec.options());
  launch_obs_mse_fwd(rec.data_ptr<float>(), tgt.data_ptr(), tgt.scalar_type() == torch::kUInt8, (int)rows,
                     (int)(rec.numel() / rows), (float)scale, (int)symlog, loss.data_ptr<float>(), stream());
  return loss;
}

torch::Tensor obs_mse_bwd(torch::Tensor rec, torch::Tensor tgt, int64_t rows, double scale, int64_t symlog, torch::Tensor g) {
  obs_check(rec, tgt, rows);
  nc_check(g, "obs_mse grad");
  TORCH_CHECK(g.numel() == rows, "obs_mse: one upstream gradient per row");
  auto drec = torch::empty_like(rec);
  launch_obs_mse_bwd(rec.data_ptr<float>(), tgt.data_ptr(), tgt.scalar_type() == torch::kUInt8, (int)rows,
                     (int)(rec.numel() / rows), (float)scale, (int)symlog, g.data_ptr<float>(), drec.data_ptr<float>(), stream());
  return drec;
}

// continue logits [T1, M(, 1)] (skip_first: [T1-1, M(, 1)], the rows 1.. - row 0 is replaced by 1 - done), dones [M]
// -> {cont_g [T1-1, M, 1], discount [T1, M, 1]}
std::vector<torch::Tensor> imag_discount(torch::Tensor clog, torch::Tensor dones, double gamma, bool skip_first) {
  nc_check(clog, "imag_discount logits");
  nc_check(dones, "imag_discount dones");
  const int64_t t0 = skip_first ? 1 : 0;
  const int64_t T1 = clog.size(0) + t0, M = clog.numel() / clog.size(0);
  TORCH_CHECK(T1 >= 2 && dones.numel() == M, "imag_discount: logits [T1, M], dones [M]");
  auto cg = torch::empty({T1 - 1, M, 1}, clog.options());
  auto disc = torch::empty({T1, M, 1}, clog.options());
  launch_imag_discount(clog.data_ptr<float>(), dones.data_ptr<float>(), (int)T1, (int)M, (float)gamma, cg.data_ptr<float>(),
                       disc.data_ptr<float>(), stream(), (int)t0);
  return {cg, disc};
}

// ------------------------------------------------------------------ persistent LSTM (lstm.hip)
// xg [T, B, 4H] (input projection + both biases), Whh [4H, H], h0 / c0 [B, H]
// -> {out [T, B, H], gates [T, B, 4H], cs [T, B, H], hT, cT}
std::vector<torch::Tensor> lstm_fwd(torch::Tensor xg, torch::Tensor Whh, torch::Tensor h0, torch::Tensor c0) {
  for (auto* t : {&xg, &Whh, &h0, &c0}) nc_check(*t, "lstm_fwd operand");
  TORCH_CHECK(xg.dim() == 3 && Whh.dim() == 2 && Whh.size(0) == 4 * Whh.size(1) && xg.size(2) == Whh.size(0), "lstm_fwd: shapes");
  const int64_t T = xg.size(0), B = xg.size(1), H = Whh.size(1);
  TORCH_CHECK(H % 16 == 0 && H <= 64 && h0.numel() == B * H && c0.numel() == B * H, "lstm_fwd: H % 16 == 0, H <= 64");
  auto o = xg.options();
  auto out = torch::empty({T, B, H}, o), gates = torch::empty({T, B, 4 * H}, o), cs = torch::empty({T, B, H}, o);
  auto hT = torch::empty({B, H}, o), cT = torch::empty({B, H}, o);
  launch_lstm_fwd(xg.data_ptr<float>(), Whh.data_ptr<float>(), h0.data_ptr<float>(), c0.data_ptr<float>(), out.data_ptr<float>(),
                  gates.data_ptr<float>(), cs.data_ptr<float>(), hT.data_ptr<float>(), cT.data_ptr<float>(), (int)T, (int)B,
                  (int)H, stream());
  return {out, gates, cs, hT, cT};
}

// -> {dgates [T, B, 4H] (pre-activation), dh0, dc0}
std::vector<torch::Tensor> lstm_bwd(torch::Tensor Whh, torch::Tensor c0, torch::Tensor gates, torch::Tensor cs, torch::Tensor dout,
                                    c10::optional<torch::Tensor> dhT, c10::optional<torch::Tensor> dcT) {
  for (auto* t : {&Whh, &c0, &gates, &cs, &dout}) nc_check(*t, "lstm_bwd operand");
  const int64_t T = gates.size(0), B = gates.size(1), H = Whh.size(1);
  TORCH_CHECK(dout.numel() == T * B * H && cs.numel() == T * B * H, "lstm_bwd: shapes");
  const float* dh = nullptr;
  const float* dc = nullptr;
  if (dhT.has_value() && dhT->defined()) {
    nc_check(*dhT, "lstm_bwd dhT");
    dh = dhT->data_ptr<float>();
  }
  if (dcT.has_value() && dcT->defined()) {
    nc_check(*dcT, "lstm_bwd dcT");
    dc = dcT->data_ptr<float>();
  }
  auto dgates = torch::empty_like(gates), dh0 = torch::empty({B, H}, gates.options()), dc0 = torch::empty({B, H}, gates.options());
  launch_lstm_bwd(Whh.data_ptr<float>(), c0.data_ptr<float>(), gates.data_ptr<float>(), cs.data_ptr<float>(), dout.data_ptr<float>(),
                  dh, dc, dgates.data_ptr<float>(), dh0.data_ptr<float>(), dc0.data_ptr<float>(), (int)T, (int)B, (int)H, stream());
  return {dgates, dh0, dc0};
}

// ------------------------------------------------------------------ plain GRU cell (gru_cell.hip)
std::vector<torch::Tensor> gru_cell_fwd(torch::Tensor gi, torch::Tensor gh, torch::Tensor h) {
  for (auto* t : {&gi, &gh, &h}) nc_check(*t, "gru_cell operand");
  const int64_t H = h.size(-1), B = h.numel() / H;
  TORCH_CHECK(gi.numel() == 3 * B * H && gh.numel() == 3 * B * H, "gru_cell: gi / gh [B, 3H]");
  auto hn = torch::empty_like(h), rzn = torch::empty_like(gi);
  launch_gru_cell_fwd(gi.data_ptr<float>(), gh.data_ptr<float>(), h.data_ptr<float>(), hn.data_ptr<float>(), rzn.data_ptr<float>(),
                      (int)B, (int)H, stream());
  return {hn, rzn};
}

std::vector<torch::Tensor> gru_cell_bwd(torch::Tensor gh, torch::Tensor h, torch::Tensor rzn, torch::Tensor dhn) {
  for (auto* t : {&gh, &h, &rzn, &dhn}) nc_check(*t, "gru_cell_bwd operand");
  const int64_t H = h.size(-1), B = h.numel() / H;
  auto dgi = torch::empty_like(gh), dgh = torch::empty_like(gh), dh = torch::empty_like(h);
  launch_gru_cell_bwd(gh.data_ptr<float>(), h.data_ptr<float>(), rzn.data_ptr<float>(), dhn.data_ptr<float>(), dgi.data_ptr<float>(),
                      dgh.data_ptr<float>(), dh.data_ptr<float>(), (int)B, (int)H, stream());
  return {dgi, dgh, dh};
}

// ------------------------------------------------------------------ replay row gather (gather.hip)
// srcs[k] [capacity, n_envs, ...] contiguous; row / env int64 [N] -> outputs [N, ...] per key.  ``err``
// (optional int32 [1]) is or-ed with 1 when an index is out of range; that row comes back zero-filled.
std::vector<torch::Tensor> gather_rows(std::vector<torch::Tensor> srcs, torch::Tensor row, torch::Tensor env,
                                       c10::optional<torch::Tensor> err) {
  TORCH_CHECK(!srcs.empty() && srcs.size() <= 16, "gather_rows: 1..16 keys");
  TORCH_CHECK(row.is_cuda() && env.is_cuda() && row.scalar_type() == torch::kLong && env.scalar_type() == torch::kLong &&
                  row.is_contiguous() && env.is_contiguous() && row.numel() == env.numel(),
              "gather_rows: int64 row / env index vectors");
  const int64_t N = row.numel();
  const int64_t n_envs = srcs[0].size(1), cap = srcs[0].size(0);
  std::vector<const void*> sp;
  std::vector<void*> dp;
  std::vector<long> rb;
  std::vector<torch::Tensor> outs;
  for (auto& s : srcs) {
    TORCH_CHECK(s.is_cuda() && s.is_contiguous() && s.dim() >= 2 && s.size(0) == cap && s.size(1) == n_envs,
                "gather_rows: every key [capacity, n_envs, ...]");
    std::vector<int64_t> shape{N};
    for (int d = 2; d < s.dim(); ++d) shape.push_back(s.size(d));
    auto o = torch::empty(shape, s.options());
    sp.push_back(s.data_ptr());
    dp.push_back(o.data_ptr());
    rb.push_back((long)(s.numel() / (s.size(0) * n_envs) * s.element_size()));
    outs.push_back(o);
  }
  int* errp = nullptr;
  if (err.has_value() && err->defined()) {
    TORCH_CHECK(err->is_cuda() && err->scalar_type() == torch::kInt && err->numel() >= 1, "gather_rows: err int32 [1]");
    errp = err->data_ptr<int>();
  }
  if (N > 0)
    launch_gather_rows(sp.data(), dp.data(), rb.data(), (int)srcs.size(), (int)n_envs, (long)cap, (int)N, row.data_ptr<int64_t>(),
                       env.data_ptr<int64_t>(), errp, stream());
  return outs;
}

// ------------------------------------------------------------------ tall-layer weight gradients (wgrad.hip)
// dW[N, Kone + Kd] = [onehot(idx) | x]^T dz over M rows, db[N] = colsum(dz).  dz [M, N] and x [M, Kd] row-strided;
// idx [M, >= G] int32 row-strided with table rows idx - off in [0, G*C) (the first Kone = G*C columns of W);
// dW / db written (or added, accumulate=true) into the given contiguous outputs.
void wgrad(torch::Tensor dz, c10::optional<torch::Tensor> x, c10::optional<torch::Tensor> idx, int64_t G, int64_t C,
           int64_t off, torch::Tensor dW, c10::optional<torch::Tensor> db, bool accumulate) {
  TORCH_CHECK(dz.is_cuda() && dz.scalar_type() == torch::kFloat32 && dz.dim() == 2 && dz.stride(1) == 1 &&
                  dz.stride(0) >= dz.size(1),
              "wgrad: dz must be a row-strided float32 [M, N] GPU tensor");
  const int64_t M = dz.size(0), N = dz.size(1);
  const bool has_x = x.has_value() && x->defined();
  const bool has_i = idx.has_value() && idx->defined();
  TORCH_CHECK(has_x || has_i, "wgrad: need x and/or idx");
  const int64_t Kone = has_i ? G * C : 0;
  const int64_t Kd = has_x ? x->size(1) : 0;
  TORCH_CHECK(dW.is_cuda() && dW.scalar_type() == torch::kFloat32 && dW.is_contiguous() && dW.dim() == 2 && dW.size(0) == N &&
                  dW.size(1) == Kone + Kd,
              "wgrad: dW must be a contiguous float32 [N, Kone + Kd] GPU tensor");
  TORCH_CHECK(M > 0 && M < (1LL << 31) && N * (Kone + Kd) < (1LL << 31), "wgrad: sizes out of range");
  const bool has_b = db.has_value() && db->defined();
  if (has_b)
    TORCH_CHECK(db->is_cuda() && db->scalar_type() == torch::kFloat32 && db->is_contiguous() && db->numel() == N,
                "wgrad: db must be a contiguous float32 [N] GPU tensor");
  TORCH_CHECK(!has_b || has_x, "wgrad: the bias column sum rides on the dense part (x required)");
  auto opts = dz.options();
  hipStream_t st = stream();
  if (has_x) {
    TORCH_CHECK(x->is_cuda() && x->scalar_type() == torch::kFloat32 && x->dim() == 2 && x->size(0) == M && x->stride(1) == 1 &&
                    x->stride(0) >= x->size(1),
                "wgrad: x must be a row-strided float32 [M, Kd] GPU tensor");
    const int S = wgrad_dense_chunks((int)M, (int)N, (int)Kd);
    auto part = torch::empty({(int64_t)S * N * Kd}, opts);
    torch::Tensor bpart;
    if (has_b) bpart = torch::empty({(int64_t)S * N}, opts);
    launch_wgrad_dense(dz.data_ptr<float>(), dz.stride(0), x->data_ptr<float>(), x->stride(0), part.data_ptr<float>(),
                       has_b ? bpart.data_ptr<float>() : nullptr, (int)M, (int)N, (int)Kd, S, st);
    launch_wgrad_reduce(part.data_ptr<float>(), S, (int)N, (int)Kd, dW.data_ptr<float>(), Kone + Kd, (int)Kone, accumulate, st);
    if (has_b) launch_wgrad_reduce(bpart.data_ptr<float>(), S, 1, (int)N, db->data_ptr<float>(), N, 0, accumulate, st);
  }
  if (has_i) {
    TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == torch::kInt && idx->dim() == 2 && idx->size(0) == M &&
                    idx->size(1) >= G && idx->stride(1) == 1 && idx->stride(0) >= G,
                "wgrad: idx must be a row-strided int32 [M, >= G] GPU tensor");
    const int S = wgrad_onehot_chunks((int)M, (int)N, (int)G, (int)C);
    TORCH_CHECK(S > 0, "wgrad: one-hot group of ", C, " classes does not fit the LDS accumulator");
    auto part = torch::empty({(int64_t)S * N * Kone}, opts);
    TORCH_CHECK(launch_wgrad_onehot(dz.data_ptr<float>(), dz.stride(0), idx->data_ptr<int>(), idx->stride(0), (int)off,
                                    part.data_ptr<float>(), (int)M, (int)N, (int)G, (int)C, S, st),
                "wgrad: one-hot launch failed");
    launch_wgrad_reduce(part.data_ptr<float>(), S, (int)N, (int)Kone, dW.data_ptr<float>(), Kone + Kd, 0, accumulate, st);
  }
}

// ------------------------------------------------------------------ rollout actor tail (actor_tail.hip)
// y = act(LN(pre)) (+ mean / rstd), logits = y Wh^T + bh, one-hot sample (unimix) into `sample` [M, >= A] and its
// column (ioff + pick) into idx [M, >= 1]; pre / y / sample / idx row-strided.  false: shape not covered.
bool actor_tail(torch::Tensor pre, torch::Tensor y, c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
                torch::Tensor mean, torch::Tensor rstd, double eps, int64_t act, torch::Tensor Wh,
                c10::optional<torch::Tensor> bh, c10::optional<torch::Tensor> uniform, double alpha, torch::Tensor sample,
                c10::optional<torch::Tensor> idx, int64_t ioff, c10::optional<torch::Tensor> logits) {
  const int64_t M = pre.size(0), N = pre.size(1), A = Wh.size(0);
  rowview(pre, "pre", M, N, torch::kFloat32);
  rowview(y, "y", M, N, torch::kFloat32);
  rowview(sample, "sample", M, A, torch::kFloat32);
  TORCH_CHECK(Wh.is_cuda() && Wh.scalar_type() == torch::kFloat32 && Wh.is_contiguous() && Wh.dim() == 2 && Wh.size(1) == N,
              "actor_tail: Wh [A, N] contiguous float32");
  TORCH_CHECK(mean.is_cuda() && mean.numel() == M && rstd.is_cuda() && rstd.numel() == M && mean.is_contiguous() &&
                  rstd.is_contiguous(),
              "actor_tail: mean / rstd [M]");
  const float* gp = optf(gamma, "gamma", N);
  const float* bp = optf(beta, "beta", N);
  const float* hp = optf(bh, "bh", A);
  const float* up = optf(uniform, "uniform", M);
  float* lp = logits.has_value() && logits->defined() ? const_cast<float*>(optf(logits, "logits", M * A)) : nullptr;
  int* ip = nullptr;
  int64_t ldi = 0;
  if (idx.has_value() && idx->defined()) {
    rowview(*idx, "idx", M, 1, torch::kInt);
    ip = idx->data_ptr<int>();
    ldi = idx->stride(0);
  }
  return launch_actor_tail(pre.data_ptr<float>(), pre.stride(0), y.data_ptr<float>(), y.stride(0), gp, bp,
                           mean.data_ptr<float>(), rstd.data_ptr<float>(), (float)eps, (int)act, Wh.data_ptr<float>(), hp,
                           (int)A, up, (float)alpha, sample.data_ptr<float>(), sample.stride(0), ip, ldi, (int)ioff, lp,
                           (int)M, (int)N, stream());
}

// ------------------------------------------------------------------ imagination prior head (prior_head.hip)
// sample = onehot(Categorical(unimix(act(LN(x)) W^T + b))) per 32-class categorical of each row: one-hot rows into
// `sample` [M, >= N] and hot columns (ioff + g * 32 + pick) into idx [M, >= N / 32]; x / sample / idx row-strided;
// uniform [M * N / 32].  false: shape not covered.
bool prior_head(torch::Tensor x, torch::Tensor gamma, torch::Tensor beta, double eps, int64_t act, torch::Tensor W,
                c10::optional<torch::Tensor> b, torch::Tensor uniform, double alpha, torch::Tensor sample,
                c10::optional<torch::Tensor> idx, int64_t ioff, c10::optional<torch::Tensor> logits_out,
                c10::optional<torch::Tensor> mean_out, c10::optional<torch::Tensor> rstd_out) {
  const int64_t M = x.size(0), K = x.size(1), N = W.size(0);
  rowview(x, "x", M, K, torch::kFloat32);
  rowview(sample, "sample", M, N, torch::kFloat32);
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == torch::kFloat32 && W.is_contiguous() && W.dim() == 2 && W.size(1) == K,
              "prior_head: W [N, K] contiguous float32");
  TORCH_CHECK(N % 32 == 0, "prior_head: N must be a multiple of 32 classes");
  const float* gp = optf(gamma, "gamma", K);
  const float* bp = optf(beta, "beta", K);
  const float* hp = optf(b, "b", N);
  const float* up = optf(uniform, "uniform", M * (N / 32));
  int* ip = nullptr;
  int64_t ldi = 0;
  if (idx.has_value() && idx->defined()) {
    rowview(*idx, "idx", M, N / 32, torch::kInt);
    ip = idx->data_ptr<int>();
    ldi = idx->stride(0);
  }
  float* lp = nullptr;
  int64_t ldl = 0;
  if (logits_out.has_value() && logits_out->defined()) {
    rowview(*logits_out, "logits_out", M, N, torch::kFloat32);
    lp = logits_out->data_ptr<float>();
    ldl = logits_out->stride(0);
  }
  float* mp = nullptr;
  float* rp = nullptr;
  if (mean_out.has_value() && mean_out->defined()) {
    TORCH_CHECK(rstd_out.has_value() && rstd_out->defined(), "prior_head: mean_out needs rstd_out");
    mp = const_cast<float*>(optf(*mean_out, "mean_out", M));
    rp = const_cast<float*>(optf(*rstd_out, "rstd_out", M));
  }
  return launch_prior_head(x.data_ptr<float>(), x.stride(0), gp, bp, (float)eps, (int)act, W.data_ptr<float>(), hp, up,
                           (float)alpha, sample.data_ptr<float>(), sample.stride(0), ip, ldi, (int)ioff, (int)M, (int)K,
                           (int)N, stream(), lp, ldl, mp, rp);
}

// Fused replay sequence sample into preallocated [L, B, ...] outputs (gather.hip seq_sample_kernel): srcs are
// the store's keys [cap, n_envs, ...]; starts uniform over [0, n1) U [start2, start2 + n2), envs uniform.
bool seq_sample_into(std::vector<torch::Tensor> srcs, std::vector<torch::Tensor> dsts, int64_t B, int64_t L, int64_t n1,
                     int64_t start2, int64_t n2, int64_t seed, int64_t counter) {
  TORCH_CHECK(srcs.size() == dsts.size() && !srcs.empty() && srcs.size() <= 16, "seq_sample_into: 1..16 matching keys");
  const int64_t cap = srcs[0].size(0), n_envs = srcs[0].size(1);
  std::vector<const void*> sp;
  std::vector<void*> dp;
  std::vector<long> rb;
  for (size_t k = 0; k < srcs.size(); ++k) {
    const auto& s = srcs[k];
    const auto& d = dsts[k];
    TORCH_CHECK(s.is_cuda() && s.is_contiguous() && s.dim() >= 2 && s.size(0) == cap && s.size(1) == n_envs,
                "seq_sample_into: every store key [cap, n_envs, ...] contiguous");
    TORCH_CHECK(d.is_cuda() && d.is_contiguous() && d.dim() == s.dim() && d.size(0) == L && d.size(1) == B &&
                    d.scalar_type() == s.scalar_type(),
                "seq_sample_into: every output [L, B, ...] contiguous with the store's dtype");
    for (int64_t i = 2; i < s.dim(); ++i) TORCH_CHECK(d.size(i) == s.size(i), "seq_sample_into: feature dims differ");
    sp.push_back(s.data_ptr());
    dp.push_back(d.data_ptr());
    rb.push_back((long)(s.numel() / (cap * n_envs) * s.element_size()));
  }
  return launch_seq_sample(sp.data(), dp.data(), rb.data(), (int)srcs.size(), (int)n_envs, (long)cap, (int)B, (int)L,
                           (long)n1, (long)start2, (long)n2, (unsigned long long)seed, (unsigned long long)counter, stream());
}

bool launch_transpose_many(int nj, const float* const* src, const long* lds, const int* rows, const int* cols,
                           float* const* dst, hipStream_t st);

// contiguous transposes of up to 8 row-strided fp32 matrices (unit column stride) in one launch
// (outs: optional contiguous [cols, rows] destinations, e.g. row blocks of one table; None entries allocate)
void launch_side_delay(float us, hipStream_t st);
std::vector<torch::Tensor> transpose_many(std::vector<torch::Tensor> xs, c10::optional<std::vector<c10::optional<torch::Tensor>>> outs) {
  TORCH_CHECK(!xs.empty() && xs.size() <= 8, "transpose_many: 1..8 matrices");
  std::vector<torch::Tensor> out;
  const float* src[8];
  float* dst[8];
  long lds[8];
  int rows[8], cols[8];
  for (size_t j = 0; j < xs.size(); ++j) {
    const torch::Tensor& x = xs[j];
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.dim() == 2 && (x.stride(1) == 1 || x.size(1) <= 1),
                "transpose_many: fp32 2-D GPU matrices with unit column stride");
    TORCH_CHECK(x.size(0) < (1 << 30) && x.size(1) < (1 << 30), "transpose_many: too large");
    torch::Tensor y;
    if (outs.has_value() && j < outs->size() && (*outs)[j].has_value() && (*outs)[j]->defined()) {
      y = *(*outs)[j];
      TORCH_CHECK(y.is_cuda() && y.scalar_type() == torch::kFloat32 && y.is_contiguous() && y.dim() == 2 &&
                      y.size(0) == x.size(1) && y.size(1) == x.size(0), "transpose_many: out ", j, " must be contiguous [cols, rows]");
    } else {
      y = torch::empty({x.size(1), x.size(0)}, x.options());
    }
    src[j] = x.data_ptr<float>();
    dst[j] = y.data_ptr<float>();
    lds[j] = x.size(0) > 1 ? (long)x.stride(0) : (long)x.size(1);
    rows[j] = (int)x.size(0);
    cols[j] = (int)x.size(1);
    out.push_back(y);
  }
  TORCH_CHECK(launch_transpose_many((int)xs.size(), src, lds, rows, cols, dst, stream()), "transpose_many: launch");
  return out;
}

void register_ext(pybind11::module& m) {
  m.def("actor_loss_cont", &actor_loss_cont);
  m.def("sac_critic_fwd", &sac_critic_fwd);
  m.def("sac_critic_wgrad", &sac_critic_wgrad);
  m.def("gather_rows", &gather_rows, pybind11::arg("srcs"), pybind11::arg("row"), pybind11::arg("env"),
        pybind11::arg("err") = pybind11::none());
  m.def("onehot_index", &onehot_index);
  m.def("seq_sample_into", &seq_sample_into);
  m.def("transpose_many", &transpose_many, pybind11::arg("xs"), pybind11::arg("outs") = pybind11::none());
  m.def("side_delay", [](double us) { launch_side_delay((float)us, stream()); });
  m.def("actor_tail", &actor_tail, pybind11::arg("pre"), pybind11::arg("y"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("eps"), pybind11::arg("act"), pybind11::arg("Wh"),
        pybind11::arg("bh"), pybind11::arg("uniform"), pybind11::arg("alpha"), pybind11::arg("sample"), pybind11::arg("idx"),
        pybind11::arg("ioff"), pybind11::arg("logits") = pybind11::none());
  m.def("prior_head", &prior_head, pybind11::arg("x"), pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("eps"),
        pybind11::arg("act"), pybind11::arg("W"), pybind11::arg("b"), pybind11::arg("uniform"), pybind11::arg("alpha"),
        pybind11::arg("sample"), pybind11::arg("idx"), pybind11::arg("ioff"), pybind11::arg("logits_out") = pybind11::none(),
        pybind11::arg("mean_out") = pybind11::none(), pybind11::arg("rstd_out") = pybind11::none());
  m.def("wgrad", &wgrad, pybind11::arg("dz"), pybind11::arg("x"), pybind11::arg("idx"), pybind11::arg("G"), pybind11::arg("C"),
        pybind11::arg("off"), pybind11::arg("dW"), pybind11::arg("db"), pybind11::arg("accumulate") = false);
  m.def("onehot_gather_ln", &onehot_gather_ln, pybind11::arg("Y"), pybind11::arg("idx"), pybind11::arg("G"), pybind11::arg("off"),
        pybind11::arg("table"), pybind11::arg("bias"), pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("eps"),
        pybind11::arg("act"), pybind11::arg("ln"), pybind11::arg("z_out"), pybind11::arg("y_out"), pybind11::arg("mean"),
        pybind11::arg("rstd"), pybind11::arg("err") = pybind11::none(), pybind11::arg("xa") = pybind11::none(),
        pybind11::arg("Wa") = pybind11::none());
  m.def("gru_cell_fwd", &gru_cell_fwd);
  m.def("gru_cell_bwd", &gru_cell_bwd);
  m.def("lstm_fwd", &lstm_fwd);
  m.def("lstm_bwd", &lstm_bwd, pybind11::arg("Whh"), pybind11::arg("c0"), pybind11::arg("gates"), pybind11::arg("cs"),
        pybind11::arg("dout"), pybind11::arg("dhT") = pybind11::none(), pybind11::arg("dcT") = pybind11::none());
  m.def("imag_discount", &imag_discount, pybind11::arg("clog"), pybind11::arg("dones"), pybind11::arg("gamma"),
        pybind11::arg("skip_first") = false);
  m.def("ens_disagreement", &ens_disagreement);
  m.def("wm_loss_fwd", &wm_loss_fwd);
  m.def("wm_loss_bwd", &wm_loss_bwd);
  m.def("symlog_cat", &symlog_cat);
  m.def("obs_mse_fwd", &obs_mse_fwd);
  m.def("obs_mse_bwd", &obs_mse_bwd);
  m.def("sac_twin_q_target", &sac_twin_q_target);
  m.def("skinny_nt", &skinny_nt, pybind11::arg("A"), pybind11::arg("W"), pybind11::arg("out"),
        pybind11::arg("add") = pybind11::none(), pybind11::arg("part") = pybind11::none());
  m.def("skinny_workspace", &skinny_workspace);
  m.def("actor_loss_discrete", &actor_loss_discrete);
  m.def("moments_update", &moments_update);
  m.def("nc_conv_fwd", &nc_conv_fwd);
  m.def("nc_conv_bwd", &nc_conv_bwd);
}
