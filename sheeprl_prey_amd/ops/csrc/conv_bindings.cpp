// Torch bindings of the implicit-GEMM k4 s2 p1 convolutions (conv.hip).  Shapes are checked here,
// before any launch: every kernel assumes power-of-two grids, NHWC inputs, channel counts that are
// multiples of 32 (or a power of two below 32 on the image side) and 32-bit element offsets.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>

#include "conv.h"

using srl::conv::ConvEpi;

bool launch_conv_down(const float*, const float*, int, int, int, int, int, const ConvEpi&, hipStream_t);
bool launch_conv_up(const float*, const float*, int, int, int, int, int, const ConvEpi&, hipStream_t);
void conv_wgrad_plan(int, int, int, int, int, int*, int*);
bool launch_conv_wgrad(const float*, const float*, float*, float*, int, int, int, int, int, int, hipStream_t);
void launch_pack_down(const float*, float*, int, int, int, hipStream_t);
void launch_pack_up(const float*, float*, int, int, int, hipStream_t);
bool launch_multi_pack(const float* const*, float* const*, const int*, const int*, const int*, const int*, int, hipStream_t);
void launch_to_nhwc4(const void*, bool, float*, int, int, int, float, hipStream_t);
void launch_to_nhwc4_sum(const float*, float*, int, int, int, float*, float*, hipStream_t);
bool launch_ln_bwd_flat(const float*, const float*, const float*, const float*, const float*, const float*, float*, float*,
                        float*, int, int, int, int, float*, int, hipStream_t);
bool launch_up_small(const float*, const float*, const float*, float, float*, int, int, int, int, int, hipStream_t);
void set_up_last_form(int);
bool conv_channels_supported(int);
int conv_tile_rows(int, int);
int conv_part_alloc_rows(int);
bool launch_part_reduce_many(const float* const*, const int*, const int*, float* const*, float* const*, const int*, int,
                             float*, bool, hipStream_t);

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

bool pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

void chk(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), name,
              " must be a contiguous float32 GPU tensor");
}
const float* optp(const c10::optional<torch::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  chk(*t, "optional operand");
  return t->data_ptr<float>();
}
float* optw(const c10::optional<torch::Tensor>& t) { return const_cast<float*>(optp(t)); }

// x: [N, H, W, C] NHWC
void chk_nhwc(const torch::Tensor& x, const char* name) {
  chk(x, name);
  TORCH_CHECK(x.dim() == 4, name, " must be NHWC [N,H,W,C]");
  const int64_t C = x.size(3);
  TORCH_CHECK(pow2(x.size(1)) && pow2(x.size(2)) && (C % 32 == 0 || (pow2(C) && C >= 4 && C < 32)), name,
              ": H and W must be powers of two, C a multiple of 32 (or 4, 8, 16)");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31), name, ": too large for 32-bit element offsets");
}

ConvEpi make_epi(int64_t mode, int64_t M, int64_t Nc, const torch::Tensor& out0, const c10::optional<torch::Tensor>& gamma,
                 const c10::optional<torch::Tensor>& beta, double eps, int64_t act) {
  ConvEpi e{};
  e.mode = (int)mode;
  (void)out0;
  (void)Nc;
  e.ln.gamma = optp(gamma);
  e.ln.beta = optp(beta);
  e.ln.eps = (float)eps;
  e.ln.act = (int)act;
  e.ln.M = (int)M;
  e.lb.gamma = e.ln.gamma;
  e.lb.beta = e.ln.beta;
  e.lb.act = (int)act;
  e.lb.M = (int)M;
  e.pl.M = (int)M;
  return e;
}

int ilog2(int64_t v) {
  int l = 0;
  while ((int64_t(1) << l) < v) ++l;
  return l;
}

}  // namespace

torch::Tensor conv_pack_down(torch::Tensor w, int64_t Bp) {
  chk(w, "w");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 4 && w.size(3) == 4, "pack_down: weight must be [A,B,4,4]");
  TORCH_CHECK(Bp >= w.size(1) && Bp % 4 == 0, "pack_down: bad padding");
  auto out = torch::empty({w.size(0), 16, Bp}, w.options());
  launch_pack_down(w.data_ptr<float>(), out.data_ptr<float>(), w.size(0), w.size(1), Bp, stream());
  return out;
}

torch::Tensor conv_pack_up(torch::Tensor w, int64_t Bp) {
  chk(w, "w");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 4 && w.size(3) == 4, "pack_up: weight must be [A,B,4,4]");
  TORCH_CHECK(Bp >= w.size(1), "pack_up: bad padding");
  auto out = torch::empty({4, Bp, 4, w.size(0)}, w.options());
  launch_pack_up(w.data_ptr<float>(), out.data_ptr<float>(), w.size(0), w.size(1), Bp, stream());
  return out;
}

// Every pack of a stack in one launch: jobs (w [A,B,4,4], kind 0 = DOWN / 1 = UP, Bp) -> the packed tensors, in order
std::vector<torch::Tensor> conv_pack_many(std::vector<torch::Tensor> ws, std::vector<int64_t> kinds, std::vector<int64_t> bps) {
  const size_t n = ws.size();
  TORCH_CHECK(n >= 1 && n <= 16 && kinds.size() == n && bps.size() == n, "pack_many: 1..16 jobs");
  std::vector<torch::Tensor> outs;
  std::vector<const float*> wp(n);
  std::vector<float*> op(n);
  std::vector<int> A(n), B(n), Bp(n), K(n);
  for (size_t j = 0; j < n; ++j) {
    auto& w = ws[j];
    chk(w, "w");
    TORCH_CHECK(w.dim() == 4 && w.size(2) == 4 && w.size(3) == 4, "pack_many: weight must be [A,B,4,4]");
    TORCH_CHECK(bps[j] >= w.size(1) && (kinds[j] == 1 || bps[j] % 4 == 0), "pack_many: bad padding");
    TORCH_CHECK(kinds[j] == 0 || kinds[j] == 1, "pack_many: kind 0 (DOWN) or 1 (UP)");
    outs.push_back(kinds[j] == 0 ? torch::empty({w.size(0), 16, bps[j]}, w.options())
                                 : torch::empty({4, bps[j], 4, w.size(0)}, w.options()));
    wp[j] = w.data_ptr<float>();
    op[j] = outs.back().data_ptr<float>();
    A[j] = (int)w.size(0);
    B[j] = (int)w.size(1);
    Bp[j] = (int)bps[j];
    K[j] = (int)kinds[j];
  }
  TORCH_CHECK(launch_multi_pack(wp.data(), op.data(), A.data(), B.data(), Bp.data(), K.data(), (int)n, stream()),
              "pack_many: launch");
  return outs;
}

// DOWN: Q NHWC [N, 2SH, 2SW, Cb], Wp [Nc, 16, Cb] -> outputs on [N, SH, SW, Nc]
// mode 0: LN_ACT -> (z, y, mean, rstd); y_nchw: y as [N, Nc*SH*SW] (C,H,W order)
// mode 1: LN_BWD (ln_z/ln_mean/ln_rstd of the output layer, dgamma/dbeta accumulated) -> (dz)
// mode 2: PLAIN (bias, c0, Nreal, nchw) -> (out)
static std::vector<torch::Tensor> conv_gemm_impl(int64_t kind, torch::Tensor src, torch::Tensor Wp, int64_t Nc, int64_t mode,
                                                 c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
                                                 double eps, int64_t act, bool out_nchw, c10::optional<torch::Tensor> ln_z,
                                                 c10::optional<torch::Tensor> ln_mean, c10::optional<torch::Tensor> ln_rstd,
                                                 c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta,
                                                 c10::optional<torch::Tensor> bias, double c0, int64_t Nreal, bool defer) {
  chk_nhwc(src, "conv input");
  chk(Wp, "packed weight");
  const bool down = kind == 0;
  const int64_t N = src.size(0), H = src.size(1), W = src.size(2), C = src.size(3);
  TORCH_CHECK(conv_channels_supported((int)Nc), "conv: output channels must be 32, 64, 96, 128, 192, 256, 384, 512, 768 or 1024");
  int64_t OH, OW, M;
  if (down) {
    TORCH_CHECK(H >= 2 && W >= 2, "conv down: input too small");
    OH = H / 2;
    OW = W / 2;
    M = N * OH * OW;
    TORCH_CHECK(Wp.numel() == Nc * 16 * C, "conv down: packed weight has the wrong size");
  } else {
    TORCH_CHECK(C % 32 == 0, "conv up: input channels must be a multiple of 32");
    OH = 2 * H;
    OW = 2 * W;
    M = N * H * W;  // per parity class
    TORCH_CHECK(Wp.numel() == 4 * Nc * 4 * C, "conv up: packed weight has the wrong size");
  }
  TORCH_CHECK(N * OH * OW * Nc < (int64_t(1) << 31), "conv: tensor too large for 32-bit pixel indices");
  auto opts = src.options();
  ConvEpi e = make_epi(mode, M, Nc, src, gamma, beta, eps, act);
  std::vector<torch::Tensor> outs;
  const int lHW = ilog2(OH * OW);
  if (mode == 0) {
    auto z = torch::empty({N, OH, OW, Nc}, opts);
    auto y = out_nchw ? torch::empty({N, Nc * OH * OW}, opts) : torch::empty({N, OH, OW, Nc}, opts);
    auto mean = torch::empty({N * OH * OW}, opts);
    auto rstd = torch::empty({N * OH * OW}, opts);
    e.ln.z = z.data_ptr<float>();
    e.ln.y = y.data_ptr<float>();
    e.ln.mean = mean.data_ptr<float>();
    e.ln.rstd = rstd.data_ptr<float>();
    e.ln.y_nchw = out_nchw ? 1 : 0;
    e.ln.lHW = lHW;
    outs = {z, y, mean, rstd};
  } else if (mode == 1) {
    TORCH_CHECK(ln_z.has_value() && ln_mean.has_value() && ln_rstd.has_value(), "conv LN_BWD needs z/mean/rstd");
    TORCH_CHECK(ln_z->numel() == N * OH * OW * Nc && ln_mean->numel() == N * OH * OW, "conv LN_BWD: saved stats size");
    auto dz = torch::empty({N, OH, OW, Nc}, opts);
    e.lb.z = optp(ln_z);
    e.lb.mean = optp(ln_mean);
    e.lb.rstd = optp(ln_rstd);
    e.lb.dz = dz.data_ptr<float>();
    e.lb.dgamma = defer ? nullptr : optw(dgamma);
    e.lb.dbeta = defer ? nullptr : optw(dbeta);
    // per-workgroup column sums (one row per workgroup of the launch), summed in a fixed order after the GEMM -
    // right behind it, or (defer) by the caller's conv_part_reduce_many with the other layers' (deterministic)
    const int64_t rows = (M + conv_tile_rows((int)Nc, 1) - 1) / conv_tile_rows((int)Nc, 1) * (down ? 1 : 4);
    outs = {dz};
    if (defer) {
      auto part = torch::empty({rows, 2 * Nc}, opts);
      e.lb.part = part.data_ptr<float>();
      e.lb.part_rows = (int)rows;
      e.lb.defer = 1;
      outs.push_back(part);
    } else if (e.lb.dgamma || e.lb.dbeta) {
      auto part = torch::empty({conv_part_alloc_rows((int)rows), 2 * Nc}, opts);
      e.lb.part = part.data_ptr<float>();
      e.lb.part_rows = (int)rows;  // freed on return: stream-ordered reuse by the caching allocator is safe
    }
  } else {
    TORCH_CHECK(Nreal >= 1 && Nreal <= Nc, "conv PLAIN: bad Nreal");
    auto out = out_nchw ? torch::empty({N, Nreal, OH, OW}, opts) : torch::empty({N, OH, OW, Nreal}, opts);
    e.pl.out = out.data_ptr<float>();
    e.pl.bias = optp(bias);
    e.pl.c0 = (float)c0;
    e.pl.Nreal = (int)Nreal;
    e.pl.nchw = out_nchw ? 1 : 0;
    e.pl.lHW = lHW;
    outs = {out};
  }
  bool ok = down ? launch_conv_down(src.data_ptr<float>(), Wp.data_ptr<float>(), N, OH, OW, C, Nc, e, stream())
                 : launch_conv_up(src.data_ptr<float>(), Wp.data_ptr<float>(), N, H, W, C, Nc, e, stream());
  TORCH_CHECK(ok, "conv: unsupported configuration");
  return outs;
}

std::vector<torch::Tensor> conv_gemm(int64_t kind, torch::Tensor src, torch::Tensor Wp, int64_t Nc, int64_t mode,
                                     c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta, double eps,
                                     int64_t act, bool out_nchw, c10::optional<torch::Tensor> ln_z,
                                     c10::optional<torch::Tensor> ln_mean, c10::optional<torch::Tensor> ln_rstd,
                                     c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta,
                                     c10::optional<torch::Tensor> bias, double c0, int64_t Nreal) {
  return conv_gemm_impl(kind, src, Wp, Nc, mode, gamma, beta, eps, act, out_nchw, ln_z, ln_mean, ln_rstd, dgamma, dbeta,
                        bias, c0, Nreal, false);
}

// LN_BWD conv whose dgamma / dbeta partials are left for conv_part_reduce_many -> (dz, part [workgroups, 2 Nc])
std::vector<torch::Tensor> conv_gemm_lnbwd_part(int64_t kind, torch::Tensor src, torch::Tensor Wp, int64_t Nc,
                                                c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
                                                int64_t act, torch::Tensor ln_z, torch::Tensor ln_mean, torch::Tensor ln_rstd) {
  return conv_gemm_impl(kind, src, Wp, Nc, 1, gamma, beta, 0.0, act, false, ln_z, ln_mean, ln_rstd, c10::nullopt,
                        c10::nullopt, c10::nullopt, 0.0, 0, true);
}

// out0[j] (=|+=) column sums of parts[j][:, :C], out1[j] of parts[j][:, C:] (C = W / 2): every deferred partial of a
// stack's backward in two launches
void conv_part_reduce_many(std::vector<torch::Tensor> parts, std::vector<torch::Tensor> out0, std::vector<torch::Tensor> out1,
                           bool assign) {
  const size_t n = parts.size();
  TORCH_CHECK(n >= 1 && n <= 16 && out0.size() == n && out1.size() == n, "part_reduce_many: 1..16 jobs");
  std::vector<const float*> pp(n);
  std::vector<float*> o0(n), o1(n);
  std::vector<int> nb(n), W(n), C(n);
  int64_t stage = 0;
  for (size_t j = 0; j < n; ++j) {
    chk(parts[j], "part");
    chk(out0[j], "out0");
    chk(out1[j], "out1");
    TORCH_CHECK(parts[j].dim() == 2 && parts[j].size(1) % 2 == 0, "part_reduce_many: part [rows, 2C]");
    const int64_t c = parts[j].size(1) / 2;
    TORCH_CHECK(out0[j].numel() == c && out1[j].numel() == c, "part_reduce_many: outputs must have C elements");
    pp[j] = parts[j].data_ptr<float>();
    o0[j] = out0[j].data_ptr<float>();
    o1[j] = out1[j].data_ptr<float>();
    nb[j] = (int)parts[j].size(0);
    W[j] = (int)(2 * c);
    C[j] = (int)c;
    stage += (int64_t)(conv_part_alloc_rows(nb[j]) - nb[j]) * W[j];
  }
  auto st = torch::empty({std::max<int64_t>(stage, 1)}, parts[0].options());
  TORCH_CHECK(launch_part_reduce_many(pp.data(), nb.data(), W.data(), o0.data(), o1.data(), C.data(), (int)n,
                                      st.data_ptr<float>(), assign, stream()),
              "part_reduce_many: launch");
}

// dW[a][b][4][4] = sum_m P[m][a] Q[gather(m, tap)][b]; P NHWC small grid [N,SH,SW,Ca], Q NHWC large [N,2SH,2SW,Cbp]
torch::Tensor conv_wgrad(torch::Tensor P, torch::Tensor Q, int64_t Cb, c10::optional<torch::Tensor> out) {
  chk_nhwc(P, "wgrad P");
  chk_nhwc(Q, "wgrad Q");
  const int64_t N = P.size(0), SH = P.size(1), SW = P.size(2), Ca = P.size(3), Cbp = Q.size(3);
  TORCH_CHECK(Q.size(0) == N && Q.size(1) == 2 * SH && Q.size(2) == 2 * SW, "wgrad: P/Q grids do not match");
  TORCH_CHECK(Ca % 32 == 0 && Ca <= 4096 && Cb <= Cbp && (16 * Cbp) % 64 == 0, "wgrad: channel counts");
  TORCH_CHECK(N * SH * SW < (int64_t(1) << 31), "wgrad: too many pixels");
  int S, kper;
  conv_wgrad_plan(N, SH, SW, Ca, Cbp, &S, &kper);
  auto slab = torch::empty({(int64_t)S, Ca, 16 * Cbp}, P.options());
  torch::Tensor dw;
  if (out.has_value() && out->defined()) {
    dw = *out;  // caller-allocated (e.g. on another stream than the one this runs on)
    TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.dim() == 4 &&
                    dw.size(0) == Ca && dw.size(1) == Cb && dw.size(2) == 4 && dw.size(3) == 4,
                "wgrad: out must be a contiguous float32 [Ca, Cb, 4, 4] GPU tensor");
  } else {
    dw = torch::empty({Ca, Cb, 4, 4}, P.options());
  }
  bool ok = launch_conv_wgrad(P.data_ptr<float>(), Q.data_ptr<float>(), slab.data_ptr<float>(), dw.data_ptr<float>(), N,
                              SH, SW, Ca, Cbp, Cb, stream());
  TORCH_CHECK(ok, "wgrad: unsupported configuration");
  return dw;
}

// NCHW (uint8 or float32, C <= 4) -> NHWC4 float32 scaled
torch::Tensor conv_to_nhwc4(torch::Tensor x, double scale) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4 && x.size(1) <= 4, "to_nhwc4: x must be NCHW with C <= 4");
  const bool u8 = x.scalar_type() == torch::kUInt8;
  TORCH_CHECK(u8 || x.scalar_type() == torch::kFloat32, "to_nhwc4: uint8 or float32");
  auto out = torch::empty({x.size(0), x.size(2), x.size(3), 4}, x.options().dtype(torch::kFloat32));
  launch_to_nhwc4(x.data_ptr(), u8, out.data_ptr<float>(), x.size(0), x.size(1), x.size(2) * x.size(3), (float)scale,
                  stream());
  return out;
}

// f32 NCHW [N, C<=4, H, W] -> (NHWC4 [N, H, W, 4], per-channel sum [C]) in one pass over x (+ a fixed-order reduce)
std::vector<torch::Tensor> conv_to_nhwc4_sum(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) <= 4 && x.is_contiguous() && x.scalar_type() == torch::kFloat32,
              "to_nhwc4_sum: contiguous f32 NCHW with <= 4 channels");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31), "to_nhwc4_sum: too large");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  auto out = torch::empty({N, x.size(2), x.size(3), 4}, x.options());
  auto csum = torch::empty({C}, x.options());
  const int nb = (int)((N * HW + 255) / 256);
  auto part = torch::empty({conv_part_alloc_rows(nb), C}, x.options());
  launch_to_nhwc4_sum(x.data_ptr<float>(), out.data_ptr<float>(), N, C, HW, csum.data_ptr<float>(), part.data_ptr<float>(),
                      stream());
  return {out, csum};
}

// row LN+act backward, dy NCHW-flat [N, C*HW], z NHWC [N, HW, C]
torch::Tensor conv_ln_bwd_flat(torch::Tensor dy, torch::Tensor z, torch::Tensor mean, torch::Tensor rstd,
                               c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta, int64_t act,
                               c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta) {
  chk(dy, "dy");
  chk_nhwc(z, "z");
  chk(mean, "mean");
  chk(rstd, "rstd");
  const int64_t N = z.size(0), HW = z.size(1) * z.size(2), C = z.size(3);
  TORCH_CHECK(dy.numel() == z.numel() && mean.numel() == N * HW, "ln_bwd_flat: sizes");
  auto dz = torch::empty_like(z);
  // per-workgroup dgamma / dbeta partials of the image-tiled kernel (one image per workgroup up to 1024), reduced in a fixed order
  const int64_t nblk = std::min<int64_t>(N, 1024);
  auto part = torch::empty({conv_part_alloc_rows((int)nblk), 2 * C}, z.options());
  bool ok = launch_ln_bwd_flat(dy.data_ptr<float>(), z.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                               optp(gamma), optp(beta), dz.data_ptr<float>(), optw(dgamma), optw(dbeta), N * HW, C, HW,
                               (int)act, part.data_ptr<float>(), (int)nblk, stream());
  TORCH_CHECK(ok, "ln_bwd_flat: channel count must be a multiple of 32 up to 1024");
  return dz;
}

// ConvT forward to CO <= 4 channels (VALU kernel): P NHWC [N,SH,SW,Ca], W [Ca,CO,4,4] -> NCHW [N,CO,2SH,2SW]
torch::Tensor conv_up_small(torch::Tensor P, torch::Tensor W, c10::optional<torch::Tensor> bias, double c0) {
  chk_nhwc(P, "P");
  chk(W, "W");
  const int64_t N = P.size(0), SH = P.size(1), SW = P.size(2), Ca = P.size(3);
  TORCH_CHECK(W.dim() == 4 && W.size(0) == Ca && W.size(2) == 4 && W.size(3) == 4, "up_small: weight shape");
  const int64_t CO = W.size(1);
  auto out = torch::empty({N, CO, 2 * SH, 2 * SW}, P.options());
  bool ok = launch_up_small(P.data_ptr<float>(), W.data_ptr<float>(), optp(bias), (float)c0, out.data_ptr<float>(), N, SH,
                            SW, Ca, CO, stream());
  TORCH_CHECK(ok, "up_small: needs Ca % 32 == 0, 1..4 outputs and a grid multiple of 16");
  return out;
}

bool launch_small_conv_stage(const void* x, bool u8, float scale, const float* w, const float* gamma, const float* beta,
                             float eps, int act, float* part, float* y, int N, int Cin, int Hi, int Wi, int Cout,
                             hipStream_t st);
int small_conv_slices(int M, int Cout, int Cin);

// Small-batch encoder stack (conv_small.hip): x [N, C, H, W] float or uint8 (scaled by `scale`), stages of
// k4 s2 p1 conv (no bias) + LayerNormChannelLast + activation -> flat [N, C_L * H_L * W_L] (C, H, W order).
torch::Tensor conv_small_encoder(torch::Tensor x, std::vector<torch::Tensor> ws, std::vector<torch::Tensor> gs,
                                 std::vector<torch::Tensor> bs, std::vector<double> eps, std::vector<int64_t> act,
                                 double scale) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous() &&
                  (x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kUInt8),
              "small encoder: x must be a contiguous NCHW float32 / uint8 CUDA tensor");
  const size_t L = ws.size();
  TORCH_CHECK(L >= 1 && gs.size() == L && bs.size() == L && eps.size() == L && act.size() == L, "small encoder: stage lists");
  const int N = (int)x.size(0);
  int C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  int64_t work = 0;
  {
    int c = C, h = H, w = W;
    for (size_t i = 0; i < L; ++i) {
      chk(ws[i], "small encoder weight");
      chk(gs[i], "small encoder LN weight");
      chk(bs[i], "small encoder LN bias");
      const int co = (int)ws[i].size(0);
      TORCH_CHECK(ws[i].dim() == 4 && ws[i].size(1) == c && ws[i].size(2) == 4 && ws[i].size(3) == 4,
                  "small encoder: weight ", i, " must be [Cout, ", c, ", 4, 4]");
      TORCH_CHECK(gs[i].numel() == co && bs[i].numel() == co, "small encoder: LN parameters of stage ", i);
      TORCH_CHECK(h % 2 == 0 && w % 2 == 0 && h >= 2 && w >= 2, "small encoder: odd input size at stage ", i);
      h /= 2;
      w /= 2;
      const int M = N * h * w;
      work = std::max<int64_t>(work, (int64_t)small_conv_slices(M, co, c) * M * co);
      c = co;
    }
  }
  auto opt = x.options().dtype(torch::kFloat32);
  torch::Tensor part = torch::empty({work}, opt);
  torch::Tensor cur = x;
  for (size_t i = 0; i < L; ++i) {
    const int co = (int)ws[i].size(0);
    torch::Tensor y = torch::empty({N, co, H / 2, W / 2}, opt);
    const bool u8 = cur.scalar_type() == torch::kUInt8;
    const bool ok = launch_small_conv_stage(cur.data_ptr(), u8, i == 0 ? (float)scale : 1.f, ws[i].data_ptr<float>(),
                                            gs[i].data_ptr<float>(), bs[i].data_ptr<float>(), (float)eps[i], (int)act[i],
                                            part.data_ptr<float>(), y.data_ptr<float>(), N, C, H, W, co, stream());
    TORCH_CHECK(ok, "small encoder: unsupported stage ", i, " (Cout % 16, Cout <= 1024, even sizes, aligned)");
    cur = y;
    C = co;
    H /= 2;
    W /= 2;
  }
  return cur.reshape({N, -1});
}

void register_conv(pybind11::module& m) {
  m.def("conv_pack_down", &conv_pack_down);
  m.def("conv_pack_up", &conv_pack_up);
  m.def("conv_pack_many", &conv_pack_many);
  m.def("conv_gemm", &conv_gemm);
  m.def("conv_wgrad", &conv_wgrad, pybind11::arg("P"), pybind11::arg("Q"), pybind11::arg("Cb"), pybind11::arg("out") = pybind11::none());
  m.def("conv_to_nhwc4", &conv_to_nhwc4);
  m.def("conv_to_nhwc4_sum", &conv_to_nhwc4_sum);
  m.def("conv_gemm_lnbwd_part", &conv_gemm_lnbwd_part);
  m.def("conv_part_reduce_many", &conv_part_reduce_many);
  m.def("conv_ln_bwd_flat", &conv_ln_bwd_flat);
  m.def("conv_up_small", &conv_up_small);
  m.def("set_up_last_form", &set_up_last_form);  // 0 = MFMA final ConvT (default), 1 = VALU (A/B, tests)
  m.def("conv_small_encoder", &conv_small_encoder);
}
