"""Implicit-GEMM k4 s2 p1 convolutions (ops/csrc/conv.hip) against fp32 PyTorch references:
each GEMM form on its own (DOWN = Conv2d fwd / ConvT data-grad, UP = ConvT fwd / Conv2d data-grad,
WGRAD) and the whole DreamerV3 encoder / decoder stacks, forward and every parameter gradient, at the
Atari-100k shapes (mult 32, 64 px RGB) and at the L / XL presets' (reference
configs/exp/dreamer_v3_XL_crafter.yaml:40-46 mult 96, dreamer_v3_L_doapp_128px_gray_combo_discrete.yaml
mult 64 at 128 px grayscale: 5 stages, 1024 channels)."""
import pytest
import torch
import torch.nn.functional as F

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.ops import conv as conv_ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, rtol=2e-4, atol=2e-4):
    scale = b.abs().max().clamp_min(1.0)
    torch.testing.assert_close(a / scale, b / scale, rtol=rtol, atol=atol)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("cin,cout,hw,n", [(4, 32, 64, 3), (32, 64, 32, 2), (64, 128, 16, 5), (128, 256, 8, 4),
                                            (4, 96, 64, 2), (96, 192, 32, 2), (192, 384, 16, 2), (384, 768, 8, 3),
                                            (256, 512, 8, 2), (512, 1024, 8, 3), (4, 64, 128, 1), (96, 96, 8, 2)])
def test_down_plain_matches_conv2d(cin, cout, hw, n):
    C = ops._ext()
    torch.manual_seed(0)
    x = torch.randn(n, cin, hw, hw, device=DEV)
    w = torch.randn(cout, cin, 4, 4, device=DEV) * 0.1
    ref = F.conv2d(x, w, stride=2, padding=1)
    wp = C.conv_pack_down(w, cin)
    out = C.conv_gemm(0, _nhwc(x), wp, cout, 2, None, None, 0.0, 0, True, None, None, None, None, None, None, 0.0, cout)[0]
    _close(out, ref)


@pytest.mark.parametrize("cin,cout,hw,n", [(256, 128, 4, 3), (128, 64, 8, 2), (64, 32, 16, 5), (64, 256, 4, 2),
                                            (768, 384, 4, 3), (384, 192, 8, 2), (192, 96, 16, 2), (1024, 512, 4, 2),
                                            (512, 256, 8, 2), (96, 768, 4, 2), (32, 1024, 4, 2)])
def test_up_plain_matches_conv_transpose(cin, cout, hw, n):
    C = ops._ext()
    torch.manual_seed(0)
    x = torch.randn(n, cin, hw, hw, device=DEV)
    w = torch.randn(cin, cout, 4, 4, device=DEV) * 0.1
    b = torch.randn(cout, device=DEV)
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=1) + 0.5
    wp = C.conv_pack_up(w, cout)
    out = C.conv_gemm(1, _nhwc(x), wp, cout, 2, None, None, 0.0, 0, True, None, None, None, None, None, b, 0.5, cout)[0]
    _close(out, ref)


@pytest.mark.parametrize("cin,cout,hw,n", [(4, 32, 64, 3), (32, 64, 32, 2), (64, 128, 16, 3), (128, 256, 8, 4),
                                            (4, 96, 64, 2), (96, 192, 32, 2), (192, 384, 16, 2), (384, 768, 8, 2),
                                            (512, 1024, 8, 2), (4, 64, 128, 1), (768, 96, 8, 2), (1024, 64, 8, 2),
                                            (96, 192, 32, 24), (192, 384, 16, 40), (384, 768, 8, 96)])
def test_wgrad_matches_autograd(cin, cout, hw, n):
    C = ops._ext()
    torch.manual_seed(0)
    x = torch.randn(n, cin, hw, hw, device=DEV)
    w = (torch.randn(cout, cin, 4, 4, device=DEV) * 0.1).requires_grad_(True)
    y = F.conv2d(x, w, stride=2, padding=1)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    dw = C.conv_wgrad(_nhwc(g), _nhwc(x), cin)
    _close(dw, w.grad, rtol=5e-4, atol=5e-4)


@pytest.mark.parametrize("form", [0, 1])
@pytest.mark.parametrize("ca,co,hw", [(32, 3, 32), (96, 3, 32), (64, 1, 64), (128, 4, 16), (64, 2, 32), (32, 3, 16)])
def test_up_small_matches_conv_transpose(ca, co, hw, form):
    """The decoder's final ConvTranspose2d: form 0 = input-centric MFMA kernel (default), 1 = VALU form."""
    C = ops._ext()
    torch.manual_seed(0)
    x = torch.randn(3, ca, hw, hw, device=DEV)
    w = torch.randn(ca, co, 4, 4, device=DEV) * 0.1
    b = torch.randn(co, device=DEV)
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=1) + 0.5
    C.set_up_last_form(form)
    try:
        out = C.conv_up_small(_nhwc(x), w, b, 0.5)
    finally:
        C.set_up_last_form(0)
    _close(out, ref)


def _encoder_decoder(mult=32, hw=64, ch=3):
    from sheeprl_prey_amd.algos.dreamer_v3.agent import CNNDecoder, CNNEncoder

    torch.manual_seed(0)
    stages = hw.bit_length() - 3  # reference: log2(screen_size) - log2(4)
    enc = CNNEncoder(["rgb"], [ch], (hw, hw), mult, stages=stages).to(DEV)
    dec = CNNDecoder(["rgb"], [ch], mult, 96, enc.output_dim, (hw, hw), stages=stages).to(DEV)
    with torch.no_grad():  # non-trivial LN affine parameters
        for m in list(enc.modules()) + list(dec.modules()):
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return enc, dec


def _run(enc, dec, x, lat, g_e, g_d, fused):
    ops.set_fused(fused)
    try:
        for p in list(enc.parameters()) + list(dec.parameters()):
            p.grad = None
        lat = lat.detach().clone().requires_grad_(True)
        e = enc({"rgb": x})
        r = dec(lat)["rgb"]
        ((e * g_e).sum() + (r * g_d).sum()).backward()
        grads = {n: p.grad.clone() for n, p in list(enc.named_parameters()) + [("d." + k, v) for k, v in dec.named_parameters()]}
        return e.detach(), r.detach(), lat.grad.clone(), grads
    finally:
        ops.set_fused(True)


@pytest.mark.parametrize("lead,mult,hw,ch", [((6,), 32, 64, 3), ((3, 2), 32, 64, 3), ((66,), 32, 64, 3),
                                             ((5,), 96, 64, 3), ((3,), 64, 128, 1), ((4,), 64, 64, 3)])
def test_encoder_decoder_stacks_match_eager(lead, mult, hw, ch, monkeypatch):
    monkeypatch.setattr(conv_ops, "MIN_FRAMES", 1)  # small batches normally go to MIOpen
    enc, dec = _encoder_decoder(mult, hw, ch)
    assert conv_ops.encoder_spec(enc.model, (hw, hw), ch) is not None
    assert conv_ops.decoder_spec(dec.model, ch) is not None
    x = torch.rand(*lead, ch, hw, hw, device=DEV)
    lat = torch.randn(*lead, 96, device=DEV)
    g_e = torch.randn(*lead, enc.output_dim, device=DEV)
    g_d = torch.randn(*lead, ch, hw, hw, device=DEV)
    e1, r1, dl1, gr1 = _run(enc, dec, x, lat, g_e, g_d, True)
    e0, r0, dl0, gr0 = _run(enc, dec, x, lat, g_e, g_d, False)
    _close(e1, e0)
    _close(r1, r0)
    _close(dl1, dl0, rtol=5e-4, atol=5e-4)
    for k in gr0:
        _close(gr1[k], gr0[k], rtol=1e-3, atol=1e-3)


def test_stack_ineligible_falls_back():
    enc, _ = _encoder_decoder(mult=4)  # channels 4..32: not on the fused path
    assert conv_ops.encoder_spec(enc.model, (64, 64), 3) is None
    out = enc({"rgb": torch.rand(2, 3, 64, 64, device=DEV)})
    assert out.shape == (2, enc.output_dim)


@pytest.mark.parametrize("n,hw,c", [(1024, 16, 256), (66, 16, 768), (7, 4, 32)])
def test_ln_bwd_flat_matches_autograd_and_is_deterministic(n, hw, c):
    """The encoder's last LayerNorm+SiLU backward with dy in NCHW-flat order (the image-tiled kernel: coalesced dy
    through an LDS transpose, dgamma / dbeta as fixed-order block partials) against autograd in fp64; two runs give
    bitwise-equal dgamma / dbeta."""
    C = ops._ext()
    torch.manual_seed(n + c)
    z = torch.randn(n, hw, c, device=DEV)
    gamma, beta = torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV) * 0.2
    dy = torch.randn(n, c * hw, device=DEV)
    z64 = z.double().requires_grad_()
    g64, b64 = gamma.double().requires_grad_(), beta.double().requires_grad_()
    y = torch.nn.functional.silu(torch.nn.functional.layer_norm(z64, (c,), g64, b64, 1e-5))
    y.permute(0, 2, 1).reshape(n, c * hw).mul(dy.double()).sum().backward()
    mean = z.mean(-1).reshape(-1)
    rstd = torch.rsqrt(z.var(-1, unbiased=False) + 1e-5).reshape(-1)
    outs = []
    for _ in range(2):
        dg, db = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)
        dz = C.conv_ln_bwd_flat(dy, z.view(n, 1, hw, c), mean, rstd, gamma, beta, ops._act_code("silu"), dg, db)
        outs.append((dz, dg, db))
    torch.testing.assert_close(outs[0][0].view(n, hw, c).double(), z64.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(outs[0][1].double(), g64.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(outs[0][2].double(), b64.grad, rtol=1e-4, atol=1e-3)
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])


def test_stack_grads_are_bitwise_reproducible(monkeypatch):
    """The fused stacks' LayerNorm-backward GEMM epilogues write per-workgroup column sums that a fixed-order kernel
    reduces (no float atomics): two identical fwd+bwd passes give bitwise-equal gradients of every parameter."""
    monkeypatch.setattr(conv_ops, "MIN_FRAMES", 1)
    enc, dec = _encoder_decoder(32, 64, 3)
    torch.manual_seed(1)
    x = torch.rand(66, 3, 64, 64, device=DEV)
    lat = torch.randn(66, 96, device=DEV)
    g_e = torch.randn(66, enc.output_dim, device=DEV)
    g_d = torch.randn(66, 3, 64, 64, device=DEV)
    runs = [_run(enc, dec, x, lat, g_e, g_d, True) for _ in range(2)]
    diff = [k for k in runs[0][3] if not torch.equal(runs[0][3][k], runs[1][3][k])]
    assert not diff, f"gradients differ run to run: {diff}"
    assert torch.equal(runs[0][2], runs[1][2])


@pytest.mark.parametrize("n,c,hw", [(5, 3, 64), (3, 1, 64), (2, 3, 6), (4, 4, 16)])
def test_to_nhwc4_uint8_matches_permute(n, c, hw):
    """The encoder input conversion: uint8 NCHW frames -> NHWC4 f32 scaled by 1/255 (channels past C zero); the
    4-pixel form (HW % 4 == 0) and the per-pixel form (HW = 36)."""
    C = ops._ext()
    x = torch.randint(0, 256, (n, c, hw, hw), dtype=torch.uint8, device=DEV)
    out = C.conv_to_nhwc4(x, 1.0 / 255.0)
    ref = torch.zeros(n, hw, hw, 4, device=DEV)
    ref[..., :c] = x.permute(0, 2, 3, 1).float() * (1.0 / 255.0)
    torch.testing.assert_close(out, ref, rtol=0, atol=1e-7)
