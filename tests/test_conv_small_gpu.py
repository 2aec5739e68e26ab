"""Small-batch (player) encoder stack, csrc/conv_small.hip, vs the eager per-layer modules in fp64 - at the
Atari-100k shape (1 and 3 frames, raw uint8 and scaled float), the XL channel ladder (mult 96) and a 1-channel
128 px 5-stage stack."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _encoder(cin, hw, mult, stages):
    from sheeprl_prey_amd.algos.dreamer_v3.agent import CNNEncoder

    torch.manual_seed(0)
    enc = CNNEncoder(["rgb"], [cin], hw, mult, stages=stages).cuda()
    with torch.no_grad():  # non-trivial LN parameters
        for m in enc.modules():
            if hasattr(m, "normalized_shape") and m.weight is not None:
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return enc


def _reference(enc, x):
    from sheeprl_prey_amd.ops import conv as conv_ops

    e64 = copy.deepcopy(enc).double()
    conv_ops.SMALL_ENABLED = False
    try:
        with torch.no_grad():
            return e64({"rgb": x.double() / 255.0 if x.dtype == torch.uint8 else x.double()})
    finally:
        conv_ops.SMALL_ENABLED = True


@pytest.mark.parametrize("n,raw", [(1, True), (3, False), (1, False)])
def test_small_encoder_atari(n, raw):
    enc = _encoder(3, (64, 64), 32, 4)
    g = torch.Generator(device="cuda").manual_seed(1)
    if raw:
        x = torch.randint(0, 256, (n, 3, 64, 64), device="cuda", generator=g, dtype=torch.int64).to(torch.uint8)
    else:
        x = torch.rand(n, 3, 64, 64, device="cuda", generator=g) - 0.5
    with torch.no_grad():
        y = enc({"rgb": x})
    assert getattr(enc, "_fused_spec", None) is not None, "fused spec not built: the small path did not run"
    ref = _reference(enc, x)
    assert y.shape == ref.shape == (n, 256 * 4 * 4)
    err = (y.double() - ref).abs().max().item()
    assert err < 2e-4, err


def test_small_encoder_xl_ladder_and_gray_128():
    g = torch.Generator(device="cuda").manual_seed(2)
    enc = _encoder(3, (64, 64), 96, 4)  # 96 / 192 / 384 / 768 channels
    x = torch.rand(2, 3, 64, 64, device="cuda", generator=g)
    with torch.no_grad():
        y = enc({"rgb": x})
    ref = _reference(enc, x)
    assert (y.double() - ref).abs().max().item() < 3e-4
    enc = _encoder(1, (128, 128), 32, 5)  # grayscale 128 px, 5 stages
    x = torch.rand(1, 1, 128, 128, device="cuda", generator=g)
    with torch.no_grad():
        y = enc({"rgb": x})
    ref = _reference(enc, x)
    assert y.shape == ref.shape
    assert (y.double() - ref).abs().max().item() < 3e-4


def test_small_encoder_native_called():
    """The no-grad few-frame call goes to the native binding (not the MIOpen modules)."""
    from sheeprl_prey_amd.ops import conv as conv_ops

    enc = _encoder(3, (64, 64), 32, 4)
    calls = []
    orig = conv_ops.encoder_small
    conv_ops.encoder_small = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        with torch.no_grad():
            enc({"rgb": torch.zeros(1, 3, 64, 64, device="cuda", dtype=torch.uint8)})
    finally:
        conv_ops.encoder_small = orig
    assert calls == [1]
