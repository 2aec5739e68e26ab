"""``skinny.hip`` (split-K weight-streaming GEMM for <= 16 rows) vs fp32 torch matmul."""
import pytest
import torch

from sheeprl_prey_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Z,M,N,K,addend", [
    (1, 16, 12288, 5120, None),     # XL GRU projection
    (1, 16, 2048, 4096, "full"),    # XL transition/representation hidden + bias/embedding projection
    (2, 16, 1024, 1024, "bcast"),   # batched heads with a broadcast bias
    (1, 5, 256, 128, "full"),       # short K: a single chunk, no reduce pass
    (1, 1, 128, 128, None),
    (1, 16, 5120, 12288, None),   # XL GRU adjoint (dgx . Wg)
])
def test_skinny_matches_torch(Z, M, N, K, addend):
    torch.manual_seed(N + K + M)
    shape = (Z,) if Z > 1 else ()
    A = torch.randn(*shape, M, K + 4, device="cuda")[..., :K]  # row stride != K
    W = torch.randn(*shape, N, K, device="cuda") / K ** 0.5
    add = None
    if addend == "full":
        add = torch.randn(*shape, M, N, device="cuda")
    elif addend == "bcast":
        add = torch.randn(*shape, 1, N, device="cuda")
    out = torch.empty(*shape, M, N, device="cuda")
    assert ops.skinny_nt(A, W, out, add)
    ref = torch.matmul(A.double(), W.double().transpose(-1, -2))
    if add is not None:
        ref = ref + add.double()
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4)


def test_skinny_in_place_accumulate_and_gate():
    A = torch.randn(16, 1024, device="cuda")
    W = torch.randn(512, 1024, device="cuda")
    acc = torch.randn(16, 512, device="cuda")
    ref = acc + A @ W.t()
    assert ops.skinny_nt(A, W, acc, acc)  # out aliases the addend (DH += du . W1)
    torch.testing.assert_close(acc, ref, rtol=1e-4, atol=1e-4)
    assert not ops.skinny_nt(torch.randn(17, 1024, device="cuda"), W, torch.empty(17, 512, device="cuda"))
    assert not ops.skinny_nt(A, torch.randn(100, 1024, device="cuda"), torch.empty(16, 100, device="cuda"))


