"""One-launch weight + bias gradient (csrc/wgrad.hip) against a plain PyTorch fp32
reference of the same op on the same bf16 rows: dW = dy^T x, db = sum_r dy.  fp32
accumulation in both; tolerance 1e-5 relative (summation order only)."""
import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,N,K", [(16384, 768, 256), (16384, 256, 128), (8192, 640, 256),
                                   (8192, 3, 256), (1024, 256, 256), (1000, 12, 100),
                                   (33, 130, 70), (1, 8, 8)])
@pytest.mark.parametrize("bias", [True, False])
def test_fused_weight_grad(cuda, R, N, K, bias):
    from ov3d_amd import gemm
    torch.manual_seed(R + N + K)
    dy = torch.randn(R, N, device=cuda).to(torch.bfloat16)
    x = torch.randn(R, K, device=cuda).to(torch.bfloat16)
    dw, db = gemm.fused_weight_grad(dy, x, bias=bias)
    ref = dy.float().t() @ x.float()
    assert ((dw - ref).norm() / ref.norm()).item() < 1e-5
    if bias:
        rb = dy.float().sum(0)
        assert ((db - rb).norm() / rb.norm()).item() < 1e-5
    else:
        assert db is None


def test_fused_weight_grad_into_row_slices(cuda):
    """_InProj writes each projection block's gradient into rows of ONE (3E, E) buffer."""
    from ov3d_amd import gemm
    E, R = 256, 4096
    dw = torch.full((3 * E, E), 7.0, device=cuda)
    db = torch.full((3 * E,), 7.0, device=cuda)
    refs = []
    for i in range(3):
        dy = torch.randn(R, E, device=cuda).to(torch.bfloat16)
        x = torch.randn(R, E, device=cuda).to(torch.bfloat16)
        gemm.fused_weight_grad(dy, x, True, out_w=dw[i * E:(i + 1) * E], out_b=db[i * E:(i + 1) * E])
        refs.append((dy.float().t() @ x.float(), dy.float().sum(0)))
    for i, (rw, rb) in enumerate(refs):
        assert ((dw[i * E:(i + 1) * E] - rw).norm() / rw.norm()).item() < 1e-5
        assert ((db[i * E:(i + 1) * E] - rb).norm() / rb.norm()).item() < 1e-5
