"""ov3d_project_box2d (csrc/project.hip) against the REFERENCE projection
(tests/golden/geometry.npz: utils/image_util.py:117-146 project_box_3d_cuda + the
criterion.py:386-391 clamp, run by make_golden.py) and against the host restatement
(image_util.project_boxes_2d on CPU tensors) on many boxes, including boxes behind the
camera, clamped at every edge, and NaN inputs (torch's min / clamp keep NaN)."""
import numpy as np
import pytest
import torch

from helpers import fixture

pytestmark = pytest.mark.gpu


def test_projection_matches_reference_golden(cuda):
    from ov3d_amd.image_util import project_boxes_2d
    fx = fixture("geometry.npz")
    B = fx["center_img"].shape[0]
    args = [torch.from_numpy(fx[k]).to(cuda) for k in ("center_img", "size", "angle")]
    out = project_boxes_2d(*args, torch.from_numpy(fx["Rtilt"]).repeat(B, 1, 1).to(cuda),
                           torch.from_numpy(fx["K"]).repeat(B, 1, 1).to(cuda),
                           torch.full((B,), 530, device=cuda), torch.full((B,), 730, device=cuda))
    np.testing.assert_allclose(out.cpu().numpy(), fx["boxes2d"], rtol=1e-5, atol=1e-3)


def test_projection_matches_host_restatement(cuda):
    from ov3d_amd.image_util import project_boxes_2d
    g = torch.Generator().manual_seed(3)
    L, B, Q = 8, 4, 128
    n = L * B
    center = torch.rand((n, Q, 3), generator=g) * torch.tensor([6.0, 6.0, 3.0]) - torch.tensor([3.0, -0.5, 1.0])
    center[:, :8, 1] = -torch.rand(8, generator=g)          # behind the camera
    size = torch.rand((n, Q, 3), generator=g) * 2 + 0.05
    heading = (torch.rand((n, Q), generator=g) - 0.5) * 2 * np.pi
    center[0, 9, 0] = float("nan")
    size[1, 10, 2] = float("nan")
    rt = torch.eye(3) + 0.05 * torch.randn((B, 3, 3), generator=g)
    kk = torch.tensor([[529.5, 0, 365.0], [0, 529.5, 265.0], [0, 0, 1]]).repeat(B, 1, 1)
    ih = torch.tensor([530, 427, 530, 441])
    iw = torch.tensor([730, 561, 681, 591])
    rep = (lambda t: t.repeat((L,) + (1,) * (t.dim() - 1)))
    host = project_boxes_2d(center, size, heading, rep(rt), rep(kk), rep(ih), rep(iw))
    dev = project_boxes_2d(center.to(cuda), size.to(cuda), heading.to(cuda), rep(rt).to(cuda),
                           rep(kk).to(cuda), rep(ih).to(cuda), rep(iw).to(cuda)).cpu()
    nan_h, nan_d = torch.isnan(host), torch.isnan(dev)
    assert torch.equal(nan_h, nan_d) and nan_h.any()
    ok = ~nan_h
    # same float32 formula; cos / sin (ocml vs SLEEF) and the matmul association differ by ulps
    torch.testing.assert_close(dev[ok], host[ok], rtol=2e-5, atol=2e-3)
    # clamps: every edge is hit somewhere and nothing escapes [0, (w, h, w, h)]
    lim = torch.stack([rep(iw), rep(ih), rep(iw), rep(ih)], 1).float()[:, None, :]
    d = torch.where(ok, dev, torch.zeros_like(dev))
    assert (d >= 0).all() and (d <= lim).all()
    assert (d == 0).any() and (d == lim).any()


def test_projection_matches_cpu_twin(cuda):
    """ov3d_project_box2d against its CPU twin (oracle ov3d_project_box2d_cpu, pinned to the
    reference golden in tests/test_oracle_twins.py): the same float32 expressions in the same
    order, so equal but for cosf / sinf (ocml vs libm, ~1 ulp) and what that moves"""
    from ov3d_amd.image_util import project_boxes_2d
    from oracle import oracle
    g = torch.Generator().manual_seed(5)
    L, B, Q = 8, 4, 128
    n = L * B
    center = torch.rand((n, Q, 3), generator=g) * torch.tensor([6.0, 6.0, 3.0]) - torch.tensor([3.0, -0.5, 1.0])
    size = torch.rand((n, Q, 3), generator=g) * 2 + 0.05
    heading = (torch.rand((n, Q), generator=g) - 0.5) * 2 * np.pi
    rt = torch.eye(3) + 0.05 * torch.randn((B, 3, 3), generator=g)
    kk = torch.tensor([[529.5, 0, 365.0], [0, 529.5, 265.0], [0, 0, 1]]).repeat(B, 1, 1)
    ih, iw = torch.tensor([530, 427, 530, 441]), torch.tensor([730, 561, 681, 591])
    rep = (lambda t: t.repeat((L,) + (1,) * (t.dim() - 1)))
    dev = project_boxes_2d(center.to(cuda), size.to(cuda), heading.to(cuda), rep(rt).to(cuda),
                           rep(kk).to(cuda), rep(ih).to(cuda), rep(iw).to(cuda)).cpu().numpy()
    twin = oracle.project_box2d(center.numpy(), size.numpy(), heading.numpy(), Q, B, rt.numpy(),
                                kk.numpy(), ih.numpy(), iw.numpy()).reshape(dev.shape)
    np.testing.assert_allclose(dev, twin, rtol=2e-5, atol=2e-3)
    assert (dev == twin).mean() > 0.5   # most boxes: the identical bits

