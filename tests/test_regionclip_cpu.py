"""RegionCLIP ROI path, host side (no GPU): the ROIAlign oracle against closed-form
cases, the module's reference layout, and the product's torch-level rewrites
(frozen BN folded into NHWC row GEMMs, reassociated first-query attention pool)
against the module's own reference formulation in fp32.  PARITY UNPINNED against
upstream RegionCLIP (not vendored, no weights)."""
import numpy as np
import torch

from helpers import ov3d  # noqa: F401
from oracle import oracle as O


def test_roi_align_oracle_linear_map_is_exact():
    """Bilinear sampling reproduces an affine map exactly away from the borders, so each
    bin equals the map at the mean of its sample points (= bin centre)."""
    H, W = 24, 32
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    f = np.stack([0.5 * xx + 0.25 * yy + 1, np.ones_like(xx)], -1)[None].astype(np.float32)
    box = np.array([[40.0, 24.0, 360.0, 280.0]], np.float32)      # /16 -> [2.5,1.5]..[22.5,17.5]
    P = 8
    out = O.roi_align(f, box, 1, 1, 1.0 / 16, P)
    x0, y0, x1, y1 = box[0] / 16 - 0.5
    cx = x0 + (np.arange(P) + 0.5) * (x1 - x0) / P
    cy = y0 + (np.arange(P) + 0.5) * (y1 - y0) / P
    expect = 0.5 * cx[None, :] + 0.25 * cy[:, None] + 1
    np.testing.assert_allclose(out[0, :, :, 0], expect, rtol=1e-6, atol=1e-5)
    np.testing.assert_array_equal(out[0, :, :, 1], 1.0)


def test_roi_align_oracle_edge_cases():
    f = np.random.default_rng(0).standard_normal((2, 5, 6, 3)).astype(np.float32)
    boxes = np.array([[0, 0, 0, 0], [30, 30, 30, 70], [-100, -100, -50, -50],
                      [0, 0, 96, 80]], np.float32)
    out = O.roi_align(f, boxes, per_image=2, nimages=2, spatial_scale=1.0 / 16, pooled=4)
    assert (out[0] == 0).all()                  # empty roi: grid 0 -> count 1 -> 0
    assert (out[1] == 0).all()                  # zero width: no samples
    # far outside the map: every sample < -1 -> 0
    assert (out[2] == 0).all()
    # roi 3 reads image (3 // 2) % 2 = 1
    assert np.isfinite(out[3]).all() and np.abs(out[3]).max() > 0
    out_img0 = O.roi_align(f[:1], boxes[3:], 1, 1, 1.0 / 16, 4)
    assert not np.array_equal(out[3], out_img0[0])


def _small(dtype=torch.float32):
    from ov3d_amd import regionclip as rc
    m = rc.RegionCLIP(layers=(1, 1, 2, 2), width=32, heads=16, compute_dtype=dtype)
    rc.init_synthetic_(m.backbone, seed=1)
    return m


def test_state_dict_layout_rn50x4():
    from ov3d_amd import regionclip as rc
    m = rc.RegionCLIP(compute_dtype=torch.float32)
    sd = m.state_dict()
    for k, shape in [("backbone.conv1.weight", (40, 3, 3, 3)),
                     ("backbone.layer1.0.downsample.0.weight", (320, 80, 1, 1)),
                     ("backbone.layer3.9.conv2.weight", (320, 320, 3, 3)),
                     ("backbone.layer4.0.downsample.1.running_var", (2560,)),
                     ("backbone.layer4.5.bn3.weight", (2560,)),
                     ("backbone.attnpool.positional_embedding", (82, 2560)),
                     ("backbone.attnpool.c_proj.weight", (640, 2560))]:
        assert tuple(sd[k].shape) == shape, k
    assert len(m.backbone.layer3) == 10 and m.backbone.attnpool.num_heads == 40


def test_folded_conv_matrices_equal_conv_plus_frozen_bn():
    """Every folded weight, applied as the product applies it (1x1: rows GEMM; 3x3: the
    (ky, kx, ci) im2col columns ov3d_im2col3x3 writes, restated with F.unfold here),
    equals conv -> FrozenBN of the reference module."""
    import torch.nn.functional as F
    from ov3d_amd.regionclip import Bottleneck, _Folded
    m = _small()
    fw = _Folded(m.backbone, torch.float32)
    blk = m.backbone.layer2[0]
    assert isinstance(blk, Bottleneck)
    for key, conv, bn in [("layer2.0.conv1", blk.conv1, blk.bn1), ("layer2.0.conv2", blk.conv2, blk.bn2),
                          ("layer2.0.down", blk.downsample[1], blk.downsample[2]),
                          ("conv1", m.backbone.conv1, m.backbone.bn1)]:
        w, b = fw.conv[key]
        stride = conv.stride[0]
        x = torch.randn(2, conv.in_channels, 11, 13)
        ref = bn(conv(x))
        if conv.kernel_size[0] == 1:
            got = x.permute(0, 2, 3, 1).reshape(-1, x.shape[1]) @ w.t() + b
        else:
            cols = F.unfold(x, 3, padding=1, stride=stride)                  # (N, C*9, L) (c, ky, kx)
            N, _, Lp = cols.shape
            C = x.shape[1]
            cols = cols.view(N, C, 9, Lp).permute(0, 3, 2, 1).reshape(N * Lp, 9 * C)
            cols = F.pad(cols, (0, w.shape[1] - 9 * C))
            got = cols @ w.t() + b
        got = got.view(ref.shape[0], ref.shape[2], ref.shape[3], -1).permute(0, 3, 1, 2)
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_reassociated_attnpool_equals_mha():
    m = _small()
    x = torch.randn(5, 1024, 9, 9) * 2             # 32 * width
    ref = m.backbone.attnpool(x)
    # token rows as ov3d_attnpool_tokens builds them on the GPU ([mean; x] + pos), then the
    # reassociated first-query pool
    rows = x.flatten(2).transpose(1, 2)                                  # (R, 81, C)
    t = torch.cat([rows.mean(1, keepdim=True), rows], 1) + m.folded().pos
    got = m._pool_tokens(t)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_build_model_regionclip_entry():
    import argparse
    m, extra = ov3d.build_model(argparse.Namespace(model_name="3detr"), None, model_name="regionclip")
    assert extra is None and not m.training
    assert m.backbone.attnpool.c_proj.out_features == 640
