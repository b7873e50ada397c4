"""RegionCLIP ROI-feature path on the GPU.

* ov3d_roi_align_fwd vs the C oracle: bit-exact in fp32, and in bf16 (the kernel
  accumulates bf16 inputs in fp32 in the oracle's order and rounds once).
* ov3d_clip_preprocess vs the torch formulation of preprocess_image (bit-exact fp32).
* RegionCLIP.inference / region_features vs the plain fp32 restatement in
  tests/regionclip_ref.py (unfolded BN, NCHW, per-image, oracle ROIAlign, MHA pool):
  fp32 within 2e-3 relative; bf16 (the training-step dtype) mean cosine >= 0.995.
  RegionCLIP itself is not available offline: PARITY UNPINNED against upstream.
* The criterion's batched alignment (one backbone pass, all layers) equals the
  reference per-layer loop through clip.inference.
"""
import numpy as np
import pytest
import torch

from helpers import ov3d  # noqa: F401  (registers ov3d_amd)
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _boxes(rng, n, H, W):
    x1 = rng.uniform(-20, W, n)
    y1 = rng.uniform(-20, H, n)
    b = np.stack([x1, y1, x1 + rng.uniform(0, W / 2, n), y1 + rng.uniform(0, H / 2, n)], 1)
    b = np.minimum(np.maximum(b, 0), [W, H, W, H])          # criterion.py:389-391 clamp
    b[0] = [0, 0, 0, 0]                                      # empty box -> zeros
    b[1] = [0, 0, W, H]                                      # whole image
    b[2] = [W - 3, H - 3, W, H]                              # bottom-right edge
    b[3] = [10.3, 12.7, 10.3, 40.1]                          # zero width
    return b.astype(np.float32)


@pytest.mark.parametrize("dtype,C,H,W,R,per,nimg", [(torch.float32, 64, 33, 45, 40, 10, 4),
                                                    (torch.bfloat16, 128, 33, 45, 48, 12, 2),
                                                    (torch.float32, 8, 7, 5, 16, 4, 4),
                                                    # LDS-window form: 16-ROI groups, a partial one
                                                    (torch.bfloat16, 64, 33, 45, 80, 40, 2),
                                                    # windows past 1536 pixels: global reads
                                                    (torch.bfloat16, 32, 40, 45, 20, 20, 1)])
@pytest.mark.parametrize("lds,affine", [("0", "1"), ("0", "0"), ("1", "1")])
def test_roi_align_bit_exact(cuda, monkeypatch, dtype, C, H, W, R, per, nimg, lds, affine):
    from ov3d_amd import _native
    monkeypatch.setenv("OV3D_ROI_LDS", lds)         # the LDS-window form of the fused pool (bf16)
    monkeypatch.setenv("OV3D_ROI_AFFINE", affine)   # image-affine XCD order of the global form
    rng = np.random.default_rng(C + R)
    feat = torch.from_numpy(rng.standard_normal((nimg, H, W, C)).astype(np.float32)).to(dtype)
    boxes = _boxes(rng, R, H * 16, W * 16)
    P = 18
    out = torch.empty((R, P, P, C), dtype=dtype, device=cuda)
    fg = feat.to(cuda)
    _native.call("ov3d_roi_align_fwd", fg, int(dtype == torch.bfloat16), nimg, H, W, C,
                 torch.from_numpy(boxes).to(cuda), R, per, nimg, 1.0 / 16, P, 0, 1, out, like=fg)
    ref = O.roi_align(feat.float().numpy(), boxes, per, nimg, 1.0 / 16, P)
    if dtype == torch.bfloat16:
        ref = torch.from_numpy(ref).to(torch.bfloat16).float().numpy()
    np.testing.assert_array_equal(out.float().cpu().numpy(), ref)
    assert (out[0] == 0).all()
    # the fused form: the same bins, plus their 2x2 pool bit-equal to torch's avg_pool2d
    out2 = torch.empty_like(out)
    pooled = torch.empty((R, P // 2, P // 2, C), dtype=dtype, device=cuda)
    _native.call("ov3d_roi_align_pool2_fwd", fg, int(dtype == torch.bfloat16), nimg, H, W, C,
                 torch.from_numpy(boxes).to(cuda), R, per, nimg, 1.0 / 16, P, 0, 1, out2, pooled,
                 like=fg)
    assert torch.equal(out2, out)
    import torch.nn.functional as F
    assert torch.equal(pooled, F.avg_pool2d(out.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1))


def test_clip_preprocess_bit_exact(cuda):
    from ov3d_amd import regionclip as rc
    m = rc.RegionCLIP(layers=(1, 1, 1, 1), width=16, compute_dtype=torch.float32).to(cuda)
    rng = np.random.default_rng(0)
    hs, ws = [30, 41, 17], [50, 33, 64]
    cap = 64 * 64 * 3
    img = np.zeros((3, cap), np.float32)
    for i in range(3):
        img[i, : hs[i] * ws[i] * 3] = rng.uniform(0, 255, hs[i] * ws[i] * 3)
    x = m._preprocess_1d(torch.from_numpy(img).to(cuda), hs, ws, max(hs), max(ws))
    from regionclip_ref import preprocess
    ims = [torch.from_numpy(img[i, : hs[i] * ws[i] * 3]).view(hs[i], ws[i], 3).permute(2, 0, 1).to(cuda)
           for i in range(3)]
    ref = preprocess(m.pixel_mean, m.pixel_std, ims).permute(0, 2, 3, 1)
    torch.testing.assert_close(x, ref, rtol=0, atol=0)


def _inputs(cuda, B, Q, H, W, seed):
    from ov3d_amd.image_util import clip_batch
    rng = np.random.default_rng(seed)
    img = torch.from_numpy(rng.uniform(0, 255, (B, H * W * 3)).astype(np.float32)).to(cuda)
    boxes = torch.from_numpy(np.stack([_boxes(rng, Q, H, W) for _ in range(B)])).to(cuda)
    h = torch.full((B,), H, dtype=torch.int64, device=cuda)
    w = torch.full((B,), W, dtype=torch.int64, device=cuda)
    return img, h, w, boxes, clip_batch(img, h, w, boxes)


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_inference_fp32_matches_reference_small(cuda):
    """Reduced-width network, ragged image sizes in one batch, empty / edge boxes."""
    from ov3d_amd import regionclip as rc
    import regionclip_ref
    from ov3d_amd.image_util import Boxes, Instances
    torch.manual_seed(0)
    m = rc.RegionCLIP(layers=(1, 2, 2, 2), width=32, heads=16, compute_dtype=torch.float32)
    rc.init_synthetic_(m.backbone, seed=3)
    m = m.to(cuda)
    rng = np.random.default_rng(1)
    inputs = []
    for (H, W, Q) in [(100, 140, 7), (131, 97, 5), (64, 64, 0)]:
        im = torch.from_numpy(rng.uniform(0, 255, (3, H, W)).astype(np.float32)).to(cuda)
        bx = torch.from_numpy(_boxes(rng, max(Q, 4), H, W)[:Q]).to(cuda)
        inputs.append({"image": im, "instances": Instances((H, W), gt_boxes=Boxes(bx))})
    got = m.inference(inputs, do_postprocess=False)
    ref = regionclip_ref.inference(m, inputs)
    assert got.shape == (12, m.backbone.attnpool.c_proj.out_features)
    assert _rel(got, ref) < 2e-3, _rel(got, ref)


def test_region_features_rn50x4_fp32_and_bf16(cuda):
    """Full RN50x4 (README.md:29-36 config) on SUN-size images: the batched path over L
    layers equals the reference per-layer clip.inference; bf16 stays close to fp32."""
    from ov3d_amd import regionclip as rc
    import regionclip_ref
    m32, _ = rc.build_regionclip(compute_dtype=torch.float32)
    m32 = m32.to(cuda)
    L, B, Q, H, W = 2, 2, 6, 530, 730
    img, h, w, boxes, _ = _inputs(cuda, B, L * Q, H, W, seed=5)
    boxes = boxes.view(B, L, Q, 4).transpose(0, 1).contiguous()          # (L,B,Q,4)
    got = m32.region_features(img, h, w, boxes)                          # (L,B,Q,640)
    from ov3d_amd.image_util import clip_batch
    for l in range(L):
        ref = regionclip_ref.inference(m32, clip_batch(img, h, w, boxes[l]))
        assert _rel(got[l].reshape(B * Q, -1), ref) < 2e-3
        per_layer = m32.inference(clip_batch(img, h, w, boxes[l]))
        assert _rel(per_layer, ref) < 2e-3
    m16, _ = rc.build_regionclip(compute_dtype=torch.bfloat16)
    m16 = m16.to(cuda)
    g16 = m16.region_features(img, h, w, boxes)
    cos = torch.nn.functional.cosine_similarity(g16.float(), got, dim=-1)
    # bf16 activations through 26 bottleneck blocks + res5 (fp32 accumulation everywhere)
    assert cos.min().item() > 0.985 and cos.mean().item() > 0.995, (cos.min().item(), cos.mean().item())


def test_criterion_alignment_batched_equals_per_layer(cuda):
    import argparse
    from ov3d_amd import regionclip as rc, synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import default_args
    ov3d_mod = ov3d
    cfg = SunrgbdDatasetConfig()
    args = default_args(nqueries=16, dec_nlayers=3, enc_nlayers=1, preenc_npoints=256,
                        loss_2dalignment_weight=2e-4)
    torch.manual_seed(0)
    model, _ = ov3d_mod.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).eval()
    crit = ov3d_mod.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(2, seed=9, num_points=2048, use_image=True, device=cuda)
    clip, _ = rc.build_regionclip(compute_dtype=torch.float32)
    clip = clip.to(cuda)

    class PerLayer:  # the reference API only: forces the per-layer clip.inference loop
        def inference(self, *a, **k):
            return clip.inference(*a, **k)

    with torch.no_grad():
        out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
        _, ld_b = crit(out, dict(batch), clip=clip)
        _, ld_r = crit(out, dict(batch), clip=PerLayer())
    keys = [k for k in ld_r if k.startswith("loss_2dalignment")]
    assert len(keys) == 3
    for k in keys:
        assert abs(ld_b[k].item() - ld_r[k].item()) <= 1e-4 * abs(ld_r[k].item()) + 1e-6, k


@pytest.mark.parametrize("dtype,N,H,W,C,stride", [(torch.bfloat16, 3, 9, 9, 64, 1),
                                                  (torch.bfloat16, 2, 17, 23, 40, 2),
                                                  (torch.float32, 2, 11, 7, 3, 2),
                                                  (torch.float32, 1, 5, 6, 12, 1)])
def test_im2col3x3_exact(cuda, dtype, N, H, W, C, stride):
    import torch.nn.functional as F
    from ov3d_amd import _native
    x = torch.randn(N, H, W, C, device=cuda).to(dtype)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    kpad = (9 * C + 15) // 16 * 16
    out = torch.full((N * Ho * Wo, kpad), 7.0, dtype=dtype, device=cuda)
    _native.call("ov3d_im2col3x3", x, x.element_size(), N, H, W, C, stride, kpad, out, like=x)
    cols = F.unfold(x.permute(0, 3, 1, 2).float(), 3, padding=1, stride=stride)   # (N, C*9, L)
    ref = cols.view(N, C, 9, Ho * Wo).permute(0, 3, 2, 1).reshape(N * Ho * Wo, 9 * C)
    assert torch.equal(out[:, : 9 * C].float(), ref)
    assert (out[:, 9 * C:] == 0).all()


@pytest.mark.parametrize("dtype,rows,cols,relu", [(torch.bfloat16, 4 * 81, 2560, 1),
                                                  (torch.bfloat16, 37, 64, 0),
                                                  (torch.float32, 50, 36, 1)])
def test_bias_residual_act_matches_fp32(cuda, dtype, rows, cols, relu):
    """Bottleneck close after the conv3 GEMM: act((y + bias) + residual) in fp32, one rounding."""
    from ov3d_amd import _native
    g = torch.Generator(device=cuda).manual_seed(5)
    y = torch.randn(rows, cols, device=cuda, generator=g).to(dtype)
    b = torch.randn(cols, device=cuda, generator=g).to(dtype)
    r = torch.randn(rows, cols, device=cuda, generator=g).to(dtype)
    ref = (y.float() + b.float()) + r.float()
    if relu:
        ref = ref.relu()
    out = y.clone()
    _native.call("ov3d_bias_residual_act", out, out.element_size(), rows, cols, b, r, relu, like=out)
    assert torch.equal(out, ref.to(dtype))


@pytest.mark.parametrize("dtype,N,H,W,C", [(torch.bfloat16, 5, 18, 18, 1280),
                                           (torch.bfloat16, 2, 17, 23, 80),
                                           (torch.float32, 3, 8, 6, 12)])
def test_avgpool2_nhwc_bit_exact(cuda, dtype, N, H, W, C):
    """The HIP 2x2 pool equals torch's avg_pool2d bit for bit (odd sizes floor)."""
    import torch.nn.functional as F
    from ov3d_amd import _native
    x = torch.randn(N, H, W, C, device=cuda).to(dtype)
    out = torch.empty((N, H // 2, W // 2, C), dtype=dtype, device=cuda)
    _native.call("ov3d_avgpool2_nhwc", x, x.element_size(), N, H, W, C, out, like=x)
    ref = F.avg_pool2d(x.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype,R,ntok,C", [(torch.bfloat16, 37, 81, 2560), (torch.float32, 5, 9, 64)])
def test_attnpool_tokens_matches_torch(cuda, dtype, R, ntok, C):
    """Token rows of the attention pool: [mean; x] + pos; the spatial rows bit-equal to torch's
    x + pos, the mean row within one rounding of torch's reduction (summation order)."""
    from ov3d_amd import _native
    x = torch.randn(R, ntok, C, device=cuda).to(dtype)
    pos = torch.randn(ntok + 1, C, device=cuda).to(dtype)
    t = torch.empty((R, ntok + 1, C), dtype=dtype, device=cuda)
    _native.call("ov3d_attnpool_tokens", x, x.element_size(), R, ntok, C, pos, t, like=x)
    ref = torch.cat([x.float().mean(1, keepdim=True).to(dtype), x], 1) + pos
    assert torch.equal(t[:, 1:], ref[:, 1:])
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert torch.allclose(t[:, 0].float(), ref[:, 0].float(), atol=tol, rtol=tol)


@pytest.mark.parametrize("R,ntok,C,H", [(37, 81, 2560, 40), (5, 9, 128, 13), (3, 94, 64, 48)])
def test_attnpool_fused_matches_token_path(cuda, R, ntok, C, H):
    """ov3d_attnpool_mean is row 0 of ov3d_attnpool_tokens bit for bit; ov3d_attnpool_fused
    (token rows on chip, scores, softmax, p.t in one launch) equals the token rows + bmm +
    softmax + bmm composition of regionclip._pool_tokens up to the bmm's summation order
    (scores rounded to bf16 on both sides), and stays within bf16 rounding of fp32."""
    from ov3d_amd import _native
    g = torch.Generator(device=cuda).manual_seed(R + ntok)
    x = torch.randn(R, ntok, C, device=cuda, generator=g).to(torch.bfloat16)
    pos = (0.5 * torch.randn(ntok + 1, C, device=cuda, generator=g)).to(torch.bfloat16)
    a = (torch.randn(H, R, C, device=cuda, generator=g) / C ** 0.5).to(torch.bfloat16)
    t = torch.empty((R, ntok + 1, C), dtype=torch.bfloat16, device=cuda)
    _native.call("ov3d_attnpool_tokens", x, 2, R, ntok, C, pos, t, like=x)
    t0 = torch.empty((R, C), dtype=torch.bfloat16, device=cuda)
    _native.call("ov3d_attnpool_mean", x, R, ntok, C, pos, t0, like=x)
    assert torch.equal(t0, t[:, 0])
    y = torch.empty((H, R, C), dtype=torch.bfloat16, device=cuda)
    _native.call("ov3d_attnpool_fused", x, t0, pos, a, a.stride(0), a.stride(1), R, ntok, C, H, y,
                 like=x)
    s = torch.bmm(a.transpose(0, 1), t.transpose(1, 2))                  # (R, H, T) bf16
    p = torch.softmax(s.float(), dim=-1).to(torch.bfloat16)
    ref = torch.bmm(p, t).transpose(0, 1)                                # (H, R, C)
    err = (y.float() - ref.float()).abs()
    assert err.max().item() < 3e-2 * ref.float().abs().max().item(), err.max().item()
    assert _rel(y.float(), ref.float()) < 4e-3, _rel(y.float(), ref.float())
    s32 = torch.bmm(a.transpose(0, 1).float(), t.float().transpose(1, 2))
    ref32 = torch.bmm(torch.softmax(s32, dim=-1), t.float()).transpose(0, 1)
    assert _rel(y.float(), ref32) < 1e-2, _rel(y.float(), ref32)
    # a strided (R, H, C) view of the same values gives the same result
    a2 = a.transpose(0, 1).contiguous().transpose(0, 1)
    y2 = torch.empty_like(y)
    _native.call("ov3d_attnpool_fused", x, t0, pos, a2, a2.stride(0), a2.stride(1), R, ntok, C, H,
                 y2, like=x)
    assert torch.equal(y2, y)


def test_attnpool_fused_module_equals_token_path(cuda):
    """RegionCLIP._attnpool through the fused launch vs through the token rows (RN50x4 pool
    shapes: 81 tokens, 2560 channels, 40 heads)."""
    from ov3d_amd import regionclip as rc
    m, _ = rc.build_regionclip(compute_dtype=torch.bfloat16)
    m = m.to(cuda)
    g = torch.Generator(device=cuda).manual_seed(4)
    x = torch.randn(24, 9, 9, 2560, device=cuda, generator=g).relu().to(torch.bfloat16)
    assert m._fused_pool_ok(x)
    got = m._attnpool(x)
    ref = m._pool_tokens(m._tokens(x))
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert cos.min().item() > 0.9999, cos.min().item()
    assert _rel(got, ref) < 1e-2
