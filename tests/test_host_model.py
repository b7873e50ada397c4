"""Host logic of the product (transformer, heads, box processing, criterion,
matcher, losses) against the REFERENCE fixtures, on CPU.  The index kernels
are swapped for the C oracle explicitly (oracle/torch_shim.py) — the GPU suite
runs the same comparison through the HIP kernels."""
import numpy as np
import pytest
import torch

from fake_clip import FakeRegionCLIP
from helpers import (batch_from_fixture, build_model_from_fixture, fixture, fixture_prefix, ov3d,
                     grad_err, grad_tol, pin_matcher, rel_err)

CASES = [("model_sun.npz", "sunrgbd"), ("model_scannet.npz", "scannet")]


@pytest.fixture()
def shim():
    from oracle import torch_shim
    saved = torch_shim.install(ov3d)
    yield
    torch_shim.uninstall(saved)


@pytest.mark.parametrize("name,ds", CASES)
def test_forward_and_losses_match_reference(shim, name, ds):
    from ov3d_amd.criterion import build_criterion
    torch.set_num_threads(8)
    fx = fixture(name)
    model, cfg, args = build_model_from_fixture(fx, "cpu", ds)
    model.train()
    batch = batch_from_fixture(fx, "cpu")
    out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
    layers = [out["outputs"]] + out["aux_outputs"]
    assert len(layers) == args.dec_nlayers
    for li, lay in enumerate(layers):
        assert len(lay) == 13
        for k, ref in fixture_prefix(fx, f"out/{li}/").items():
            assert rel_err(lay[k].detach().numpy(), ref) < 1e-4, (li, k)
    crit = build_criterion(args, cfg)
    clip = FakeRegionCLIP()
    seen = {}
    solve = crit.matcher.forward

    def spy(cost, nact):
        seen.update(solve(cost, nact))
        return seen
    crit.matcher.forward = spy
    loss, ld = crit(out, dict(batch), clip=clip)
    # matching: same assignment as the reference except for near-tie flips
    L, B, Q = fx["match_inds"].shape
    same = (seen["per_prop_gt_inds"].view(L, B, Q).numpy() == fx["match_inds"]) | (fx["match_mask"] == 0)
    same &= seen["proposal_matched_mask"].view(L, B, Q).numpy() == fx["match_mask"]
    assert same.mean() > 0.97
    ref_ld = fixture_prefix(fx, "ld/")
    assert list(ld) == list(ref_ld) or set(ld) == set(ref_ld)
    assert len(ld) == 56
    for k, v in ref_ld.items():
        assert abs(ld[k].item() - float(v)) <= 1e-4 * max(abs(float(v)), 1e-3), k
    assert abs(loss.item() - float(fx["loss"])) <= 1e-4 * abs(float(fx["loss"]))
    if args.loss_2dalignment_weight > 0:
        assert clip.calls == args.dec_nlayers
    else:
        assert clip.calls == 0  # gated: output-identical (criterion.py:404-413)


@pytest.mark.parametrize("name,ds", CASES)
def test_gradients_match_reference(shim, name, ds):
    from ov3d_amd.criterion import build_criterion
    torch.set_num_threads(8)
    fx = fixture(name)
    model, cfg, args = build_model_from_fixture(fx, "cpu", ds)
    model.train()
    batch = batch_from_fixture(fx, "cpu")
    out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
    crit = pin_matcher(build_criterion(args, cfg), fx, "cpu")
    loss, _ = crit(out, dict(batch), clip=FakeRegionCLIP())
    loss.backward()
    named = dict(model.named_parameters())
    grads = fixture_prefix(fx, "grad/")
    assert len(grads) >= 10
    for k, g in grads.items():
        assert grad_err(named[k].grad.numpy(), g) < grad_tol(k), k


def test_geometry_matches_reference():
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from ov3d_amd.image_util import project_boxes_2d
    fx = fixture("geometry.npz")
    cfg = SunrgbdDatasetConfig()
    c, s, a = (torch.from_numpy(fx[k]) for k in ("center", "size", "angle"))
    corners = cfg.box_parametrization_to_corners(c, s, a)
    np.testing.assert_allclose(corners.numpy(), fx["corners"], atol=2e-6)
    B = c.shape[0]
    boxes = project_boxes_2d(torch.from_numpy(fx["center_img"]), s, a,
                             torch.from_numpy(fx["Rtilt"]).repeat(B, 1, 1),
                             torch.from_numpy(fx["K"]).repeat(B, 1, 1),
                             torch.full((B,), 530), torch.full((B,), 730))
    np.testing.assert_allclose(boxes.numpy(), fx["boxes2d"], rtol=1e-5, atol=1e-3)


def test_state_dict_keys_follow_reference():
    fx = fixture("model_sun.npz")
    keys = set(fixture_prefix(fx, "sd/"))
    for k in ("pre_encoder.mlp_module.layer0.conv.weight", "pre_encoder.mlp_module.layer0.bn.bn.running_mean",
              "encoder.layers.0.self_attn.in_proj_weight", "encoder.layers.0.self_attn.out_proj.weight",
              "decoder.layers.7.multihead_attn.in_proj_bias", "pos_embedding.gauss_B",
              "mlp_heads.sem_cls_head.weight"):
        assert k in keys


def test_sa_module_matches_reference_semantics(shim):
    """The product SA module (channels-last GEMM rows + BN over rows + max over nsample)
    against the pointnet2 restatement (Conv2d/BatchNorm2d/max_pool2d) on identical inputs:
    forward and every parameter gradient."""
    import copy
    from oracle import pointnet2_ref as R
    fx = fixture("model_sun.npz")
    model, cfg, args = build_model_from_fixture(fx, "cpu", "sunrgbd")
    xyz = batch_from_fixture(fx, "cpu")["point_clouds"][..., :3].contiguous()
    mine = copy.deepcopy(model.pre_encoder).train()
    ref = R.PointnetSAModuleVotes(radius=0.2, nsample=64, npoint=args.preenc_npoints,
                                  mlp=[0, 64, 128, args.enc_dim], normalize_xyz=True).train()
    ref.load_state_dict(mine.state_dict())
    o1, o2 = mine(xyz)[1], ref(xyz)[1]
    assert rel_err(o1.detach().numpy(), o2.detach().numpy()) < 1e-4
    g = torch.randn_like(o1)
    (o1 * g).sum().backward()
    (o2 * g).sum().backward()
    for (n, p1), (_, p2) in zip(mine.named_parameters(), ref.named_parameters()):
        assert rel_err(p1.grad.numpy(), p2.grad.numpy()) < 1e-3, n
    sd1, sd2 = mine.state_dict(), ref.state_dict()
    for k in sd1:   # running statistics / num_batches_tracked updated identically
        assert torch.allclose(sd1[k].double(), sd2[k].double(), rtol=1e-4, atol=1e-6), k
