"""HIP set-criterion losses (csrc/setloss.hip) against the torch expression of the same
terms (criterion.SetCriterion._losses_torch, fp32) on the same model outputs, matches and
targets: every loss_dict entry, the total, and the gradients of every head output the
losses read.  Tolerance 1e-5 relative (fp64 vs fp32 summation order only).  The reference
fixtures (test_model_gpu.py) pin both paths against the reference criterion."""
import numpy as np
import pytest
import torch

from fake_clip import FakeRegionCLIP
from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu

KEYS = ("sem_cls_logits", "angle_logits", "angle_residual_normalized", "center_normalized",
        "size_normalized", "box_corners", "visual_embeds")


def _outputs(cuda, B, Q, L, T, NB, seed):
    """stacked (L, B, Q, ...) head outputs with grads, plus consistent derived keys"""
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from ov3d_amd.model_3detr import BoxProcessor
    g = torch.Generator(device="cpu").manual_seed(seed)

    def r(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(cuda).requires_grad_()

    st = {"sem_cls_logits": r(L, B, Q, T, scale=3.0),
          "angle_logits": r(L, B, Q, NB, scale=2.0),
          "angle_residual_normalized": r(L, B, Q, NB),
          "center_normalized": torch.rand(L, B, Q, 3, generator=g).to(cuda).requires_grad_(),
          "size_normalized": (0.05 + 0.3 * torch.rand(L, B, Q, 3, generator=g)).to(cuda).requires_grad_(),
          "visual_embeds": r(L, B, Q, 640)}
    bp = BoxProcessor(SunrgbdDatasetConfig())
    with torch.no_grad():
        prob = torch.softmax(st["sem_cls_logits"], -1)
        st["sem_cls_prob"], st["objectness_prob"] = prob[..., :-1], 1 - prob[..., -1]
        cu = st["center_normalized"] * 6 - 3
        sz = st["size_normalized"] * 4
        ang = (torch.rand(L, B, Q, generator=g) * 6 - 3).to(cuda)
        st["center_unnormalized"], st["size_unnormalized"], st["angle_continuous"] = cu, sz, ang
        st["box_corners"] = bp.box_parametrization_to_corners(
            cu.reshape(L * B, Q, 3), sz.reshape(L * B, Q, 3), ang.reshape(L * B, Q)).view(L, B, Q, 8, 3)
    st["box_corners"].requires_grad_()
    return st


def _criterion(cuda, giou_w, align_w):
    import argparse
    from ov3d_amd.criterion import build_criterion
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    a = argparse.Namespace(matcher_giou_cost=3.0, matcher_cls_cost=1.0, matcher_center_cost=5.0,
                           matcher_objectness_cost=5.0, loss_giou_weight=giou_w,
                           loss_sem_cls_weight=1.0, loss_no_object_weight=0.1,
                           loss_angle_cls_weight=0.1, loss_angle_reg_weight=0.5,
                           loss_center_weight=5.0, loss_size_weight=1.0,
                           loss_2dalignment_weight=align_w)
    return build_criterion(a, SunrgbdDatasetConfig()).to(cuda)


def _run(crit, st, batch, fused, stacked, clip):
    crit.fused_losses = fused
    leaves = {k: v.detach().clone().requires_grad_() for k, v in st.items() if k in KEYS}
    full = dict(st)
    full.update(leaves)
    L = st["sem_cls_logits"].shape[0]
    if stacked:
        outs = {"_layers_stacked": full}
    else:
        layers = [{k: v[l] for k, v in full.items()} for l in range(L)]
        outs = {"outputs": layers[-1], "aux_outputs": layers[:-1]}
    loss, ld = crit(outs, dict(batch), clip=clip)
    loss.backward()
    return loss.detach(), {k: v.detach() for k, v in ld.items()}, \
        {k: (v.grad if v.grad is not None else torch.zeros_like(v)) for k, v in leaves.items()}


@pytest.mark.parametrize("giou_w,align_w,stacked", [(0.0, 0.0, True), (1.0, 0.0, True),
                                                     (0.0, 2e-4, False), (1.0, 2e-4, True)])
def test_fused_losses_equal_torch(cuda, giou_w, align_w, stacked):
    from ov3d_amd import synthetic
    B, Q, L, T, NB = 8, 128, 8, 21, 12
    st = _outputs(cuda, B, Q, L, T, NB, seed=3)
    batch = synthetic.make_batch(B, seed=5, num_points=2048, device=cuda, use_image=align_w > 0)
    if giou_w > 0:
        batch["gt_box_angles"].zero_()   # differentiable GIoU: axis-aligned GT (ScanNet-style)
    crit = _criterion(cuda, giou_w, align_w)
    clip = FakeRegionCLIP() if align_w > 0 else None
    lt, dt, gt = _run(crit, st, batch, False, stacked, clip)
    lf, df, gf = _run(crit, st, batch, True, stacked, clip)
    assert set(dt) == set(df)
    assert abs(lf.item() - lt.item()) <= 1e-5 * abs(lt.item()), (lf.item(), lt.item())
    for k in dt:
        a, b = df[k].item(), dt[k].item()
        assert abs(a - b) <= 1e-5 * max(abs(b), 1e-6), (k, a, b)
    for k in gt:
        a, b = gf[k].cpu().numpy(), gt[k].cpu().numpy()
        den = max(np.abs(b).max(), 1e-12)
        assert np.abs(a - b).max() / den < 1e-5, k


def test_fused_losses_no_gt_boxes(cuda):
    """a replica without GT boxes: every proposal unmatched, box terms exactly zero"""
    from ov3d_amd import synthetic
    B, Q, L, T, NB = 2, 64, 3, 21, 12
    st = _outputs(cuda, B, Q, L, T, NB, seed=4)
    batch = synthetic.make_batch(B, seed=6, num_points=1024, device=cuda)
    batch["gt_box_present"].zero_()
    crit = _criterion(cuda, 0.0, 0.0)
    lt, dt, gt = _run(crit, st, batch, False, True, None)
    lf, df, gf = _run(crit, st, batch, True, True, None)
    for k in ("loss_angle_cls", "loss_angle_reg", "loss_center", "loss_size"):
        assert df[k].item() == 0.0 and dt[k].item() == 0.0, k
    assert abs(lf.item() - lt.item()) <= 1e-5 * abs(lt.item())
    for k in gt:
        assert torch.allclose(gf[k], gt[k], rtol=1e-5, atol=1e-9), k


def test_fused_losses_inside_graph_replay(cuda):
    """the ticket counter resets itself: repeated launches (graph replays) stay equal"""
    from ov3d_amd import synthetic
    B, Q, L, T, NB = 4, 128, 8, 21, 12
    st = _outputs(cuda, B, Q, L, T, NB, seed=7)
    batch = synthetic.make_batch(B, seed=8, num_points=2048, device=cuda)
    crit = _criterion(cuda, 0.0, 0.0)
    vals = [_run(crit, st, batch, True, True, None)[0].item() for _ in range(5)]
    assert len(set(vals)) == 1, vals


def test_matcher_cost_and_counts_match_torch(cuda):
    """ov3d_matcher_cost / ov3d_targets_prep against Matcher.cost + the torch counts"""
    from ov3d_amd import setloss, synthetic
    from ov3d_amd.box_util import generalized_box3d_iou
    B, Q, L, T, NB = 8, 128, 8, 21, 12
    st = _outputs(cuda, B, Q, L, T, NB, seed=9)
    batch = synthetic.make_batch(B, seed=10, num_points=2048, device=cuda)
    crit = _criterion(cuda, 0.0, 0.0)
    nact, nrep, nb, rot, total = setloss.target_counts(batch["gt_box_present"], batch, L)
    ref_n = batch["gt_box_present"].sum(1).long()
    assert torch.equal(nact, ref_n) and torch.equal(nrep, ref_n.repeat(L).int())
    assert int(total) == int(ref_n.sum()) and float(nb) == max(float(ref_n.sum()), 1.0)
    assert int(rot) == int((batch["gt_box_angles"] > 0).any())

    def cat(k):
        t = st[k]
        return t.reshape(L * B, *t.shape[2:])

    gious = generalized_box3d_iou(cat("box_corners").detach(), batch["gt_box_corners"].repeat(L, 1, 1, 1),
                                  nrep, rotated_boxes=rot)
    m = crit.matcher
    cost = setloss.matcher_cost(cat("sem_cls_prob"), cat("objectness_prob"),
                                cat("center_normalized").detach(), gious, batch, B,
                                (m.cost_class, m.cost_objectness, m.cost_center, m.cost_giou))
    cn = cat("center_normalized").detach()
    gc = batch["gt_box_centers_normalized"].repeat(L, 1, 1)
    dist = (cn[:, :, None, :] - gc[:, None, :, :]).abs().sum(-1)
    ref = m.cost(cat("sem_cls_prob"), cat("objectness_prob"), dist, gious,
                 batch["gt_box_sem_cls_label"].repeat(L, 1))
    assert torch.allclose(cost, ref, rtol=1e-6, atol=1e-6), (cost - ref).abs().max()


@pytest.mark.parametrize("fused", [True, False])
def test_invalid_matching_cost_poisons_total(cuda, fused):
    """A NaN matcher cost (scipy's linear_sum_assignment raises ValueError there,
    criterion.py:79) must not train on silently: the device matcher reports status -1 and
    the criterion's total becomes NaN, so engine.py's non-finite-loss exit fires.  The
    objectness probability enters the matching cost only, so the loss terms stay finite."""
    from ov3d_amd import synthetic
    B, Q, L, T, NB = 2, 64, 3, 21, 12
    st = _outputs(cuda, B, Q, L, T, NB, seed=11)
    batch = synthetic.make_batch(B, seed=12, num_points=1024, device=cuda)
    crit = _criterion(cuda, 0.0, 0.0)
    ok, _, _ = _run(crit, st, batch, fused, True, None)
    assert torch.isfinite(ok)
    st["objectness_prob"] = st["objectness_prob"].clone()
    st["objectness_prob"][1, 0, 5] = float("nan")
    bad, ld, _ = _run(crit, st, batch, fused, True, None)
    assert torch.isnan(bad)
    assert all(torch.isfinite(v) for v in ld.values())


@pytest.mark.parametrize("giou_w,align_w", [(0.0, 0.0), (1.0, 2e-4)])
def test_split_loss_forward_equals_per_layer(cuda, monkeypatch, giou_w, align_w):
    """ov3d_set_loss_fwd_split (a workgroup per 256 proposals and layer, chunk sums added in
    chunk order) vs the per-layer launch: the same loss dict and total up to fp64 rounding
    of the sums (1e-6 relative), identical gradients (the backward reads the same raw rows
    up to that rounding)"""
    from ov3d_amd import setloss, synthetic
    B, Q, L, T, NB = 8, 128, 8, 21, 12
    st = _outputs(cuda, B, Q, L, T, NB, seed=4)
    batch = synthetic.make_batch(B, seed=6, num_points=2048, device=cuda, use_image=align_w > 0)
    if giou_w > 0:
        batch["gt_box_angles"].zero_()
    crit = _criterion(cuda, giou_w, align_w)
    clip = FakeRegionCLIP() if align_w > 0 else None
    res = {}
    for split in (True, False):
        monkeypatch.setattr(setloss, "SPLIT_FWD", split)
        res[split] = _run(crit, st, batch, True, True, clip)
    (ls, ds, gs), (lp, dp, gp) = res[True], res[False]
    assert abs(ls.item() - lp.item()) <= 1e-6 * abs(lp.item())
    for k in dp:
        assert abs(ds[k].item() - dp[k].item()) <= 1e-6 * max(abs(dp[k].item()), 1e-6), k
    for k in gp:
        a, b = gs[k].cpu().numpy(), gp[k].cpu().numpy()
        assert np.abs(a - b).max() <= 1e-6 * max(np.abs(b).max(), 1e-12), k
