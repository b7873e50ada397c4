"""The product model + criterion on the GPU (HIP sampling / grouping / GIoU
kernels) against the REFERENCE fixtures (fp32, within 1e-3 relative), and the
full BASELINE-size training step through size-independent properties."""
import numpy as np
import pytest
import torch

from fake_clip import FakeRegionCLIP
from helpers import (batch_from_fixture, build_model_from_fixture, fixture, fixture_prefix,
                     grad_err, grad_tol, pin_matcher, rel_err)

pytestmark = pytest.mark.gpu

CASES = [("model_sun.npz", "sunrgbd"), ("model_scannet.npz", "scannet")]


def _no_tf32():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False


@pytest.mark.parametrize("name,ds", CASES)
def test_model_matches_reference_on_gpu(cuda, name, ds):
    from ov3d_amd.criterion import build_criterion
    _no_tf32()
    fx = fixture(name)
    model, cfg, args = build_model_from_fixture(fx, cuda, ds)
    model.train()
    batch = batch_from_fixture(fx, cuda)
    out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")})
    layers = [out["outputs"]] + out["aux_outputs"]
    for li, lay in enumerate(layers):
        for k, ref in fixture_prefix(fx, f"out/{li}/").items():
            assert rel_err(lay[k].detach().cpu().numpy(), ref) < 1e-3, (li, k)
    crit = pin_matcher(build_criterion(args, cfg).to(cuda), fx, cuda)
    loss, ld = crit(out, dict(batch), clip=FakeRegionCLIP())
    for k, v in fixture_prefix(fx, "ld/").items():
        assert abs(ld[k].item() - float(v)) <= 1e-3 * max(abs(float(v)), 1e-3), k
    loss.backward()
    named = dict(model.named_parameters())
    for k, g in fixture_prefix(fx, "grad/").items():
        assert grad_err(named[k].grad.cpu().numpy(), g) < grad_tol(k), k


def test_full_size_train_step_properties(cuda):
    """BASELINE config 2 shapes (B=8, 20000 pts, 128 queries, 256-d, 8 decoder layers)."""
    import ov3d_amd
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import default_args
    args = default_args()
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(8, seed=1, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(inputs)
    loss, ld = crit(out, batch)
    assert torch.isfinite(loss) and len(ld) == 48  # 6 weighted+cardinality keys x 8 (no 2D branch)
    loss.backward()
    gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1)
    assert torch.isfinite(gn)
    # sampling invariants at full size
    from ov3d_amd import pointnet2_utils as pu
    idx, nx = pu.furthest_point_sample_gather(batch["point_clouds"], 2048)
    assert (idx[:, 0] == 0).all()
    for b in range(8):
        assert torch.unique(idx[b]).numel() == 2048
    bq = pu.ball_query(0.2, 64, batch["point_clouds"], nx)
    d = ((batch["point_clouds"][torch.arange(8, device=cuda)[:, None, None], bq.long()] - nx[:, :, None]) ** 2).sum(-1)
    assert (d < 0.2 ** 2 + 1e-6).all()
    assert (bq[..., 1:] >= bq[..., :1]).all()   # padded with the first hit, ascending


def test_full_size_c4_train_step_properties(cuda):
    """BASELINE config C4 shapes (ScanNet: B=8, 40000 points + colour, masked encoder with
    the interim SA, 256 queries, GIoU loss, enc_dropout 0.3), bf16: the HIP kernels of the
    masked path run (packed mask, masked flash attention, interim SA row kernels, the
    neighbour max-pool), the step is finite, and the sampling invariants hold at N=40000."""
    import ov3d_amd
    from ov3d_amd import _native, synthetic
    from ov3d_amd.dataset_config import ScannetDatasetConfig
    from bench import WORKLOADS, default_args
    wl = WORKLOADS["scannet"]
    args = default_args(**wl["args"])
    cfg = ScannetDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding(cfg.num_semcls + 1))
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(8, seed=2, num_points=wl["points"], device=cuda, dataset="scannet",
                                 use_color=True)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    _native.census_start()
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(inputs)
        loss, ld = crit(out, batch)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        called = _native.census_stop()
    for k in ("ov3d_attn_mask_pack", "ov3d_attn_fwd_masked", "ov3d_attn_bwd_masked",
              "ov3d_giou3d_bwd", "ov3d_sa_layer_pool_fwd", "ov3d_fps", "ov3d_ball_query_cells",
              "ov3d_rows256"):
        assert called.get(k), (k, sorted(called))
    # the interim SA's last BN + ReLU inside its neighbour max-pool (heads.bn_relu_pool_rows)
    assert called.get("ov3d_nbr_max_bnrelu_fwd") and called.get("ov3d_rows_bn_bwd_pooled"), \
        sorted(called)
    # the interim SA's grouped rows: bf16, zero-padded to 264 columns (aligned GEMM K)
    assert called.get("ov3d_group_rows_bf16"), sorted(called)
    assert called.get("ov3d_group_bwd_csr_bf16"), sorted(called)
    assert torch.isfinite(loss) and len(ld) == 56
    assert out["outputs"]["sem_cls_logits"].shape[:2] == (8, 256)
    gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1)
    assert torch.isfinite(gn) and gn > 0
    from ov3d_amd import pointnet2_utils as pu
    idx, nx = pu.furthest_point_sample_gather(batch["point_clouds"][..., :3].contiguous(), 2048)
    assert (idx[:, 0] == 0).all()
    for b in range(8):
        assert torch.unique(idx[b]).numel() == 2048


def test_graphed_step_equals_eager(cuda):
    """hipGraph replay of forward+backward gives the eager results (dropout off)."""
    import copy
    import ov3d_amd
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from ov3d_amd.graphs import GraphedModel
    from bench import default_args
    args = default_args(enc_dropout=0.0, dec_dropout=0.0, mlp_dropout=0.0, preenc_npoints=512,
                        nqueries=64)
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    twin = copy.deepcopy(model)
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(2, seed=4, num_points=4096, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    graphed = GraphedModel(twin, batch, amp_dtype=None, warmup_iters=1)
    # warm-up iterations ran the BN updates on `twin`: align the eager model's buffers
    model.load_state_dict(twin.state_dict())
    loss_e, _ = crit(model(inputs), dict(batch))
    loss_e.backward()
    loss_g, _ = crit(graphed(inputs), dict(batch))
    loss_g.backward()
    assert abs(loss_e.item() - loss_g.item()) <= 1e-5 * abs(loss_e.item())
    ge = dict(model.named_parameters())
    for n, p in twin.named_parameters():
        if p.grad is not None:
            torch.testing.assert_close(p.grad, ge[n].grad, rtol=1e-4, atol=1e-6)


def test_step_has_no_host_sync_and_matcher_equals_scipy(cuda):
    """Full-size forward + criterion + backward run without a single device->host
    synchronisation (torch sync-debug mode "error"), and the device Hungarian
    assignments equal scipy.optimize.linear_sum_assignment (criterion.py:79) on the
    same cost matrices."""
    import ov3d_amd
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import default_args
    from scipy.optimize import linear_sum_assignment
    args = default_args()
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(8, seed=3, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    seen = {}
    solve = crit.matcher.forward

    def spy(cost, nact):
        seen["cost"], seen["nact"] = cost, nact
        seen.update(solve(cost, nact))
        return seen
    crit.matcher.forward = spy
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(inputs)
        loss, _ = crit(out, batch)
        loss.backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert torch.isfinite(loss)
    cost = seen["cost"].float().cpu().numpy()
    nact = seen["nact"].cpu().numpy()
    inds = seen["per_prop_gt_inds"].cpu().numpy()
    mask = seen["proposal_matched_mask"].cpu().numpy()
    assert int(seen["status"].abs().sum()) == 0
    for p in range(cost.shape[0]):
        exp_i = np.zeros(cost.shape[1], np.int64)
        exp_m = np.zeros(cost.shape[1], np.float32)
        if nact[p]:
            r, c = linear_sum_assignment(cost[p, :, :nact[p]])
            exp_i[r], exp_m[r] = c, 1
        np.testing.assert_array_equal(mask[p], exp_m)
        np.testing.assert_array_equal(inds[p], exp_i)
    asg = seen["assignments"]
    assert len(asg) == cost.shape[0] and len(asg[0]) in (0, 2)


@pytest.mark.parametrize("mid_start,split_at", [("0", "encoder"), ("1", "encoder"),
                                                ("1", "pre_encoder")])
def test_step_graph_equals_eager_step(cuda, monkeypatch, mid_start, split_at):
    """graphs.StepGraph (whole step captured once: forward, criterion, backward, clip, fused
    AdamW) replays the eager step: same loss, same updated parameters and BN statistics.  Also
    as two graphs with the sampling plan released between them (OV3D_PLAN_MID_START=1), split
    after the encoder or after the pre-encoder SA."""
    import copy
    import ov3d_amd
    from ov3d_amd import graphs
    monkeypatch.setattr(graphs, "MID_START", mid_start)
    monkeypatch.setattr(graphs, "SPLIT_AT", split_at)
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from ov3d_amd.graphs import StepGraph
    from bench import default_args, train_step
    args = default_args(enc_dropout=0.0, dec_dropout=0.0, mlp_dropout=0.0, preenc_npoints=512,
                        nqueries=64)
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    twin = copy.deepcopy(model)
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)

    def adamw(m):
        return torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=args.base_lr,
                                 weight_decay=args.weight_decay, fused=True, capturable=True)
    opt_e, opt_g = adamw(model), adamw(twin)
    b1 = synthetic.make_batch(2, seed=4, num_points=4096, device=cuda)
    b2 = synthetic.make_batch(2, seed=5, num_points=4096, device=cuda)
    amp = torch.bfloat16
    sg = StepGraph(twin, crit, opt_g, b1, amp_dtype=amp, clip=args.clip_gradient, warmup_iters=1)
    assert (sg.graph2 is not None) == (mid_start == "1")
    # start the eager side from the graph side's state (parameters, BN buffers, AdamW state):
    # one step then differs only by run-to-run noise of atomics-based kernels
    model.load_state_dict(twin.state_dict())
    opt_e.load_state_dict(opt_g.state_dict())
    loss_e = train_step(model, crit, opt_e, b2, args, amp)
    loss_g = sg.step(b2)
    torch.cuda.synchronize()
    assert abs(loss_e.item() - loss_g.item()) <= 2e-3 * abs(loss_e.item())
    # gradients (after clipping) agree up to run-to-run noise of atomics-based kernels;
    # parameters after AdamW would amplify that noise on near-zero gradients (m / sqrt(v))
    ge = dict(model.named_parameters())
    for n, p in twin.named_parameters():
        if p.grad is None:
            continue
        d = (p.grad.float() - ge[n].grad.float()).norm() / ge[n].grad.float().norm().clamp_min(1e-12)
        assert d.item() < 2e-2, (n, d.item())
    be, bg = dict(model.named_buffers()), dict(twin.named_buffers())
    for k, v in be.items():
        if v.is_floating_point():
            torch.testing.assert_close(bg[k], v, rtol=1e-3, atol=1e-5, msg=k)
        else:
            assert torch.equal(bg[k], v), k


@pytest.mark.parametrize("masked", [False, True])
def test_sampling_plan_inputs_give_identical_forward(cuda, masked):
    """Model3DETR.sampling_plan (pre-encoder FPS + points, its ball query, the query FPS;
    masked encoder: also the interim SA's FPS + points and ball query: computed ahead of
    time by graphs.StepGraph on a side stream) fed back as inputs gives the forward
    without it, bit for bit"""
    import ov3d_amd
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import ScannetDatasetConfig, SunrgbdDatasetConfig
    from bench import default_args
    extra_args = dict(enc_type="masked", use_color=True) if masked else {}
    args = default_args(enc_dropout=0.0, dec_dropout=0.0, mlp_dropout=0.0, preenc_npoints=512,
                        nqueries=64, **extra_args)
    cfg = ScannetDatasetConfig() if masked else SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding(
        cfg.num_semcls + 1))
    model = model.to(cuda).train()
    b = synthetic.make_batch(2, seed=6, num_points=4096, device=cuda,
                             dataset="scannet" if masked else "sunrgbd", use_color=masked)
    inputs = {k: b[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    plan = model.sampling_plan(b["point_clouds"])
    interim = {k for k in model.PLAN_KEYS if k.startswith("interim")}
    assert set(plan) == (set(model.PLAN_KEYS) if masked else set(model.PLAN_KEYS) - interim)
    outs = []
    for extra in ({}, plan):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            outs.append(model({**inputs, **extra}))
    for k in ("sem_cls_logits", "center_unnormalized", "size_unnormalized", "angle_continuous"):
        assert torch.equal(outs[0]["outputs"][k], outs[1]["outputs"][k]), k


def test_second_forward_does_not_change_first_backward(cuda):
    """Dropout masks are regenerated in the backward from the seed SNAPSHOT the forward used
    (attention._seed, saved on every op's ctx).  The reference's --use_pseudo_labels loop
    runs a second train-mode forward (EMA teacher) between a forward and its backward
    (engine.py): the first forward's gradients must equal a plain forward + backward."""
    import ov3d_amd
    from ov3d_amd import attention as flash
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import default_args
    args = default_args(preenc_npoints=512, nqueries=64)   # dropout ON (0.1 / 0.3)
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(2, seed=8, num_points=4096, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    live0 = flash._live(cuda).clone()

    def run(second):
        flash._live(cuda).copy_(live0)
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(inputs)
            if second:   # teacher-style pass: train mode, new masks, its own graph
                out2 = model(inputs)
        loss, _ = crit(out, dict(batch))
        loss.backward()
        if second:
            assert not torch.equal(out2["outputs"]["center_normalized"],
                                   out["outputs"]["center_normalized"])
        return loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters()
                             if p.grad is not None}

    l1, g1 = run(False)
    l2, g2 = run(True)
    assert l1 == l2
    assert g1.keys() == g2.keys()
    for n in g1:
        d = (g1[n] - g2[n]).norm() / g1[n].norm().clamp_min(1e-12)
        assert d.item() < 1e-3, (n, d.item())


def test_decoder_rows_fp32_unless_fused_heads(cuda):
    """The fused decoder writes its layer outputs as bf16 rows only when the fused heads
    launch consumes them (train, bf16 autocast); in eval the per-head fp32 path gets fp32
    decoder outputs (transformer.py xb_into)."""
    import ov3d_amd
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import default_args
    args = default_args()
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda)
    batch = synthetic.make_batch(2, seed=4, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    seen = {}
    orig = model.get_box_predictions

    def spy(qx, dims, feats):
        seen["feats"] = feats
        return orig(qx, dims, feats)
    model.get_box_predictions = spy
    for mode in ("train", "eval"):
        getattr(model, mode)()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            model(inputs)
        seen[mode] = seen.pop("feats")
    assert seen["train"].dtype == torch.bfloat16
    assert seen["eval"].dtype == torch.float32
    assert torch.isfinite(seen["eval"]).all()
