"""Fused prediction heads (heads.py + csrc/bnrows.hip + ov3d_wgrad) against the five
per-head GenericMLPs evaluated in fp32 PyTorch on the same rows: outputs, BatchNorm
running statistics and every parameter gradient.  bf16 operands inside the fused path:
outputs within 3e-2 relative (Frobenius), and running statistics and every
gradient no further from fp32 than PyTorch's own bf16-autocast evaluation of the same
heads (x1.5, or 3e-2): the two BatchNorm backward passes amplify bf16 rounding."""
import copy

import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


def _model(cuda):
    from bench import default_args
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    import ov3d_amd
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(default_args(), SunrgbdDatasetConfig(),
                                    text_embedding=synthetic.text_embedding())
    return model.to(cuda).train()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def test_fused_heads_match_per_head_fp32(cuda):
    from ov3d_amd import heads as H
    model = _model(cuda)
    ref_heads = copy.deepcopy(model.mlp_heads)
    fus_heads = model.mlp_heads
    for hs in (ref_heads, fus_heads):
        for m in hs.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
    torch.manual_seed(1)
    rows = torch.randn(8192, 256, device=cuda)
    g = {n: torch.randn(8192, fus_heads[n].layers[-1].out_channels, device=cuda) for n in H.HEAD_ORDER}

    out_r = {n: ref_heads[n].rows(rows) for n in H.HEAD_ORDER}
    sum(((out_r[n] * g[n]).sum() for n in H.HEAD_ORDER)).backward()
    # PyTorch's own bf16 autocast evaluation of the per-head MLPs: the error budget
    bf_heads = copy.deepcopy(ref_heads)
    for p_ in bf_heads.parameters():
        p_.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out_b = {n: bf_heads[n].rows(rows) for n in H.HEAD_ORDER}
    sum(((out_b[n].float() * g[n]).sum() for n in H.HEAD_ORDER)).backward()

    pack = H.HeadPack(fus_heads)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert H.supported(pack, rows)
        out_f = H.fused_heads(pack, rows)
    sum(((out_f[n] * g[n]).sum() for n in H.HEAD_ORDER)).backward()

    for n in H.HEAD_ORDER:
        assert out_f[n].shape == out_r[n].shape
        assert _rel(out_f[n], out_r[n]) < 3e-2, (n, _rel(out_f[n], out_r[n]))
        for (name, pr), pf, pb in zip(ref_heads[n].named_parameters(), fus_heads[n].parameters(),
                                      bf_heads[n].parameters()):
            assert pf.grad is not None, (n, name)
            ef, eb = _rel(pf.grad, pr.grad), _rel(pb.grad, pr.grad)
            # no further from fp32 than PyTorch's bf16 autocast path (or within 3e-2)
            assert ef <= max(1.5 * eb, 3e-2), (n, name, ef, eb)
        for (name, br), bf, bb in zip(ref_heads[n].named_buffers(), fus_heads[n].buffers(),
                                      bf_heads[n].buffers()):
            if br.dtype.is_floating_point:
                ef, eb = _rel(bf, br), _rel(bb, br)
                assert ef <= max(1.5 * eb, 5e-3), (n, name, ef, eb)
            else:
                assert torch.equal(bf, br), (n, name)
    # the state dict keeps the reference keys and shapes
    assert set(model.state_dict()) == set(_model(cuda).state_dict())


@pytest.mark.parametrize("lq", [0, 128])
def test_fused_heads_text_alignment(cuda, lq):
    """the sem_cls Linear folded into the heads' output launch (model_3detr.py:152-154,
    237-238): logits (row-major, or the reference's transposed Q8 layout) and every head
    gradient, against fp32 PyTorch, no further off than PyTorch's bf16 autocast"""
    from ov3d_amd import heads as H
    model = _model(cuda)
    sem = model.mlp_heads["sem_cls_head"]
    ref_heads = copy.deepcopy(model.mlp_heads)
    fus_heads = model.mlp_heads
    for hs in (ref_heads, fus_heads):
        for m in hs.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
    torch.manual_seed(2)
    R = 8192
    rows = torch.randn(R, 256, device=cuda)
    T = sem.weight.shape[0]
    gl = torch.randn(R, T, device=cuda)
    gv = torch.randn(R, 640, device=cuda)

    def ref_loss(hs, amp):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            vis = hs["visual_embed_head"].rows(rows)
        vis = vis.float()
        lg = vis @ sem.weight.t()
        if lq:
            lg = lg.reshape(R // lq, lq, T).transpose(1, 2).reshape(R, T)
        (lg * gl).sum().backward(retain_graph=True)
        (vis * gv).sum().backward()
        return lg.detach()

    lg_r = ref_loss(ref_heads, False)
    bf_heads = copy.deepcopy(ref_heads)
    for p_ in bf_heads.parameters():
        p_.grad = None
    lg_b = ref_loss(bf_heads, True)
    pack = H.HeadPack(fus_heads)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = H.fused_heads(pack, rows, sem=sem, lq=lq)
    assert "sem_cls_logits" in out
    ((out["sem_cls_logits"] * gl).sum() + (out["visual_embed_head"] * gv).sum()).backward()
    el, eb = _rel(out["sem_cls_logits"], lg_r), _rel(lg_b, lg_r)
    assert el <= max(1.5 * eb, 1e-2), (el, eb)
    for (name, pr), pf, pb in zip(ref_heads["visual_embed_head"].named_parameters(),
                                  fus_heads["visual_embed_head"].parameters(),
                                  bf_heads["visual_embed_head"].parameters()):
        ef, eb = _rel(pf.grad, pr.grad), _rel(pb.grad, pr.grad)
        assert ef <= max(1.5 * eb, 3e-2), (name, ef, eb)


def test_fused_heads_dropout_and_step(cuda):
    """Model-level: a bf16 training step takes the fused heads (dropout 0.3 active) and
    produces finite losses and gradients for every head parameter."""
    from bench import default_args
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    import ov3d_amd
    model = _model(cuda)
    crit = ov3d_amd.build_criterion(default_args(), SunrgbdDatasetConfig()).to(cuda)
    batch = synthetic.make_batch(4, seed=3, device=cuda)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min",
                                           "point_cloud_dims_max")})
    assert model._head_pack is not None and model._head_pack.store is not None
    loss, _ = crit(out, batch)
    loss.backward()
    assert torch.isfinite(loss)
    for n, p in model.mlp_heads.named_parameters():
        if p.requires_grad:
            assert p.grad is not None and torch.isfinite(p.grad).all(), n


def test_bn_relu_rows_projection_matches_torch(cuda):
    """encoder -> decoder projection GenericMLP (model_3detr.py:106-120) in training under
    bf16 autocast: the fused BN + ReLU row launches (heads.bn_relu_rows) against PyTorch's
    BatchNorm1d + ReLU on the same module: outputs, running statistics and gradients."""
    import copy
    from ov3d_amd.helpers import GenericMLP
    torch.manual_seed(0)
    m0 = GenericMLP(input_dim=256, hidden_dims=[256, 256], output_dim=256, norm_fn_name="bn1d",
                    activation="relu", use_conv=True, output_use_activation=True,
                    output_use_norm=True, output_use_bias=False).to(cuda).train()
    m1 = copy.deepcopy(m0)
    x = torch.randn(16384, 256, device=cuda)
    outs, grads = [], []
    for m, fused in ((m0, False), (m1, True)):
        xi = x.clone().requires_grad_()
        if fused:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = m.rows(xi)
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = xi
                for layer in m.layers:   # plain module chain (reference semantics)
                    if isinstance(layer, torch.nn.Conv1d):
                        y = y @ layer.weight.view(layer.weight.shape[0], -1).t().to(y.dtype)
                    else:
                        y = layer(y)
        (y.float() * torch.linspace(-1, 1, 256, device=cuda)).sum().backward()
        outs.append(y.float().detach())
        grads.append([xi.grad] + [p.grad for p in m.parameters()])
    assert _rel(outs[1], outs[0]) < 2e-2
    for bn0, bn1 in zip([l for l in m0.layers if isinstance(l, torch.nn.BatchNorm1d)],
                        [l for l in m1.layers if isinstance(l, torch.nn.BatchNorm1d)]):
        assert _rel(bn1.running_mean, bn0.running_mean) < 1e-2
        assert _rel(bn1.running_var, bn0.running_var) < 1e-2
        assert int(bn1.num_batches_tracked) == int(bn0.num_batches_tracked) == 1
    for a, b in zip(grads[1], grads[0]):
        assert _rel(a, b) < 3e-2


@pytest.mark.parametrize("ds", ["sunrgbd", "scannet"])
def test_box_param_fused_matches_torch(cuda, ds):
    """csrc/boxparam.hip (model_3detr._BoxParam) against the torch BoxProcessor expressions on
    the same raw head rows: all 13 outputs and the raw-row gradient, corners included."""
    import numpy as np
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import CONFIGS
    model = _model(cuda)
    cfg = CONFIGS[ds]()
    model.box_processor.dataset_config = cfg
    L, B, Q, NB = 8, 4, 128, cfg.num_angle_bin
    R = L * B * Q
    g = torch.Generator().manual_seed(1)
    raw = (torch.randn(R, 6 + 2 * NB, generator=g) * 2).to(cuda)
    vis = torch.randn(R, 640, generator=g).to(cuda)
    if ds == "scannet":
        sem = torch.nn.Linear(640, 19, bias=False).to(cuda)
        model.mlp_heads["sem_cls_head"] = sem
    batch = synthetic.make_batch(B, seed=4, num_points=2048, device=cuda)
    dims = [batch["point_cloud_dims_min"].float(), batch["point_cloud_dims_max"].float()]
    qxyz = batch["point_clouds"][:, :Q, :3].contiguous()
    res = {}
    for fused in (False, True):
        r = raw.clone().requires_grad_()
        names = ("center_head", "size_head", "angle_cls_head", "angle_residual_head")
        widths = (3, 3, NB, NB)
        pre = {"visual_embed_head": vis}
        o = 0
        for n, w in zip(names, widths):
            pre[n] = r[:, o:o + w]
            o += w
        if fused:
            pre["_raw"] = r
        out = model._box_predictions(qxyz, dims, None, (L, Q, B), pre)["_layers_stacked"]
        gen = torch.Generator(device=cuda).manual_seed(7)
        loss = 0
        for k in ("center_normalized", "center_unnormalized", "size_normalized",
                  "size_unnormalized", "angle_logits", "angle_residual",
                  "angle_residual_normalized", "angle_continuous", "box_corners"):
            loss = loss + (out[k] * torch.randn(out[k].shape, device=cuda, generator=gen)).sum()
        loss.backward()
        res[fused] = ({k: v.detach() for k, v in out.items()}, r.grad)
    (a, ga), (b, gb) = res[True], res[False]
    for k in b:
        assert a[k].shape == b[k].shape, k
        assert torch.allclose(a[k], b[k], rtol=1e-5, atol=1e-5), (k, (a[k] - b[k]).abs().max())
    assert torch.allclose(ga, gb, rtol=1e-4, atol=1e-5), (ga - gb).abs().max()
    assert np.isfinite(ga.cpu().numpy()).all()


def test_fourier_pe_kernel_matches_torch(cuda):
    """ov3d_fourier_pe against the module's torch expression (run on the CPU, fp32)"""
    from ov3d_amd.position_embedding import PositionEmbeddingCoordsSine
    torch.manual_seed(3)
    pe = PositionEmbeddingCoordsSine(d_pos=256, pos_type="fourier", normalize=True)
    xyz = torch.rand(4, 2048, 3) * 6 - 3
    rng = [xyz.min(1).values - 0.1, xyz.max(1).values + 0.1]
    ref = pe.rows(xyz, input_range=rng)
    out = pe.to(cuda).rows(xyz.to(cuda), input_range=[r.to(cuda) for r in rng]).cpu()
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() < 2e-5


@pytest.mark.parametrize("C,nparts", [(256, 1024), (1280, 1024), (64, 37)])
def test_bn_stats_finalize_one_launch_bitwise(cuda, C, nparts):
    """ov3d_bn_stats_finalize / ov3d_bn_bwd_stats_finalize (column totals + finalize in one
    launch) equal ov3d_reduce_partials followed by ov3d_bn_finalize / ov3d_bn_bwd_finalize"""
    from ov3d_amd import _native as nat
    g = torch.Generator(device=cuda).manual_seed(C)
    parts = torch.rand((nparts, 2 * C), dtype=torch.float64, device=cuda, generator=g)
    parts[:, C:] += parts[:, :C] ** 2   # sum of squares >= square of sum / n
    gamma = torch.randn(C, device=cuda, generator=g)
    beta = torch.randn(C, device=cuda, generator=g)
    count = float(nparts * 3)
    outs = []
    for fused in (True, False):
        rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
        nbt = torch.zeros((), dtype=torch.int64, device=cuda)
        st = [torch.empty(C, device=cuda) for _ in range(4)]
        bw = [torch.empty(C, device=cuda) for _ in range(5)]
        if fused:
            nat.call("ov3d_bn_stats_finalize", parts, nparts, C, count, gamma, beta, 1e-5, 0.1, rm,
                     rv, *st, nbt, like=parts)
            nat.call("ov3d_bn_bwd_stats_finalize", parts, nparts, C, count, gamma, st[0], st[1],
                     *bw, like=parts)
        else:
            tot = torch.empty(2 * C, dtype=torch.float64, device=cuda)
            nat.call("ov3d_reduce_partials", parts, nparts, 2 * C, tot, like=parts)
            nat.call("ov3d_bn_finalize", tot, count, C, gamma, beta, 1e-5, 0.1, rm, rv, *st, nbt,
                     like=parts)
            nat.call("ov3d_bn_bwd_finalize", tot, count, C, gamma, st[0], st[1], *bw, like=parts)
        outs.append(st + bw + [rm, rv, nbt])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert int(outs[0][-1]) == 1
