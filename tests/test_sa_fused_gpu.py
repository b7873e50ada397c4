"""Fused SA MLP (csrc/sa_mlp.hip via sa_fused.py) on the GPU.

Floating-point kernels: checked against plain PyTorch fp32 computations.
  * kernel level, on identical bf16 inputs: each layer's GEMM + folded BN + ReLU, the
    BN statistics, the pooled max / arg rows (tolerance: one bf16 ulp of the output,
    accumulation order differs);
  * module level: PointnetSAModuleVotes training step under bf16 autocast (fused) vs
    the same module in fp32 (unfused rows path = reference semantics): outputs,
    running statistics and every parameter gradient within bf16 tolerances.
"""
import copy

import numpy as np
import pytest
import torch

from helpers import ov3d

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def test_layer_kernel_matches_torch(cuda):
    from ov3d_amd import _native as nat
    g = torch.Generator(device="cpu").manual_seed(0)
    R, K, N = 64 * 300, 64, 128
    y = (torch.randn(R, K, generator=g) * 2).to(torch.bfloat16).to(cuda)
    sc = (torch.randn(K, generator=g)).to(cuda)
    sh = (torch.randn(K, generator=g) * 0.5).to(cuda)
    W = (torch.randn(N, K, generator=g) * 0.2).to(torch.bfloat16).to(cuda)
    z = torch.empty(R, K, dtype=torch.bfloat16, device=cuda)
    out = torch.empty(R, N, dtype=torch.bfloat16, device=cuda)
    parts = torch.empty(64, 2, N, dtype=torch.float64, device=cuda)
    nat.call("ov3d_sa_layer_fwd", y, sc, sh, W, R, K, N, z, out, parts, 64, like=y)
    zr = torch.relu(torch.addcmul(sh, sc, y.float())).to(torch.bfloat16)
    zr2 = torch.relu(sc * y.float() + sh).to(torch.bfloat16)
    # fmaf vs mul+add may differ by an ulp before rounding: accept either
    assert ((z == zr) | (z == zr2)).float().mean().item() > 0.999
    ref = z.float() @ W.float().t()
    assert _rel(out.float(), ref) < 8e-3
    tot = parts.sum(0)
    o = out.double()
    torch.testing.assert_close(tot[0], o.sum(0), rtol=1e-5, atol=1e-2)   # fp32 per-lane sums
    torch.testing.assert_close(tot[1], (o * o).sum(0), rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("S", [64, 32])
def test_pool_kernel_max_min_rows(cuda, S):
    from ov3d_amd import _native as nat
    g = torch.Generator(device="cpu").manual_seed(1)
    R, K, N = 64 * 128, 128, 256
    y = torch.randn(R, K, generator=g).to(torch.bfloat16).to(cuda)
    sc = torch.rand(K, generator=g).to(cuda) + 0.5
    sh = torch.randn(K, generator=g).to(cuda) * 0.1
    W = (torch.randn(N, K, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    P = R // S
    pmax, pmin = (torch.empty(P, N, device=cuda) for _ in range(2))
    imax, imin = (torch.empty(P, N, dtype=torch.uint8, device=cuda) for _ in range(2))
    parts = torch.empty(32, 2, N, dtype=torch.float64, device=cuda)
    z = torch.empty(R, K, dtype=torch.bfloat16, device=cuda)
    nat.call("ov3d_sa_layer_pool_fwd", y, sc, sh, W, R, K, N, S, z, pmax, pmin, imax, imin, None,
             parts, 32, like=y)
    yf = (z.float() @ W.float().t()).to(torch.bfloat16).float().view(P, S, N)
    assert _rel(pmax, yf.max(1).values) < 8e-3
    assert _rel(pmin, yf.min(1).values) < 8e-3
    # the recorded rows hold the recorded extremes (up to accumulation-order ulps)
    at_max = torch.gather(yf, 1, imax.long()[:, None, :])[:, 0]
    at_min = torch.gather(yf, 1, imin.long()[:, None, :])[:, 0]
    assert (at_max - pmax).abs().max().item() <= 0.02 * pmax.abs().max().item()
    assert (at_min - pmin).abs().max().item() <= 0.02 * pmin.abs().max().item()
    assert int(imax.max()) < S and int(imin.max()) < S


@pytest.mark.parametrize("S", [64, 32])
def test_pool_one_extreme_equals_both(cuda, S):
    """Given the BN weight, the layer-3 pool kernel keeps only the extreme its sign selects
    (MODE_POOL1): those values, rows and the BN partial sums are the bits the two-extreme
    kernel produces."""
    from ov3d_amd import _native as nat
    g = torch.Generator(device="cpu").manual_seed(3)
    R, K, N = 64 * 256, 128, 256
    y = torch.randn(R, K, generator=g).to(torch.bfloat16).to(cuda)
    sc = torch.rand(K, generator=g).to(cuda) + 0.5
    sh = torch.randn(K, generator=g).to(cuda) * 0.1
    W = (torch.randn(N, K, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    gamma = torch.randn(N, generator=g).to(cuda)
    gamma[:8] = 0.0
    gamma[8:16] = -0.0
    P = R // S
    out = []
    for gm in (None, gamma):
        pmax, pmin = (torch.full((P, N), float("nan"), device=cuda) for _ in range(2))
        imax, imin = (torch.full((P, N), 255, dtype=torch.uint8, device=cuda) for _ in range(2))
        parts = torch.empty(64, 2, N, dtype=torch.float64, device=cuda)
        nat.call("ov3d_sa_layer_pool_fwd", y, sc, sh, W, R, K, N, S, None, pmax, pmin, imax, imin,
                 gm, parts, 64, like=y)
        out.append((pmax, pmin, imax, imin, parts))
    up = ~(gamma < 0)        # ov3d_sa_pool_fwd's a >= 0 (a = gamma * invstd)
    (amx, amn, aix, ain, ap), (bmx, bmn, bix, bin_, bp) = out
    assert torch.equal(torch.where(up, amx, amn), torch.where(up, bmx, bmn))
    assert torch.equal(torch.where(up, aix, ain), torch.where(up, bix, bin_))
    assert torch.equal(ap, bp)
    assert int(up.sum()) not in (0, N)


def _sa_copies(cuda, n, seed=0):
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    torch.manual_seed(seed)
    sa = PointnetSAModuleVotes(radius=0.2, nsample=64, npoint=2048, mlp=[0, 64, 128, 256],
                               normalize_xyz=True).to(cuda).train()
    with torch.no_grad():   # non-trivial BN affine, some negative gammas (min-pool branch)
        for layer in sa.mlp_module:
            bn = layer.bn.bn
            bn.weight.copy_(torch.randn_like(bn.weight) * 0.5 + 0.6)
            bn.bias.copy_(torch.randn_like(bn.bias) * 0.2)
    return [copy.deepcopy(sa) for _ in range(n)]


def _run(sa, xyz, gw, amp, fused, monkeypatch):
    from ov3d_amd import sa_fused
    if not fused:
        monkeypatch.setattr(sa_fused, "supported", lambda *a: False)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        _, f, inds = sa(xyz)
    monkeypatch.undo()
    (f.float() * gw).sum().backward()
    return f.detach().float(), inds, {n: p.grad for n, p in sa.named_parameters()}


def test_sa_module_fused_vs_fp32_reference(cuda, monkeypatch):
    """fused bf16 vs fp32 reference: outputs / running stats within bf16 tolerance, and every
    gradient no further from fp32 than PyTorch's own bf16-autocast path (+ slack)."""
    from ov3d_amd import synthetic
    ref, unf, fus = _sa_copies(cuda, 3)
    xyz = synthetic.make_batch(4, seed=5, device=cuda)["point_clouds"]
    gw = torch.randn(4, 256, 2048, device=cuda)
    f_ref, i_ref, g_ref = _run(ref, xyz, gw, False, False, monkeypatch)
    f_unf, _, g_unf = _run(unf, xyz, gw, True, False, monkeypatch)
    f_fus, i_fus, g_fus = _run(fus, xyz, gw, True, True, monkeypatch)
    assert torch.equal(i_fus, i_ref)
    assert f_fus.shape == f_ref.shape == (4, 256, 2048)
    e_out, e_out_unf = _rel(f_fus, f_ref), _rel(f_unf, f_ref)
    assert e_out < 3e-2, (e_out, e_out_unf)
    for lf, lr in zip(fus.mlp_module, ref.mlp_module):
        bf, br = lf.bn.bn, lr.bn.bn
        assert int(bf.num_batches_tracked) == int(br.num_batches_tracked) == 1
        assert _rel(bf.running_mean, br.running_mean) < 2e-2
        assert _rel(bf.running_var, br.running_var) < 2e-2
    report = {n: (round(_rel(g_fus[n], g_ref[n]), 4), round(_rel(g_unf[n], g_ref[n]), 4))
              for n in g_ref}
    print("grad rel err (fused, torch-bf16):", report)
    for n, (ef, eu) in report.items():
        assert ef <= max(2.0 * eu, 3e-2), (n, ef, eu)


def test_model_step_uses_fused_sa_and_trains(cuda):
    """Full-size bf16 step: the pre-encoder SA runs the fused kernels, loss finite."""
    import ov3d_amd
    from ov3d_amd import _native, synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import default_args
    args = default_args()
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(8, seed=2, device=cuda)
    _native.timing_enable(["ov3d_sa_layer_pool_fwd", "ov3d_sa_layer_dy", "ov3d_sa_dy_fused"])
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model({k: batch[k] for k in ("point_clouds", "point_cloud_dims_min",
                                           "point_cloud_dims_max")})
    loss, _ = crit(out, batch)
    loss.backward()
    t = _native.timing_collect()
    assert len(t["ov3d_sa_layer_pool_fwd"]) == 1
    assert len(t["ov3d_sa_dy_fused"]) == 1 and len(t["ov3d_sa_layer_dy"]) == 0   # one-pass bwd
    assert torch.isfinite(loss)
    w = model.pre_encoder.mlp_module.layer0.conv.weight
    assert w.grad is not None and torch.isfinite(w.grad).all() and w.grad.abs().sum() > 0


@pytest.mark.parametrize("nsample", [64, 32])
def test_last_layer_backward_one_pass_equals_three_passes(cuda, monkeypatch, nsample):
    """csrc/sa_bwd.hip (dy3 -> dz2 and dW3 in one pass, dy3 / z2 never stored) against the dy
    recompute kernel + dW GEMM + dgrad GEMM: same gradients up to fp32 summation order"""
    from ov3d_amd import sa_fused, synthetic
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    torch.manual_seed(3)
    sa = PointnetSAModuleVotes(radius=0.2, nsample=nsample, npoint=2048, mlp=[0, 64, 128, 256],
                               normalize_xyz=True).to(cuda).train()
    with torch.no_grad():
        for layer in sa.mlp_module:
            bn = layer.bn.bn
            bn.weight.copy_(torch.randn_like(bn.weight) * 0.5 + 0.6)
            bn.bias.copy_(torch.randn_like(bn.bias) * 0.2)
    xyz = synthetic.make_batch(2, seed=9, device=cuda)["point_clouds"]
    gw = torch.randn(2, 256, 2048, device=cuda)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(sa_fused, "FUSED_BWD", fused)
        twin = copy.deepcopy(sa)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, f, _ = twin(xyz[..., :3].contiguous())
        (f.float() * gw).sum().backward()
        res[fused] = {n: p.grad.clone() for n, p in twin.named_parameters()}
    for n in res[False]:
        e = _rel(res[True][n], res[False][n])
        assert e < 2e-3, (n, e)


@pytest.mark.parametrize("kind", ["scannet_colour", "scannet_colour_rows", "interim"])
def test_sa_rows_bn_relu_path_vs_fp32(cuda, monkeypatch, kind):
    """ScanNet pre-encoder SA with colour (6 input channels): the fused MFMA kernels
    (sa_fused, first layer on 6 channels) — and, forced off, the rows path; the masked
    encoder's interim SA (256 features + xyz, gradient to the features): BN + ReLU on the
    HIP row kernels (heads.bn_relu_rows).  Under bf16 autocast, against the fp32 module:
    outputs, running statistics and gradients no further from fp32 than PyTorch's own bf16
    batch_norm path (+ slack)."""
    from ov3d_amd import heads, sa_fused, synthetic
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    torch.manual_seed(4)
    if kind.startswith("scannet_colour"):
        sa = PointnetSAModuleVotes(radius=0.2, nsample=64, npoint=512, mlp=[3, 64, 128, 256],
                                   normalize_xyz=True)
        B, N, C = 2, 4096, 3
    else:
        sa = PointnetSAModuleVotes(radius=0.4, nsample=32, npoint=256, mlp=[256, 256, 256, 256])
        B, N, C = 2, 1024, 256
    sa = sa.to(cuda).train()
    with torch.no_grad():
        for layer in sa.mlp_module:
            bn = layer.bn.bn
            bn.weight.copy_(torch.randn_like(bn.weight) * 0.5 + 0.6)
            bn.bias.copy_(torch.randn_like(bn.bias) * 0.2)
    xyz = synthetic.make_batch(B, seed=6, device=cuda)["point_clouds"][:, :N, :3].contiguous()
    feats0 = torch.randn(B, C, N, device=cuda)
    gw = None
    res = {}
    for name, amp, rows in (("ref", False, True), ("torch", True, False), ("hip", True, True)):
        twin = copy.deepcopy(sa)
        feats = feats0.clone().requires_grad_(kind == "interim")
        if not rows:
            monkeypatch.setattr(heads, "bn_relu_rows_ok", lambda *a: False)
        if not rows or kind != "scannet_colour":
            monkeypatch.setattr(sa_fused, "supported", lambda *a: False)
        calls, fcalls, pcalls = [], [], []
        real, freal, preal = heads.bn_relu_rows, sa_fused.sa_mlp_pool, heads.bn_relu_pool_rows
        monkeypatch.setattr(heads, "bn_relu_rows", lambda *a, **k: calls.append(1) or real(*a, **k))
        monkeypatch.setattr(heads, "bn_relu_pool_rows",
                            lambda *a, **k: pcalls.append(1) or preal(*a, **k))
        monkeypatch.setattr(sa_fused, "sa_mlp_pool", lambda *a, **k: fcalls.append(1) or freal(*a, **k))
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            _, f, _ = twin(xyz, feats)
        monkeypatch.undo()
        if gw is None:
            gw = torch.randn(f.shape, device=cuda)
        (f.float() * gw).sum().backward()
        fused = name == "hip" and kind == "scannet_colour"
        assert len(fcalls) == (1 if fused else 0), (name, len(fcalls))
        # the rows path: layers 1-2 on bn_relu_rows, the last BN + ReLU inside the pool
        # (heads.bn_relu_pool_rows) unless OV3D_BN_POOL=0
        rows_hip = name == "hip" and not fused
        assert len(pcalls) == (1 if rows_hip and heads.BN_POOL else 0), (name, len(pcalls))
        assert len(calls) + len(pcalls) == (3 if rows_hip else 0), (name, len(calls))
        g = {n: p.grad.clone() for n, p in twin.named_parameters()}
        if feats.requires_grad:
            g["features"] = feats.grad.clone()
        res[name] = (f.detach().float(), g, twin)
    f_ref, g_ref, m_ref = res["ref"]
    assert _rel(res["hip"][0], f_ref) < max(2.0 * _rel(res["torch"][0], f_ref), 3e-2)
    for lh, lr in zip(res["hip"][2].mlp_module, m_ref.mlp_module):
        bh, br = lh.bn.bn, lr.bn.bn
        assert int(bh.num_batches_tracked) == int(br.num_batches_tracked) == 1
        assert _rel(bh.running_mean, br.running_mean) < 2e-2
        assert _rel(bh.running_var, br.running_var) < 2e-2
    for n in g_ref:
        eh, et = _rel(res["hip"][1][n], g_ref[n]), _rel(res["torch"][1][n], g_ref[n])
        assert eh <= max(2.0 * et, 3e-2), (n, eh, et)


@pytest.mark.parametrize("S,C", [(32, 256), (64, 128), (5, 24)])
def test_neighbour_max_pool_kernel(cuda, S, C):
    """csrc/pool.hip: pooled values bit-exact vs torch max; the arg row is the first
    maximum of the window (max_pool2d order; bf16 rows have many ties); the backward routes
    each pooled gradient to that row and writes zeros elsewhere"""
    from ov3d_amd.pointnet2_modules import _NbrMax
    g = torch.Generator(device="cpu").manual_seed(S + C)
    P = 300
    y = (torch.randn(P * S, C, generator=g) * 3).round().to(torch.bfloat16).to(cuda)  # ties
    y.requires_grad_()
    out = _NbrMax.apply(y, S)
    ref = y.detach().view(P, S, C).max(dim=1).values
    assert torch.equal(out, ref)
    first = np.argmax(y.detach().float().view(P, S, C).cpu().numpy(), axis=1)   # first max
    gout = torch.randn(P, C, generator=g).to(torch.bfloat16).to(cuda)
    out.backward(gout)
    exp = torch.zeros(P, S, C, dtype=torch.bfloat16)
    exp.scatter_(1, torch.from_numpy(first).long()[:, None, :], gout.cpu()[:, None, :])
    assert torch.equal(y.grad.cpu(), exp.view(P * S, C))


@pytest.mark.parametrize("nparts,shape", [(256, (256, 128)), (256, (128, 64)), (37, (3, 5)),
                                          (1, (1000,)), (200, (64, 1024))])
def test_colsum_f32_equals_torch_sum(cuda, nparts, shape):
    """ov3d_colsum_f32 (the fused SA backward's dW partial sums) == part.sum(0) up to the
    summation order (f32); deterministic across calls."""
    from ov3d_amd import sa_fused
    g = torch.Generator(device="cpu").manual_seed(nparts)
    part = torch.randn((nparts,) + shape, generator=g).to(cuda)
    got = sa_fused._colsum(part)
    ref = part.double().sum(0).float()
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * nparts ** 0.5)
    assert torch.equal(got, sa_fused._colsum(part))


@pytest.mark.parametrize("nwg", [256, 1024])
def test_fused_backward_is_run_to_run_deterministic(cuda, monkeypatch, nwg):
    """the fused SA backward (sa_dy9 for layer 3, sa_dy2_fused for layer 2 with y1 recomputed from
    x0) gives bit-identical gradients run to run, at the default workgroup count and at 1024
    workgroups (four per CU's worth of work queued: any co-residency the register budget allows).
    Round 5's opt-in sa_dy2b failed exactly this at two workgroups per CU and was removed in
    round 6 (Fused SA MLP)."""
    from ov3d_amd import sa_fused, synthetic
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    monkeypatch.setattr(sa_fused, "NWG_DY2", nwg)
    monkeypatch.setattr(sa_fused, "NWG_DY_FUSED", nwg)
    torch.manual_seed(4)
    sa = PointnetSAModuleVotes(radius=0.2, nsample=64, npoint=2048, mlp=[0, 64, 128, 256],
                               normalize_xyz=True).to(cuda).train()
    xyz = synthetic.make_batch(8, seed=11, device=cuda)["point_clouds"][..., :3].contiguous()
    gw = torch.randn(8, 256, 2048, device=cuda)
    runs = []
    for _ in range(3):
        twin = copy.deepcopy(sa)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, f, _ = twin(xyz)
        (f.float() * gw).sum().backward()
        runs.append({n: p.grad.clone() for n, p in twin.named_parameters()})
    for r in runs[1:]:
        for n in runs[0]:
            assert torch.equal(r[n], runs[0][n]), n


def test_fused_sa_matches_cpu_twin(cuda):
    """the fused bf16 SA MLP + max-pool (sa_fused.sa_mlp_pool over the HIP kernels) against the
    boundary's CPU twin (oracle ov3d_sa_mlp_fwd_cpu / _bwd_cpu, float64, pinned to torch's
    Conv2d + BatchNorm2d + ReLU + max_pool2d in tests/test_oracle_twins.py): output and every
    weight / BN-affine gradient no further from the twin than PyTorch's own bf16 autocast of the
    same layers (x2, or within 3e-2)"""
    import torch.nn.functional as F
    from ov3d_amd import sa_fused
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    from oracle import oracle
    torch.manual_seed(7)
    sa = PointnetSAModuleVotes(radius=0.2, nsample=64, npoint=256, mlp=[0, 64, 128, 256],
                               normalize_xyz=True).to(cuda).train()
    with torch.no_grad():
        for layer in sa.mlp_module:
            bn = layer.bn.bn
            bn.weight.copy_(torch.randn_like(bn.weight) * 0.5 + 0.6)
            bn.bias.copy_(torch.randn_like(bn.bias) * 0.2)
    S, P = 64, 256
    g = torch.Generator(device="cpu").manual_seed(8)
    x0 = (torch.rand((P * S, 3), generator=g) * 2 - 1).to(cuda)
    dout = torch.randn((P, 256), generator=g).to(cuda)
    layers = list(sa.mlp_module)
    ws = [l.conv.weight.detach().view(l.conv.weight.shape[0], -1) for l in layers]
    gs = [l.bn.bn.weight.detach() for l in layers]
    bs = [l.bn.bn.bias.detach() for l in layers]
    cpu = lambda ts: [t.float().cpu().numpy() for t in ts]   # noqa: E731
    out_t, _, _, _ = oracle.sa_mlp(x0.cpu().numpy(), S, cpu(ws), cpu(gs), cpu(bs))
    dW_t, dg_t, db_t = oracle.sa_mlp_bwd(x0.cpu().numpy(), S, cpu(ws), dout.cpu().numpy(),
                                         cpu(gs), cpu(bs))
    twin = [torch.from_numpy(a) for a in [out_t] + dW_t + dg_t + db_t]

    def grads_of(params):
        return [p.grad.detach().float().cpu().view(p.shape[0], -1).squeeze(-1) if p.dim() > 1
                else p.grad.detach().float().cpu() for p in params]

    # fused HIP path
    for p in sa.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = sa_fused.sa_mlp_pool(sa.mlp_module, x0, S)
    (out.float() * dout).sum().backward()
    params = [l.conv.weight for l in layers] + [l.bn.bn.weight for l in layers] + \
        [l.bn.bn.bias for l in layers]
    fused = [out.detach().float().cpu()] + grads_of(params)
    # PyTorch's own bf16 autocast of the same layers (the reference modules' ops)
    wt = [w.clone().requires_grad_() for w in ws]
    gt = [t.clone().requires_grad_() for t in gs]
    bt = [t.clone().requires_grad_() for t in bs]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        x = x0.T.reshape(1, 3, P, S)
        for w, gm, bb in zip(wt, gt, bt):
            x = F.relu(F.batch_norm(F.conv2d(x, w[:, :, None, None]), None, None, gm, bb,
                                    training=True))
        ref = F.max_pool2d(x, kernel_size=[1, S]).squeeze(-1)[0].T
    (ref.float() * dout).sum().backward()
    torchbf = [ref.detach().float().cpu()] + [t.grad.float().cpu() for t in wt + gt + bt]
    names = ["out"] + [f"dW{i}" for i in range(3)] + [f"dgamma{i}" for i in range(3)] + \
        [f"dbeta{i}" for i in range(3)]
    for n, f, tb, tw in zip(names, fused, torchbf, twin):
        ef, et = _rel(f, tw.view(f.shape)), _rel(tb, tw.view(f.shape))
        assert ef <= max(2.0 * et, 3e-2), (n, ef, et)
