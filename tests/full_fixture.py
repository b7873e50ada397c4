"""Shared runner for the full-shape float64 reference fixtures (model_*_full.npz, made by
tests/golden/make_golden.py): builds the product model with the fixture's deterministic
weights (tests/golden/det_init.py), runs forward + criterion + backward with the
reference's recorded matcher assignments, and compares outputs, the 56 losses and every
parameter gradient (element-wise for the stored ones, norm + probe projection for all).

The bars (DESIGN.md "Oracle and parity"):
  fp32  outputs / losses / gradients <= 1e-3 relative to the float64 reference
  bf16  (autocast, the benchmarked kernels) see BF16_TOL
"""
import contextlib

import numpy as np
import torch

from helpers import batch_from_fixture, fixture, fixture_args, fixture_prefix, pin_matcher
import det_init  # noqa: E402  (tests/golden, on the path through helpers)
from fake_clip import FakeRegionCLIP  # noqa: E402

CASES = [("model_sun_full.npz", "sunrgbd"), ("model_scannet_full.npz", "scannet")]

FP32_TOL = 1e-3
GRAD_FLOOR = 1e-6        # as make_golden.py: below 1e-6 x the total norm a gradient is zero
# bf16 autocast: GEMM / attention inputs rounded to 8 mantissa bits (2^-9 = 2e-3 relative per
# element); through 3 encoder + 8 decoder layers the outputs move by a few 1e-2 of their max
BF16_TOL = dict(out=5e-2, loss=3e-2, grad_norm=5e-2, grad=1e-1, grad_proj=1e-1)
BF16_GRAD_FLOOR = 1e-3   # bf16: gradients below this fraction of the total norm count as zero


def build(fx, device, dataset):
    from ov3d_amd.dataset_config import CONFIGS
    from ov3d_amd.model_3detr import build_3detr
    args = fixture_args(fx)
    cfg = CONFIGS[dataset]()
    model, _ = build_3detr(args, cfg, text_embedding=torch.from_numpy(fx["text"]))
    filled = det_init.fill_(model, int(fx["seed"]))
    assert filled == sorted(str(x) for x in fx["filled"]), "state-dict keys differ from the reference"
    return model.to(device).train(), cfg, args


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


@contextlib.contextmanager
def float64_host():
    """Tensor.float() keeps float64 tensors in float64 for the duration: the product's host
    code then runs its whole algorithm in float64 (its .float() casts exist to lift bf16
    autocast outputs).  CPU parity runs only (the index ops come from the C oracle)."""
    orig = torch.Tensor.float

    def f(self, *a, **k):
        return self if self.dtype == torch.float64 else orig(self, *a, **k)
    torch.Tensor.float = f
    try:
        yield
    finally:
        torch.Tensor.float = orig


@contextlib.contextmanager
def torch_bf16_path():
    """The same model under bf16 autocast with every HIP dense / fused kernel switched off:
    PyTorch's own autocast execution (hipBLASLt GEMMs, SDPA attention, torch BatchNorm /
    LayerNorm / ReLU, torch weight gradients).  The precision baseline the HIP bf16 kernels
    are measured against (they must be no less accurate against the float64 reference)."""
    from ov3d_amd import attention, gemm, heads, resnorm, sa_fused, transformer
    patches = [(sa_fused, "supported", lambda *a, **k: False),
               (heads, "supported", lambda *a, **k: False),
               (heads, "bn_relu_rows_ok", lambda *a, **k: False),
               (resnorm, "supported", lambda *a, **k: False),
               (attention, "supported", lambda *a, **k: False),
               (transformer, "memory_kv_ok", lambda *a, **k: False),
               (gemm, "_fused_ok", lambda *a, **k: False),
               (gemm, "ROWS_GEMM_MAX_M", 0)]
    saved = [(m, n, getattr(m, n)) for m, n, _ in patches]
    for m, n, v in patches:
        setattr(m, n, v)
    try:
        yield
    finally:
        for m, n, v in saved:
            setattr(m, n, v)


def step(name, dataset, device, amp=None):
    """one training step (forward, criterion, backward) on the fixture -> (loss, loss dict,
    {parameter: gradient})"""
    from ov3d_amd.criterion import build_criterion
    fx = fixture(name)
    model, cfg, args = build(fx, device, dataset)
    batch = batch_from_fixture(fx, device)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    with torch.autocast("cuda", dtype=amp or torch.float32, enabled=amp is not None):
        out = model(inputs)
    crit = pin_matcher(build_criterion(args, cfg).to(device), fx, device)
    loss, ld = crit(out, dict(batch), clip=FakeRegionCLIP())
    loss.backward()
    return loss.detach(), {k: v.detach() for k, v in ld.items()}, \
        {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


def run(name, dataset, device, amp=None, f64=False, grad_floor=None):
    """-> dict of error reports (max relative error per group, worst key)"""
    from ov3d_amd.criterion import build_criterion
    fx = fixture(name)
    model, cfg, args = build(fx, device, dataset)
    batch = batch_from_fixture(fx, device)
    ctx = contextlib.nullcontext()
    if f64:
        model = model.double()
        batch = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
        ctx = float64_host()
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    with ctx:
        if amp is not None:
            with torch.autocast("cuda", dtype=amp):
                out = model(inputs)
        else:
            out = model(inputs)
        crit = pin_matcher(build_criterion(args, cfg).to(device), fx, device)
        loss, ld = crit(out, dict(batch), clip=FakeRegionCLIP())
        loss.backward()
    rep = {"out": [], "out_l2": [], "loss": [], "grad": [], "grad_norm": [], "grad_proj": []}
    layers = [out["outputs"]] + out["aux_outputs"]
    for li, lay in enumerate(layers):
        for k, ref in fixture_prefix(fx, f"out/{li}/").items():
            got = lay[k].detach().double().cpu().numpy()
            rep["out"].append((rel(got, ref), f"{li}/{k}"))
            rep["out_l2"].append((float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)),
                                  f"{li}/{k}"))
    ref_ld = fixture_prefix(fx, "ld/")
    assert set(ld) == set(ref_ld), set(ld) ^ set(ref_ld)
    for k, v in ref_ld.items():
        rep["loss"].append((abs(ld[k].item() - float(v)) / max(abs(float(v)), 1e-3), k))
    rep["loss"].append((abs(loss.item() - float(fx["loss"])) / abs(float(fx["loss"])), "loss"))
    named = dict(model.named_parameters())
    norms = fixture_prefix(fx, "gradnorm/")
    assert set(norms) == {n for n, p in named.items() if p.grad is not None}
    floor = (GRAD_FLOOR if grad_floor is None else grad_floor) * float(fx["gradtotal"])
    for n, gn in norms.items():
        g = named[n].grad.detach().double().cpu().numpy()
        den = max(gn, floor)
        rep["grad_norm"].append((abs(np.linalg.norm(g) - gn) / den, n))
        pr = float((g * det_init.probe(n, g.shape)).sum())
        # the projection on a random unit-variance probe is ~ |g|: relative to the norm
        rep["grad_proj"].append((abs(pr - float(fx["gradproj/" + n])) / den, n))
    for n, ref in fixture_prefix(fx, "grad/").items():
        g = named[n].grad.detach().float().cpu().numpy()
        g = g[: ref.shape[0]] if g.shape != ref.shape else g
        den = max(float(np.linalg.norm(ref)), floor)
        rep["grad"].append((float(np.linalg.norm(g.astype(np.float64) - ref)) / den, n))
    return {k: sorted(v, reverse=True) for k, v in rep.items()}


def worst(rep, k):
    return rep[k][0] if rep[k] else (0.0, None)


REF32_KEY = {"out": "out/", "out_l2": "out/", "loss": "ld/", "grad": "grad/", "grad_norm": "gradnorm/",
             "grad_proj": "gradproj/"}


def fp32_failures(rep, fx, tol=FP32_TOL, slack=2.0):
    """entries above max(tol, slack x the reference's own fp32 error on that entry)"""
    bad = []
    for group, entries in rep.items():
        for err, key in entries:
            r32 = fx.get("ref32err/" + REF32_KEY[group] + key) if key != "loss" else None
            bar = max(tol, slack * float(r32)) if r32 is not None else tol
            if not err <= bar:
                bad.append((group, key, err, bar))
    return bad
