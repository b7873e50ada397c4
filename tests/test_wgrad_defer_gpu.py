"""Deferred, grouped weight gradients (gemm.DEFER_WGRAD, csrc/wgrad.hip ov3d_wgrad_group):
the full BASELINE-size training step gives the same parameter gradients with the deferral
on and off, including the in_proj row blocks.  The grouped launch uses 256 x 256 tiles and
1024-row splits, the immediate one 128 x 128 tiles and its own split count: every row chunk
is accumulated in the same order, only the fp32 sum of the split partials is grouped
differently (relative error <= 1e-4: the bias column sums over 16384 rows cancel)."""
import pytest
import torch

from helpers import ov3d  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("single_min_r", [1 << 17, 1 << 13])
def test_deferred_weight_grads_equal_immediate(cuda, monkeypatch, single_min_r):
    """single_min_r = 2^13: the R = 16384 problems leave the grouped launch for their own
    ov3d_wgrad launches (gemm.WGRAD_SINGLE_MIN_R, the path of the long SA problems)"""
    import ov3d_amd
    from bench import default_args
    from ov3d_amd import gemm, synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    monkeypatch.setattr(gemm, "WGRAD_SINGLE_MIN_R", single_min_r)
    args = default_args(enc_dropout=0.0, dec_dropout=0.0, mlp_dropout=0.0)
    cfg = SunrgbdDatasetConfig()
    torch.manual_seed(0)
    model, _ = ov3d_amd.build_model(args, cfg, text_embedding=synthetic.text_embedding())
    model = model.to(cuda).train()
    crit = ov3d_amd.build_criterion(args, cfg).to(cuda)
    batch = synthetic.make_batch(4, seed=2, num_points=20000, device=cuda)
    inputs = {k: batch[k] for k in ("point_clouds", "point_cloud_dims_min", "point_cloud_dims_max")}
    grads = {}
    for defer in (False, True):
        gemm.DEFER_WGRAD = defer
        try:
            model.zero_grad(set_to_none=True)
            torch.manual_seed(5)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(inputs)
            loss, _ = crit(out, dict(batch))
            loss.backward()
            assert not gemm._PENDING
            grads[defer] = {n: p.grad.clone() for n, p in model.named_parameters()
                            if p.grad is not None}
        finally:
            gemm.DEFER_WGRAD = False
    assert set(grads[True]) == set(grads[False])
    for n in grads[False]:
        a, b = grads[True][n], grads[False][n]
        err = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert err <= 1e-4, (n, err)
