"""The functional RegionCLIP restatement (tests/regionclip_ref.py: weight tensors by their
upstream key names, F.conv2d / F.multi_head_attention_forward) against the module
formulation of the same weights (regionclip.ModifiedResNet.forward / layer4 / attnpool) on
the CPU in float64, at a reduced width: the GPU parity test (tests/test_regionclip_gpu.py)
compares the product's fused path with the functional restatement, so this pins the
restatement itself.  Parity vs upstream RegionCLIP: unpinned (no weights offline)."""
import numpy as np
import torch

from helpers import ov3d  # noqa: F401


def test_functional_restatement_equals_module_formulation():
    import regionclip_ref as R
    from ov3d_amd import regionclip as rc
    torch.manual_seed(0)
    m = rc.RegionCLIP(layers=(1, 2, 2, 2), width=16, heads=4, output_dim=32,
                      compute_dtype=torch.float32)
    rc.init_synthetic_(m.backbone, seed=3)
    m = m.double()
    sd = {k: v for k, v in m.state_dict().items()}
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.uniform(-2, 2, (2, 3, 48, 64)))
    with torch.no_grad():
        want = m.backbone(x)["res4"]
        got = R.stem(sd, "backbone.", x)
        for name in ("layer1", "layer2", "layer3"):
            got = R.res_layer(sd, "backbone." + name, got)
        torch.testing.assert_close(got, want, rtol=1e-10, atol=1e-10)
        r = torch.from_numpy(rng.uniform(-1, 1, (5, 16 * 4 * 4, 18, 18)))
        want = m.backbone.attnpool(m.backbone.layer4(r))
        got = R.attnpool(sd, "backbone.attnpool.", R.res_layer(sd, "backbone.layer4", r), 4)
        torch.testing.assert_close(got, want, rtol=1e-10, atol=1e-10)
