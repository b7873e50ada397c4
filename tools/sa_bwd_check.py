"""Fused SA backward (csrc/sa_bwd.hip) vs the three-pass path on one SA module, per-parameter
relative gradient error (tests/test_sa_fused_gpu.py's last-layer check, printed instead of
asserted; run under OV3D_SA_* environment variants to localise a difference)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def main():
    ov3d_import.load()
    from ov3d_amd import sa_fused, synthetic
    from ov3d_amd.pointnet2_modules import PointnetSAModuleVotes
    cuda = torch.device("cuda")
    feat = int(os.environ.get("SA_CHECK_FEATURES", "0"))   # 3: colour input (stored y1 rows)
    for nsample in (64, 32):
        torch.manual_seed(3)
        sa = PointnetSAModuleVotes(radius=0.2, nsample=nsample, npoint=2048, mlp=[feat, 64, 128, 256],
                                   normalize_xyz=True).to(cuda).train()
        with torch.no_grad():
            for layer in sa.mlp_module:
                bn = layer.bn.bn
                bn.weight.copy_(torch.randn_like(bn.weight) * 0.5 + 0.6)
                bn.bias.copy_(torch.randn_like(bn.bias) * 0.2)
        xyz = synthetic.make_batch(2, seed=9, device=cuda)["point_clouds"]
        gw = torch.randn(2, 256, 2048, device=cuda)
        res = {}
        for fused in (True, False, True):
            sa_fused.FUSED_BWD = fused
            twin = copy.deepcopy(sa)
            feats = torch.rand(xyz.shape[0], feat, xyz.shape[1], device=cuda,
                               generator=torch.Generator(device=cuda).manual_seed(5)) if feat else None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                _, f, _ = twin(xyz[..., :3].contiguous(), feats)
            (f.float() * gw).sum().backward()
            res.setdefault(fused, []).append({n: p.grad.clone() for n, p in twin.named_parameters()})
        sa_fused.FUSED_BWD = True
        ref = res[False][0]
        for n in ref:
            e = [((r[n] - ref[n]).norm() / ref[n].norm()).item() for r in res[True]]
            rep = ((res[True][0][n] - res[True][1][n]).norm() / ref[n].norm()).item()
            print(f"S={nsample} {n:36s} err {e[0]:.2e} {e[1]:.2e}  fused run-to-run {rep:.1e}")


if __name__ == "__main__":
    main()
