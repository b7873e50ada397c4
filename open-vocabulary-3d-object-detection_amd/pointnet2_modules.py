"""Drop-in for ``third_party.pointnet2.pointnet2_modules`` / ``pytorch_utils``:
``PointnetSAModuleVotes`` (built at models/model_3detr.py:353-362 and
385-391 of the reference) on the ov3d HIP kernels.

State-dict layout follows upstream ``pytorch_utils.SharedMLP`` so reference
checkpoints load: ``mlp_module.layer{i}.conv.weight``,
``mlp_module.layer{i}.bn.bn.{weight,bias,running_mean,running_var}``.
"""

import torch.nn as nn

from . import pointnet2_utils as pu


class _BNWrap(nn.Sequential):
    """upstream pytorch_utils.BatchNorm2d: a Sequential holding `bn`."""

    def __init__(self, channels):
        super().__init__()
        self.add_module("bn", nn.BatchNorm2d(channels))
        nn.init.ones_(self.bn.weight)
        nn.init.zeros_(self.bn.bias)


class _ConvBNReLU(nn.Sequential):
    """upstream pytorch_utils.Conv2d(bn=True): 1x1 conv (no bias) -> BN -> ReLU."""

    def __init__(self, cin, cout, bn=True):
        super().__init__()
        conv = nn.Conv2d(cin, cout, kernel_size=(1, 1), bias=not bn)
        nn.init.kaiming_normal_(conv.weight)
        if conv.bias is not None:
            nn.init.zeros_(conv.bias)
        self.add_module("conv", conv)
        if bn:
            self.add_module("bn", _BNWrap(cout))
        self.add_module("activation", nn.ReLU(inplace=True))


class SharedMLP(nn.Sequential):
    def __init__(self, args, *, bn=False, activation=None, preact=False, first=False, name=""):
        super().__init__()
        if preact:
            raise NotImplementedError("pre-activation SharedMLP is not on the reference path")
        for i in range(len(args) - 1):
            self.add_module(f"{name}layer{i}", _ConvBNReLU(args[i], args[i + 1], bn=bn))


class PointnetSAModuleVotes(nn.Module):
    """Set abstraction: FPS -> ball query -> group (+xyz, /radius) -> SharedMLP -> max over nsample."""

    def __init__(self, *, mlp, npoint=None, radius=None, nsample=None, bn=True, use_xyz=True,
                 pooling="max", sigma=None, normalize_xyz=False, sample_uniformly=False,
                 ret_unique_cnt=False):
        super().__init__()
        if npoint is None or pooling != "max":
            raise NotImplementedError("only the FPS + max-pool form is on the reference path")
        self.npoint, self.radius, self.nsample = npoint, radius, nsample
        self.pooling = pooling
        self.use_xyz = use_xyz
        self.normalize_xyz = normalize_xyz
        self.grouper = pu.QueryAndGroup(radius, nsample, use_xyz=use_xyz, ret_grouped_xyz=True,
                                        normalize_xyz=normalize_xyz)
        mlp_spec = mlp
        if use_xyz and len(mlp_spec) > 0:
            mlp_spec[0] += 3  # upstream mutates the caller's list (reference relies on it)
        self.mlp_module = SharedMLP(mlp_spec, bn=bn)

    def forward(self, xyz, features=None, inds=None):
        xyz = xyz.detach()
        if inds is None:
            inds, new_xyz = pu.furthest_point_sample_gather(xyz, self.npoint)
        else:
            if inds.shape[1] != self.npoint:
                raise ValueError("inds must have npoint columns")
            new_xyz = pu.gather_operation(xyz.transpose(1, 2).contiguous(), inds).transpose(1, 2)
            new_xyz = new_xyz.contiguous()
        grouped, _ = self.grouper(xyz, new_xyz, features)
        new_features = self.mlp_module(grouped)
        # max over nsample (== F.max_pool2d(kernel [1, nsample]) of the reference); amax runs as one
        # reduction instead of PyTorch's generic pooling kernel
        return new_xyz, new_features.amax(dim=3), inds


__all__ = ["PointnetSAModuleVotes", "SharedMLP"]
