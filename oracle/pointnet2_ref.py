"""TEST INFRASTRUCTURE ONLY — CPU restatement of the un-vendored
``third_party.pointnet2`` Python API that ``models/model_3detr.py:8-9`` imports.

Index kernels (FPS, ball query) call the C oracle; gathers/grouping use plain
``torch`` indexing so autograd works; the SharedMLP follows the upstream
``pytorch_utils`` layout so state-dict keys match
(``mlp_module.layer{i}.conv.weight``, ``mlp_module.layer{i}.bn.bn.*``).
Semantics: SURVEY.md Appendix A.1-A.4 (PARITY UNPINNED by the reference,
which vendors neither the sources nor fixtures of this package).

Uses: (1) makes the reference ``Model3DETR`` importable in this container to
produce golden fixtures; (2) the CPU baseline of ``bench.py``.
"""
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import oracle as _o


# ----------------------------------------------------------- pointnet2_utils
def furthest_point_sample(xyz, npoint):
    idx = _o.fps(xyz.detach().cpu().numpy(), int(npoint))
    return torch.from_numpy(idx).to(xyz.device)


def gather_operation(features, idx):
    """(B,C,N), (B,npoint) int -> (B,C,npoint)"""
    B, C, _ = features.shape
    idx = idx.long()
    return torch.gather(features, 2, idx[:, None, :].expand(B, C, idx.shape[1]))


def ball_query(radius, nsample, xyz, new_xyz):
    idx = _o.ball_query(xyz.detach().cpu().numpy(), new_xyz.detach().cpu().numpy(), float(radius),
                        int(nsample))
    return torch.from_numpy(idx).to(xyz.device)


def grouping_operation(features, idx):
    """(B,C,N), (B,M,S) int -> (B,C,M,S)"""
    B, C, N = features.shape
    _, M, S = idx.shape
    flat = idx.long().reshape(B, 1, M * S).expand(B, C, M * S)
    return torch.gather(features, 2, flat).reshape(B, C, M, S)


class QueryAndGroup(nn.Module):
    def __init__(self, radius, nsample, use_xyz=True, ret_grouped_xyz=False, normalize_xyz=False,
                 sample_uniformly=False, ret_unique_cnt=False):
        super().__init__()
        self.radius, self.nsample, self.use_xyz = radius, nsample, use_xyz
        self.ret_grouped_xyz = ret_grouped_xyz
        self.normalize_xyz = normalize_xyz
        assert not sample_uniformly and not ret_unique_cnt

    def forward(self, xyz, new_xyz, features=None):
        idx = ball_query(self.radius, self.nsample, xyz, new_xyz)
        xyz_trans = xyz.transpose(1, 2).contiguous()
        grouped_xyz = grouping_operation(xyz_trans, idx)
        grouped_xyz = grouped_xyz - new_xyz.transpose(1, 2).unsqueeze(-1)
        if self.normalize_xyz:
            grouped_xyz = grouped_xyz / self.radius
        if features is not None:
            grouped_features = grouping_operation(features, idx)
            new_features = torch.cat([grouped_xyz, grouped_features], dim=1) if self.use_xyz \
                else grouped_features
        else:
            new_features = grouped_xyz
        if self.ret_grouped_xyz:
            return new_features, grouped_xyz
        return new_features

    def rows(self, xyz, new_xyz, features=None):
        """channels-last view (B, npoint, nsample, 3+C) (product call surface)"""
        out = self.forward(xyz, new_xyz, features)
        out = out[0] if isinstance(out, tuple) else out
        return out.permute(0, 2, 3, 1).contiguous()


# ------------------------------------------------------------- pytorch_utils
class _BN2d(nn.Sequential):
    def __init__(self, c):
        super().__init__()
        self.add_module("bn", nn.BatchNorm2d(c))
        nn.init.constant_(self[0].weight, 1.0)
        nn.init.constant_(self[0].bias, 0)


class _Conv2dBlock(nn.Sequential):
    def __init__(self, cin, cout, bn=True):
        super().__init__()
        conv = nn.Conv2d(cin, cout, kernel_size=(1, 1), bias=not bn)
        nn.init.kaiming_normal_(conv.weight)
        if not bn:
            nn.init.constant_(conv.bias, 0)
        self.add_module("conv", conv)
        if bn:
            self.add_module("bn", _BN2d(cout))
        self.add_module("activation", nn.ReLU(inplace=True))


class SharedMLP(nn.Sequential):
    def __init__(self, args, *, bn=False):
        super().__init__()
        for i in range(len(args) - 1):
            self.add_module(f"layer{i}", _Conv2dBlock(args[i], args[i + 1], bn=bn))


# --------------------------------------------------------- pointnet2_modules
class PointnetSAModuleVotes(nn.Module):
    def __init__(self, *, mlp, npoint=None, radius=None, nsample=None, bn=True, use_xyz=True,
                 pooling="max", sigma=None, normalize_xyz=False, sample_uniformly=False,
                 ret_unique_cnt=False):
        super().__init__()
        assert npoint is not None and pooling == "max"
        self.npoint, self.radius, self.nsample, self.pooling = npoint, radius, nsample, pooling
        self.use_xyz = use_xyz
        self.normalize_xyz = normalize_xyz
        self.grouper = QueryAndGroup(radius, nsample, use_xyz=use_xyz, ret_grouped_xyz=True,
                                     normalize_xyz=normalize_xyz)
        mlp_spec = mlp
        if use_xyz and len(mlp_spec) > 0:
            mlp_spec[0] += 3
        self.mlp_module = SharedMLP(mlp_spec, bn=bn)

    def forward(self, xyz, features=None, inds=None):
        xyz_flipped = xyz.transpose(1, 2).contiguous()
        if inds is None:
            inds = furthest_point_sample(xyz, self.npoint)
        new_xyz = gather_operation(xyz_flipped, inds).transpose(1, 2).contiguous()
        grouped_features, _ = self.grouper(xyz, new_xyz, features)
        new_features = self.mlp_module(grouped_features)
        new_features = F.max_pool2d(new_features, kernel_size=[1, new_features.size(3)])
        return new_xyz, new_features.squeeze(-1), inds


def install_as_third_party():
    """Register this module as ``third_party.pointnet2.*`` (for importing the reference)."""
    tp = types.ModuleType("third_party")
    tp.__path__ = []
    pn = types.ModuleType("third_party.pointnet2")
    pn.__path__ = []
    me = sys.modules[__name__]
    sys.modules["third_party"] = tp
    sys.modules["third_party.pointnet2"] = pn
    for sub in ("pointnet2_utils", "pointnet2_modules", "pytorch_utils"):
        sys.modules["third_party.pointnet2." + sub] = me
        setattr(pn, sub, me)
    tp.pointnet2 = pn
    return me


__all__ = ["furthest_point_sample", "gather_operation", "ball_query", "grouping_operation",
           "QueryAndGroup", "SharedMLP", "PointnetSAModuleVotes", "install_as_third_party", "np"]
