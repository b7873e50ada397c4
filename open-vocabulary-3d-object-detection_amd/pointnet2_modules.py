"""Drop-in for ``third_party.pointnet2.pointnet2_modules`` / ``pytorch_utils``:
``PointnetSAModuleVotes`` (built at models/model_3detr.py:353-362 and
385-391 of the reference) on the ov3d HIP kernels.

State-dict layout follows upstream ``pytorch_utils.SharedMLP`` so reference
checkpoints load: ``mlp_module.layer{i}.conv.weight``,
``mlp_module.layer{i}.bn.bn.{weight,bias,running_mean,running_var}``.
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as nat
from . import pointnet2_utils as pu
from . import sa_fused
from .gemm import rows_linear


def batch_norm_rows(bn, x):
    """BatchNorm over the rows of a channels-last (R, C) tensor with the parameters /
    running statistics of `bn` (BatchNorm1d/2d or SyncBatchNorm): statistics over R,
    which are exactly the (N, H, W) positions of the channel-first module."""
    if isinstance(bn, nn.SyncBatchNorm):
        from . import dist
        if bn.training and not x.is_cuda and dist.is_distributed():
            return dist.sync_batch_norm_rows(bn, x)   # torch's SyncBatchNorm is GPU-only
        return bn(x)
    training = bn.training or bn.running_mean is None
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    return F.batch_norm(x, bn.running_mean if not bn.training or bn.track_running_stats else None,
                        bn.running_var if not bn.training or bn.track_running_stats else None,
                        bn.weight, bn.bias, training, bn.momentum if bn.momentum is not None else 0.0,
                        bn.eps)


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

    def rows(self, x, pool=None):
        """The 1x1-conv stack on channels-last rows (R, Cin) -> (R, Cout): each layer is one
        GEMM + BN over rows + ReLU; no NCHW<->NHWC transposes.  Training under bf16 autocast:
        BN + ReLU as one HIP row pass each way (heads.bn_relu_rows; the ScanNet SA with colour
        and the masked encoder's interim SA, which the fused 3-channel kernels of sa_fused.py
        do not take).  pool=S: -> (y, pooled); pooled: the last layer's BN + ReLU went straight
        into the max over each S rows (heads.bn_relu_pool_rows), y is (R / S, Cout).  A BN + ReLU
        followed by a 256 x 256 product over >= 2^17 rows runs inside it
        (heads.bn_relu_linear_rows)."""
        from . import heads
        from .gemm import rows_linear_padk
        layers = list(self)
        last = len(layers) - 1
        pend = None   # a layer output whose BN + ReLU runs inside this layer's product
        for i, layer in enumerate(layers):
            w = layer.conv.weight
            w2 = w.view(w.shape[0], w.shape[1])
            if pend is not None:
                x = heads.bn_relu_linear_rows(x, pend, w2)
                pend = None
            elif x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] > w2.shape[1]:
                x = rows_linear_padk(x, w2, layer.conv.bias)   # zero-padded bf16 group rows
            else:
                x = rows_linear(x, w2, layer.conv.bias)
            if hasattr(layer, "bn"):
                bn = layer.bn.bn
                if pool is not None and i == last and heads.bn_relu_pool_ok(x, bn, layer.activation,
                                                                              pool):
                    return heads.bn_relu_pool_rows(x, bn, pool), True
                if i < last:   # the next 256 x 256 product applies this BN + ReLU as it loads
                    nxt = layers[i + 1].conv
                    if heads.bn_relu_linear_ok(x, bn, layer.activation, nxt.weight, nxt.bias):
                        pend = bn
                        continue
                if heads.bn_relu_rows_ok(x, bn, layer.activation, None):
                    x = heads.bn_relu_rows(x, bn)
                    continue
                x = batch_norm_rows(bn, x)
            x = torch.relu(x)
        return (x, False) if pool is not None else x


def _nbr_max_ok(y, S):
    return (y.is_cuda and y.dtype == torch.bfloat16 and y.dim() == 2 and y.shape[1] % 8 == 0
            and 0 < S <= 256 and y.shape[0] % S == 0)


class _NbrMax(torch.autograd.Function):
    """max over the S neighbour rows of each centroid (bf16 (P*S, C) -> (P, C)) on
    csrc/pool.hip: the arg row is the first maximum (max_pool2d's window order) and the
    backward writes the dense row gradient in one pass (no scatter, no zero fill)."""

    @staticmethod
    def forward(ctx, y, S):
        y = y.contiguous()
        R, C = y.shape
        P = R // S
        out = torch.empty((P, C), dtype=y.dtype, device=y.device)
        arg = torch.empty((P, C), dtype=torch.uint8, device=y.device)
        nat.call("ov3d_nbr_max_fwd", y, P, S, C, out, arg, like=y)
        ctx.save_for_backward(arg)
        ctx.S = S
        return out

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        P, C = arg.shape
        S = ctx.S
        g = g.to(torch.bfloat16).contiguous()
        dy = torch.empty((P * S, C), dtype=torch.bfloat16, device=g.device)
        nat.call("ov3d_nbr_max_bwd", g, arg, P, S, C, dy, like=g)
        return dy, None


# fused SA output stored sequence-first (the pool kernel's seq_m); False: (B, M, C) rows
SEQ_FIRST_OUT = True


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

    def forward(self, xyz, features=None, inds=None, new_xyz=None, ball=None, inverse=None):
        """inds / new_xyz / ball: the FPS indices, sampled points and ball-query indices
        computed ahead of time from the same points (Model3DETR.sampling_plan); identical
        results."""
        xyz = xyz.detach()
        if inds is None:
            inds, new_xyz = pu.furthest_point_sample_gather(xyz, self.npoint)
        else:
            if inds.shape[1] != self.npoint:
                raise ValueError("inds must have npoint columns")
            if new_xyz is None:
                new_xyz = pu.gather_operation(xyz.transpose(1, 2).contiguous(), inds).transpose(1, 2)
                new_xyz = new_xyz.contiguous()
        return new_xyz, self._mlp_pool(xyz, new_xyz, features, ball, inverse).transpose(1, 2), inds

    def _mlp_pool(self, xyz, new_xyz, features, ball=None, inverse=None):
        """grouped rows -> SharedMLP -> max over nsample: (B, npoint, Cout)."""
        # bf16 rows with an aligned width for the GEMM path under bf16 autocast (the masked
        # encoder's interim SA: 256 features + xyz -> 264 columns); fp32 rows otherwise and for
        # the fused SA kernels' 3- / 6-channel first layers
        bf16_rows = (features is not None and features.shape[1] > 3 and xyz.is_cuda
                     and torch.is_autocast_enabled("cuda")
                     and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        kw = {"bf16_rows": True} if bf16_rows else {}
        g = self.grouper.rows(xyz, new_xyz, features, **kw) if ball is None else \
            self.grouper.rows(xyz, new_xyz, features, idx=ball, inverse=inverse, **kw)   # (B,M,S,3+C)
        B, M, S, C = g.shape
        rows = g.view(B * M * S, C)
        if self.training and sa_fused.supported(self.mlp_module, rows, S):
            # training under bf16 autocast: fused MFMA kernels (sa_fused.py); the pool kernel
            # writes the rows sequence-first (M, B, C), the encoder's input layout, and this
            # returns the (B, M, C) view of them (same values, no transpose pass either way)
            if SEQ_FIRST_OUT:
                return sa_fused.sa_mlp_pool(self.mlp_module, rows, S, seq_m=M).view(
                    M, B, -1).transpose(0, 1)
            return sa_fused.sa_mlp_pool(self.mlp_module, rows, S).view(B, M, -1)
        y, pooled = self.mlp_module.rows(rows, pool=S)
        if pooled:   # the last BN + ReLU fused into the pool (heads.bn_relu_pool_rows)
            return y.view(B, M, -1)
        # == F.max_pool2d(kernel [1, nsample]) of the reference
        if _nbr_max_ok(y, S):
            return _NbrMax.apply(y, S).view(B, M, -1)
        return y.view(B, M, S, -1).max(dim=2).values


__all__ = ["PointnetSAModuleVotes", "SharedMLP"]
