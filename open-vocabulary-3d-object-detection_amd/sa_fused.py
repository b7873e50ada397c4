"""Fused training path of the set-abstraction MLP + max-pool (ov3d_sa_* kernels).

Replaces, for training under bf16 autocast, the SharedMLP([3, C1, C2, C3]) +
F.max_pool2d([1, nsample]) of PointnetSAModuleVotes (reference
models/model_3detr.py:353-362; pointnet2 pytorch_utils.SharedMLP: 1x1 conv
without bias -> BatchNorm (batch statistics) -> ReLU per layer).

Forward (csrc/sa_mlp.hip):
  layer 1  ov3d_sa_l1_fwd      x0 (R,3) f32 -> BN partials (y1 = bf16(x0 W1^T) is recomputed
                               by its consumers from x0, never stored, when the fused backward
                               runs; otherwise stored)
  layer 2  ov3d_sa_layer_fwd   relu(bn1(y1)) -> MFMA W2 -> y2 bf16 + partials (z1 kept);
           ov3d_sa_layer_fwd_x0 the same with y1 recomputed from x0 in the prologue
  layer 3  ov3d_sa_layer_pool_fwd  relu(bn2(y2)) -> MFMA W3 -> per-centroid max/min of
           y3 (never stored) + partials (z2 kept);  ov3d_sa_pool_fwd applies bn3 + ReLU
           to the max (or min when gamma*invstd < 0: relu(a*y+b) is monotone in y).
Backward: the pooled gradient only reaches one row per (centroid, channel); the BN
backward reductions over all R rows therefore come from P*C3 values
(ov3d_sa_pool_bwd), and dy3 = cA*g + cB*y3 + cC is produced while recomputing y3
(ov3d_sa_layer_dy).  dz2 = dy3 W3 and the weight gradients are hipBLASLt GEMMs;
the layer-2/1 ReLU + BN backward are two row passes each (ov3d_bn_relu_bwd), the
layer-1 weight gradient is reduced against x0 inside the last pass.

BatchNorm semantics are torch's training batch_norm: biased variance to normalise,
unbiased for running_var, momentum update, num_batches_tracked += 1; SyncBatchNorm
all-reduces the per-channel sums (one all-reduce per layer, forward and backward).
"""
import os

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.autograd import Function

from . import _native as nat
from .gemm import cast_param, weight_grad

NPARTS_LAYER = 1024    # MFMA workgroups over 64-row tiles (more than resident: no tail when
                       # the side-stream FPS holds a few CUs; tools/sa_layer_probe.py)
NPARTS_ROWS = 1024     # row-pass workgroups
NPARTS_POOL = 1024    # pooled-gradient pass: 16 centroids per thread at P = 16384 (was 64: latency-bound)
# last layer's backward in one pass (csrc/sa_bwd.hip): one persistent workgroup per CU
FUSED_BWD = os.environ.get("OV3D_SA_FUSED_BWD", "1") != "0"
NWG_DY_FUSED = int(os.environ.get("OV3D_SA_DY_NWG", "256"))
# the layer-2 backward's workgroups (one 4-wave workgroup per CU)
NWG_DY2 = int(os.environ.get("OV3D_SA_DY2_NWG", "256"))
# layer 3's pooling tracks one extreme per channel, chosen by the sign of its BN weight
# (OV3D_SA_POOL_BOTH=1: both, as before round 5)
POOL_ONE_EXTREME = os.environ.get("OV3D_SA_POOL_BOTH", "0") == "0"
FUSED_STATS = os.environ.get("OV3D_SA_FUSED_STATS", "1") != "0"   # + layer 2's BN-bwd stats


def _bn(layer):
    return layer.bn.bn


FORCE_SYNC = os.environ.get("OV3D_FORCE_SYNC_BN", "0") == "1"   # test hook: sync even at world 1


def _sync_group(bn):
    """the process group a SyncBatchNorm's statistics are all-reduced over (None: local)"""
    if isinstance(bn, nn.SyncBatchNorm) and dist.is_available() and dist.is_initialized() \
            and (FORCE_SYNC or dist.get_world_size(bn.process_group) > 1):
        return bn.process_group if bn.process_group is not None else dist.group.WORLD
    return None


def supported(mlp, x0, S):
    """True when the fused path applies (else the caller runs the unfused rows path)."""
    if not (x0.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    layers = list(mlp)
    # first-layer input: grouped xyz (3), or xyz + colour (6: ScanNet --use_color)
    if len(layers) != 3 or x0.requires_grad or x0.dim() != 2 or x0.shape[1] not in (3, 6):
        return False
    if S not in (32, 64) or x0.shape[0] % 64:
        return False
    dims = [x0.shape[1]]
    for l in layers:
        if not hasattr(l, "bn") or l.conv.bias is not None:
            return False
        bn = _bn(l)
        if not bn.training or not bn.track_running_stats or bn.momentum is None or not bn.affine:
            return False
        dims.append(l.conv.weight.shape[0])
    c1, c2, c3 = dims[1:]
    lib = nat.load()
    return (256 % c1 == 0 and 256 % c3 == 0 and lib.ov3d_sa_layer_supported(c1, c2) == 1
            and lib.ov3d_sa_layer_supported(c2, c3) == 1
            and all(c % 8 == 0 and 256 % (c // 8) == 0 for c in (c1, c2)))


def _colsum(part):
    """(nparts, ...) f32 partials -> their sum over dim 0 (ov3d_colsum_f32, fixed order)"""
    out = torch.empty(part.shape[1:], dtype=torch.float32, device=part.device)
    nat.call("ov3d_colsum_f32", part, part.shape[0], out.numel(), out, like=part)
    return out


def _totals(partials, nparts, width, group):
    tot = torch.empty(width, dtype=torch.float64, device=partials.device)
    nat.call("ov3d_reduce_partials", partials, nparts, width, tot, like=partials)
    if group is not None:
        dist.all_reduce(tot, group=group)
    return tot


def _finalize(tot, count, bn, C):
    dev = tot.device
    mean, invstd, scale, shift = (torch.empty(C, dtype=torch.float32, device=dev) for _ in range(4))
    nbt = bn.num_batches_tracked if (bn.track_running_stats and
                                     bn.num_batches_tracked is not None) else None
    nat.call("ov3d_bn_finalize", tot, float(count), C, bn.weight, bn.bias, float(bn.eps),
             float(bn.momentum), bn.running_mean, bn.running_var, mean, invstd, scale, shift, nbt,
             like=tot)
    return mean, invstd, scale, shift


def bn_affine(parts, nparts, C, group, count, gamma, beta, eps, momentum, rm, rv, nbt):
    """(nparts, 2C) partial (sum, sum of squares) -> mean, invstd, scale, shift (+ running
    statistics, num_batches_tracked): one launch for a single replica, else the totals are
    all-reduced over the SyncBatchNorm group between the reduction and the finalize."""
    dev = parts.device
    mean, invstd, scale, shift = (torch.empty(C, dtype=torch.float32, device=dev) for _ in range(4))
    if group is None:
        nat.call("ov3d_bn_stats_finalize", parts, nparts, C, float(count), gamma, beta, float(eps),
                 float(momentum), rm, rv, mean, invstd, scale, shift, nbt, like=parts)
    else:
        tot = _totals(parts, nparts, 2 * C, group)
        nat.call("ov3d_bn_finalize", tot, float(count), C, gamma, beta, float(eps),
                 float(momentum), rm, rv, mean, invstd, scale, shift, nbt, like=tot)
    return mean, invstd, scale, shift


def bn_bwd_affine(parts, nparts, C, group, count, gamma, mean, invstd):
    """(nparts, 2C) partial (sum dt, sum dt*xhat) -> cA, cB, cC, dgamma, dbeta (one launch
    for a single replica)"""
    if group is not None:
        # SyncBatchNorm: the input-gradient coefficients from the totals over every rank, the
        # weight / bias gradients from this rank's own rows (torch's SyncBatchNorm.backward
        # returns the local sums; the data-parallel gradient mean averages them)
        tot = _totals(parts, nparts, 2 * C, None)
        db, dg = tot[:C].float(), tot[C:].float()
        dist.all_reduce(tot, group=group)
        cA, cB, cC, _, _ = _bwd_coefs(tot, count, gamma, mean, invstd, C, local=False)
        return cA, cB, cC, dg, db
    dev = parts.device
    cA, cB, cC, dg, db = (torch.empty(C, dtype=torch.float32, device=dev) for _ in range(5))
    nat.call("ov3d_bn_bwd_stats_finalize", parts, nparts, C, float(count), gamma, mean, invstd,
             cA, cB, cC, dg, db, like=parts)
    return cA, cB, cC, dg, db


def _bn_stats(parts, nparts, C, group, count, bn):
    nbt = bn.num_batches_tracked if (bn.track_running_stats and
                                     bn.num_batches_tracked is not None) else None
    return bn_affine(parts, nparts, C, group, count, bn.weight, bn.bias, bn.eps, bn.momentum,
                     bn.running_mean, bn.running_var, nbt)


def _bwd_coefs(tot, count, gamma, mean, invstd, C, local=True):
    dev = tot.device
    cA, cB, cC = (torch.empty(C, dtype=torch.float32, device=dev) for _ in range(3))
    dg, db = ((torch.empty(C, dtype=torch.float32, device=dev) for _ in range(2)) if local
              else (None, None))
    nat.call("ov3d_bn_bwd_finalize", tot, float(count), C, gamma, mean, invstd, cA, cB, cC, dg, db,
             like=tot)
    return cA, cB, cC, dg, db


class _SAMLPPool(Function):
    @staticmethod
    def forward(ctx, x0, w1, w2, w3, g1, b1, g2, b2, g3, b3, bns, S, seq_m=0):
        dev = x0.device
        R, cin = x0.shape
        P = R // S
        c1, c2, c3 = w1.shape[0], w2.shape[0], w3.shape[0]
        groups = [_sync_group(bn) for bn in bns]
        world = [dist.get_world_size(g) if g is not None else 1 for g in groups]
        x0 = x0.contiguous()
        bf = torch.bfloat16
        # z1 is kept for the backward only when that does not recompute it (sa_dy2_fused); with
        # the 3 xyz inputs y1 is not stored either: every consumer recomputes it from x0 (12 B
        # per row instead of 128 B: the (R, 64) first-layer output never reaches HBM).  With
        # colour (ScanNet, cin = 6) y1 is stored and sa_dy2_fused reads it.
        fused_bwd2 = FUSED_BWD and c1 == 64 and c2 == 128 and \
            bool(nat.load().ov3d_sa_dy_fused_supported(c2, w3.shape[0]))
        recompute_y1 = fused_bwd2 and cin == 3
        w1f = w1.float().contiguous()
        # layer 1 (statistics only when y1 is recomputed)
        y1 = None if recompute_y1 else torch.empty((R, c1), dtype=bf, device=dev)
        parts = torch.empty((NPARTS_ROWS, 2, c1), dtype=torch.float64, device=dev)
        nat.call("ov3d_sa_l1_fwd_cin", x0, cin, w1f, R, c1, y1, parts, NPARTS_ROWS, like=x0)
        st1 = _bn_stats(parts, NPARTS_ROWS, c1, groups[0], R * world[0], bns[0])
        # layer 2
        w2b = cast_param(w2, bf).contiguous()
        z1 = None if fused_bwd2 else torch.empty((R, c1), dtype=bf, device=dev)
        y2 = torch.empty((R, c2), dtype=bf, device=dev)
        parts = torch.empty((NPARTS_LAYER, 2, c2), dtype=torch.float64, device=dev)
        if recompute_y1:
            nat.call("ov3d_sa_layer_fwd_x0", x0, w1f, st1[2], st1[3], w2b, R, c1, c2, y2, parts,
                     NPARTS_LAYER, like=x0)
        else:
            nat.call("ov3d_sa_layer_fwd", y1, st1[2], st1[3], w2b, R, c1, c2, z1, y2, parts,
                     NPARTS_LAYER, like=x0)
        st2 = _bn_stats(parts, NPARTS_LAYER, c2, groups[1], R * world[1], bns[1])
        # layer 3 + pool (z2 is kept for the backward only when it is not recomputed there)
        w3b = cast_param(w3, bf).contiguous()
        fused_bwd = FUSED_BWD and bool(nat.load().ov3d_sa_dy_fused_supported(c2, c3))
        z2 = None if fused_bwd else torch.empty((R, c2), dtype=bf, device=dev)
        pmax, pmin = (torch.empty((P, c3), dtype=torch.float32, device=dev) for _ in range(2))
        imax, imin = (torch.empty((P, c3), dtype=torch.uint8, device=dev) for _ in range(2))
        parts = torch.empty((NPARTS_LAYER, 2, c3), dtype=torch.float64, device=dev)
        # the BN weight's sign picks each channel's extreme (POOL_ONE_EXTREME; None: both)
        g3s = g3.detach().float().contiguous() if (POOL_ONE_EXTREME and g3 is not None) else None
        nat.call("ov3d_sa_layer_pool_fwd", y2, st2[2], st2[3], w3b, R, c2, c3, S, z2, pmax, pmin,
                 imax, imin, g3s, parts, NPARTS_LAYER, like=x0)
        st3 = _bn_stats(parts, NPARTS_LAYER, c3, groups[2], R * world[2], bns[2])
        out = torch.empty((P, c3), dtype=torch.float32, device=dev)
        ysel = torch.empty((P, c3), dtype=torch.float32, device=dev)
        isel = torch.empty((P, c3), dtype=torch.uint8, device=dev)
        nat.call("ov3d_sa_pool_fwd", pmax, pmin, imax, imin, st3[2], st3[3], P, c3, seq_m, out, ysel,
                 isel, like=x0)
        ctx.save_for_backward(x0, y1, z1, y2, z2, w2b, w3b, g1, g2, g3, ysel, isel, w1f, *st1, *st2,
                              *st3)
        ctx.meta = (R, S, P, c1, c2, c3, groups, world, tuple(w1.shape), fused_bwd, fused_bwd2,
                    seq_m)
        return out

    @staticmethod
    def backward(ctx, dout):
        (x0, y1, z1, y2, z2, w2b, w3b, g1, g2, g3, ysel, isel, w1f,
         m1, i1, a1, s1, m2, i2, a2, s2, m3, i3, a3, s3) = ctx.saved_tensors
        R, S, P, c1, c2, c3, groups, world, w1shape, fused_bwd, fused_bwd2, seq_m = ctx.meta
        dev = x0.device
        bf = torch.bfloat16
        dout = dout.float().contiguous()
        # layer 3: pooled gradient -> BN backward coefficients -> dy3 (recomputed y3)
        gsel = torch.empty((P, c3), dtype=torch.float32, device=dev)
        parts = torch.empty((NPARTS_POOL, 2, c3), dtype=torch.float64, device=dev)
        nat.call("ov3d_sa_pool_bwd", dout, ysel, a3, s3, m3, i3, P, c3, seq_m, gsel, parts, NPARTS_POOL,
                 like=dout)
        cA, cB, cC, dg3, db3 = bn_bwd_affine(parts, NPARTS_POOL, c3, groups[2], R * world[2], g3,
                                             m3, i3)
        parts2 = None
        if fused_bwd:   # dy3 -> dz2 and dW3 inside one pass (csrc/sa_bwd.hip)
            nwg = min(NWG_DY_FUSED, R // 64)
            dz2 = torch.empty((R, c2), dtype=bf, device=dev)
            part = torch.empty((nwg, c3, c2), dtype=torch.float32, device=dev)
            # + layer 2's ReLU + BN backward partials (the stats pass over dz2 and y2)
            parts2 = torch.empty((nwg, 2, c2), dtype=torch.float64, device=dev) \
                if FUSED_STATS else None
            nat.call("ov3d_sa_dy_fused", y2, a2, s2, w3b, R, c2, c3, S, gsel, isel, ysel, cA, cB, cC, dz2,
                     part, m2, i2, parts2, nwg, like=dout)
            dw3 = _colsum(part)
            del part
        else:
            dy3 = torch.empty((R, c3), dtype=bf, device=dev)
            nat.call("ov3d_sa_layer_dy", y2, a2, s2, w3b, R, c2, c3, S, gsel, isel, cA, cB, cC, dy3,
                     NPARTS_LAYER, like=dout)
            dw3 = weight_grad(dy3, z2)
            dz2 = torch.mm(dy3, w3b)
            del dy3
        # layer 2: ReLU + BN backward (stats pass, unless done by the fused kernel; apply
        # pass), dz1 and dW2
        if fused_bwd and parts2 is not None:
            parts, nparts = parts2, nwg
        else:
            parts, nparts = torch.empty((NPARTS_ROWS, 2, c2), dtype=torch.float64, device=dev), \
                NPARTS_ROWS
            nat.call("ov3d_bn_relu_bwd", 0, dz2, y2, a2, s2, m2, i2, None, None, None, None, R, c2,
                     parts, None, NPARTS_ROWS, None, like=dout)
        cA, cB, cC, dg2, db2 = bn_bwd_affine(parts, nparts, c2, groups[1], R * world[1], g2, m2, i2)
        if fused_bwd2:   # dy2 -> dz1, dW2 and layer 1's statistics in one pass
            nwg2 = min(NWG_DY2, R // 64)
            dz1 = torch.empty((R, c1), dtype=bf, device=dev)
            part = torch.empty((nwg2, c2, c1), dtype=torch.float32, device=dev)
            parts, nparts = torch.empty((2 * nwg2, 2, c1), dtype=torch.float64, device=dev), \
                2 * nwg2
            nat.call("ov3d_sa_dy2_fused", y1, x0, w1f, a1, s1, y2, a2, s2, dz2, cA, cB, cC, w2b, m1,
                     i1, R, c1, c2, dz1, part, parts, nwg2, like=dout)
            dw2 = _colsum(part)
            del dz2, part
        else:
            dy2 = torch.empty((R, c2), dtype=bf, device=dev)
            nat.call("ov3d_bn_relu_bwd", 1, dz2, y2, a2, s2, None, None, cA, cB, cC, None, R, c2,
                     None, dy2, NPARTS_ROWS, None, like=dout)
            del dz2
            dw2 = weight_grad(dy2, z1)
            dz1 = torch.mm(dy2, w2b)
            del dy2
            parts, nparts = torch.empty((NPARTS_ROWS, 2, c1), dtype=torch.float64, device=dev), \
                NPARTS_ROWS
            nat.call("ov3d_bn_relu_bwd", 0, dz1, y1, a1, s1, m1, i1, None, None, None, None, R, c1,
                     parts, None, NPARTS_ROWS, None, like=dout)
        # layer 1: ReLU + BN backward, dW1 reduced against x0 (dy1 never stored)
        cA, cB, cC, dg1, db1 = bn_bwd_affine(parts, nparts, c1, groups[0], R * world[0], g1, m1, i1)
        cin = x0.shape[1]
        parts = torch.empty((NPARTS_ROWS, c1, cin), dtype=torch.float64, device=dev)
        nat.call("ov3d_bn_relu_bwd_cin", 2, dz1, y1, a1, s1, None, None, cA, cB, cC, x0, cin, R, c1,
                 parts, None, NPARTS_ROWS, w1f, like=dout)
        dw1 = torch.empty(cin * c1, dtype=torch.float32, device=dev)
        nat.call("ov3d_reduce_partials_f32", parts, NPARTS_ROWS, cin * c1, dw1, like=parts)
        dw1 = dw1.view(w1shape)
        return (None, dw1, dw2.view(c2, c1), dw3.view(c3, c2), dg1, db1, dg2, db2, dg3, db3, None,
                None, None)


def sa_mlp_pool(mlp, x0, S, seq_m=0):
    """(R, 3) grouped xyz rows (or (R, 6) xyz + colour) -> (R / S, C3) pooled features
    (fp32), fused training path.  seq_m = M (centroids per scene): rows in (m, b) order,
    the encoder's sequence-first layout, written by the pool kernel directly."""
    layers = list(mlp)
    ws = [l.conv.weight for l in layers]
    ws = [w.view(w.shape[0], w.shape[1]) for w in ws]
    bns = tuple(_bn(l) for l in layers)
    return _SAMLPPool.apply(x0, ws[0], ws[1], ws[2], bns[0].weight, bns[0].bias, bns[1].weight,
                            bns[1].bias, bns[2].weight, bns[2].bias, bns, S, seq_m)
