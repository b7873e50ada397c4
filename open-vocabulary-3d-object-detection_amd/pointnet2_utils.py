"""Drop-in for ``third_party.pointnet2.pointnet2_utils`` (un-vendored upstream,
imported at models/model_3detr.py:9 of the reference) on the HIP kernels of
libov3d_hip.so.

Same names, argument meaning and return types as the upstream module:
``furthest_point_sample(xyz, npoint) -> int32 (B, npoint)``,
``gather_operation``, ``ball_query``, ``grouping_operation``, ``QueryAndGroup``.
Semantics: SURVEY.md Appendix A (FPS tie rule: DESIGN.md §FPS).
"""
import os

import torch
import torch.nn as nn
from torch.autograd import Function

from . import _native as nat


def _f32(t, name, ndim):
    return nat.check(t.contiguous() if t.dtype == torch.float32 else t.float().contiguous(), name,
                     torch.float32, ndim)


def _i32(t, name, ndim):
    return nat.check(t.to(torch.int32).contiguous(), name, torch.int32, ndim)


def _fps_workspace(B, N, device):
    """scratch of ov3d_fps for N > 20480 points (ov3d_fps_workspace floats), else None"""
    n = nat.load().ov3d_fps_workspace(B, N)
    return torch.empty((n,), dtype=torch.float32, device=device) if n > 0 else None


def fps_pair_status(ws, B, N, npoint):
    """(B,) int32 device tensor: 1 where the two-workgroup FPS (20480 < N <= 40960) lost its
    partner workgroup on the last ov3d_fps of workspace `ws` (that scene's sampled coordinates
    are NaN), else 0 (ov3d_fps_pair_status)."""
    st = torch.empty((B,), dtype=torch.int32, device=ws.device if ws is not None else "cuda")
    nat.call("ov3d_fps_pair_status", ws, B, N, int(npoint), st, like=st)
    return st


class FPSPairLost(RuntimeError):
    """the two-workgroup FPS lost its partner workgroup: the sampled indices are wrong"""


def _check_pair(ws, B, N, npoint, device):
    """eager callers: raise on a lost exchange (a host sync; skipped inside graph capture, where
    the NaN sampled coordinates of furthest_point_sample_gather turn the loss NaN)"""
    if ws is None or torch.cuda.is_current_stream_capturing():
        return
    st = fps_pair_status(ws, B, N, npoint)
    if bool(st.any()):
        raise FPSPairLost(f"furthest_point_sample: scenes {st.nonzero().flatten().tolist()} lost "
                          "their partner workgroup (indices invalid)")


class FurthestPointSampling(Function):
    @staticmethod
    def forward(ctx, xyz, npoint):
        xyz = _f32(xyz, "xyz", 3)
        B, N, _ = xyz.shape
        idx = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
        ws = _fps_workspace(B, N, xyz.device)
        nat.call("ov3d_fps", xyz, B, N, int(npoint), idx, None, ws, like=xyz)
        _check_pair(ws, B, N, npoint, xyz.device)
        ctx.mark_non_differentiable(idx)
        return idx

    @staticmethod
    def backward(ctx, g):
        return None, None


furthest_point_sample = FurthestPointSampling.apply


def furthest_point_sample_gather(xyz, npoint, check=False):
    """FPS with the gather fused into the sampling kernel: returns
    (idx int32 (B,npoint), new_xyz (B,npoint,3)).  Equals
    (furthest_point_sample(xyz, n), gather_operation(xyz^T, idx)^T) bit for bit.
    A scene whose two-workgroup sampling lost its partner gets NaN new_xyz (the step's loss
    turns NaN, no host sync); check=True raises FPSPairLost eagerly instead."""
    with torch.no_grad():
        xyz = _f32(xyz.detach(), "xyz", 3)
        B, N, _ = xyz.shape
        idx = torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
        new_xyz = torch.empty((B, npoint, 3), dtype=torch.float32, device=xyz.device)
        ws = _fps_workspace(B, N, xyz.device)
        nat.call("ov3d_fps", xyz, B, N, int(npoint), idx, new_xyz, ws, like=xyz)
        if check:
            _check_pair(ws, B, N, npoint, xyz.device)
    return idx, new_xyz


class GatherOperation(Function):
    @staticmethod
    def forward(ctx, features, idx):
        features = _f32(features, "features", 3)
        idx = _i32(idx, "idx", 2)
        B, C, N = features.shape
        M = idx.shape[1]
        out = torch.empty((B, C, M), dtype=torch.float32, device=features.device)
        nat.call("ov3d_gather_fwd", features, idx, B, C, N, M, out, like=features)
        ctx.save_for_backward(idx)
        ctx.N = N
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        g = _f32(g, "grad", 3)
        B, C, M = g.shape
        gf = torch.empty((B, C, ctx.N), dtype=torch.float32, device=g.device)
        nat.call("ov3d_gather_bwd", g, idx, B, C, ctx.N, M, gf, like=g)
        return gf, None


gather_operation = GatherOperation.apply


def ball_query(radius, nsample, xyz, new_xyz):
    """-> int32 (B, npoint, nsample): first nsample in-radius indices, ascending."""
    xyz = _f32(xyz.detach(), "xyz", 3)
    new_xyz = _f32(new_xyz.detach(), "new_xyz", 3)
    B, N, _ = xyz.shape
    M = new_xyz.shape[1]
    idx = torch.empty((B, M, nsample), dtype=torch.int32, device=xyz.device)
    # the per-scene cell index (csrc/group.hip bq_cells_*): a stream-ordered temporary from the
    # caching allocator (a graph's private pool under capture)
    nbytes = int(nat.load().ov3d_ball_query_ws_bytes(B, N))
    ws = torch.empty((max(nbytes, 16),), dtype=torch.uint8, device=xyz.device)
    nat.call("ov3d_ball_query_cells", xyz, new_xyz, B, N, M, float(radius), int(nsample), idx,
             ws, nbytes, like=xyz)
    return idx


def _dense_strides(t):
    """Element strides (b, n, c) of a (B,C,N) view when its storage is dense (any dim
    order), else None."""
    B, C, N = t.shape
    order = sorted(range(3), key=lambda d: t.stride(d))
    expect = 1
    for d in order:
        if t.shape[d] > 1 and t.stride(d) != expect:
            return None
        expect *= t.shape[d]
    return t.stride(0), t.stride(2), t.stride(1)


class _Group(Function):
    """Fused QueryAndGroup body -> channels-last rows (B,M,S,3+C):
    (xyz[idx]-new_xyz)[/r] ++ features[idx]; features may be any dense (B,C,N) view."""

    @staticmethod
    def forward(ctx, xyz, new_xyz, features, idx, radius, normalize, inverse=None):
        B, N, _ = xyz.shape
        _, M, S = idx.shape
        C = 0 if features is None else features.shape[1]
        strides = (0, 0, 0)
        if C:
            strides = _dense_strides(features)
            if strides is None:
                features = features.contiguous()
                strides = _dense_strides(features)
        out = torch.empty((B, M, S, 3 + C), dtype=torch.float32, device=xyz.device)
        nat.call("ov3d_group_fwd", xyz, new_xyz, features, *strides, idx, B, C, N, M, S,
                 float(radius), int(bool(normalize)), out, like=xyz)
        ctx.save_for_backward(idx)
        ctx.meta = (B, C, N, M, S, strides, tuple(features.shape) if C else None,
                    tuple(features.stride()) if C else None)
        ctx.inverse = inverse
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, C, N, M, S, strides, shape, stride = ctx.meta
        if C == 0 or not ctx.needs_input_grad[2]:
            return None, None, None, None, None, None, None
        g = nat.check(g.float().contiguous(), "grad", torch.float32, 4)
        gf = torch.empty_strided(shape, stride, dtype=torch.float32, device=g.device)
        if ctx.inverse is not None:   # gather form: one pass, no atomics, no zero fill
            off, rows = ctx.inverse
            nat.call("ov3d_group_bwd_csr", g, off, rows, B, C, N, *strides, gf, like=g)
        else:
            nat.call("ov3d_group_bwd", g, idx, B, C, N, M, S, *strides, gf, like=g)
        return None, None, gf, None, None, None, None


# column alignment of the bf16 group rows (the masked encoder's interim SA: 3 + 256 -> 264).
# 64 (K = 320, whole K chunks for gemm256) measured slower at C4: 7.33 vs 7.29 ms median, the
# wider rows cost the grouping, the GEMMs and the dgrad more than the K tail costs gemm256
ROW_ALIGN = int(os.environ.get("OV3D_GROUP_ROW_ALIGN", "8"))


class _GroupBf16(Function):
    """_Group's rows in bf16, zero-padded to Cp = round_up(3 + C, ROW_ALIGN) columns (aligned
    GEMM K);
    the backward gathers the feature columns of the bf16 row gradient through the inverse."""

    @staticmethod
    def forward(ctx, xyz, new_xyz, features, idx, radius, normalize, inverse=None):
        B, N, _ = xyz.shape
        _, M, S = idx.shape
        C = features.shape[1]
        strides = _dense_strides(features)
        if strides is None:
            features = features.contiguous()
            strides = _dense_strides(features)
        cp = (3 + C + ROW_ALIGN - 1) // ROW_ALIGN * ROW_ALIGN
        out = torch.empty((B, M, S, cp), dtype=torch.bfloat16, device=xyz.device)
        nat.call("ov3d_group_rows_bf16", xyz, new_xyz, features, *strides, idx, B, C, N, M, S,
                 float(radius), int(bool(normalize)), cp, out, like=xyz)
        ctx.meta = (B, C, N, strides, tuple(features.shape), tuple(features.stride()), cp)
        ctx.inverse = inverse
        return out

    @staticmethod
    def backward(ctx, g):
        B, C, N, strides, shape, stride, cp = ctx.meta
        if not ctx.needs_input_grad[2]:
            return None, None, None, None, None, None, None
        if ctx.inverse is None:
            raise RuntimeError("_GroupBf16: the gradient needs the ball query's inverse")
        g = g.to(torch.bfloat16)
        if g.stride(-1) != 1 or g.stride(-2) != cp or not g.view(-1, cp).is_contiguous():
            g = g.contiguous()
        gf = torch.empty_strided(shape, stride, dtype=torch.float32, device=g.device)
        off, rows = ctx.inverse
        nat.call("ov3d_group_bwd_csr_bf16", g, cp, off, rows, B, C, N, *strides, gf, like=g)
        return None, None, gf, None, None, None, None


def group_inverse(idx, N):
    """(B, M, S) int32 ball-query indices over N points -> (offsets (B*N+1), rows (B*M*S)):
    the rows that read each point (ov3d_group_inverse), for the gather-form backward."""
    B, M, S = idx.shape
    dev = idx.device
    cnt, cur = (torch.empty((B * N,), dtype=torch.int32, device=dev) for _ in range(2))
    off = torch.empty((B * N + 1,), dtype=torch.int32, device=dev)
    rows = torch.empty((B * M * S,), dtype=torch.int32, device=dev)
    nat.call("ov3d_group_inverse", idx, B, N, M, S, cnt, off, cur, rows, like=idx)
    return off, rows


def grouping_operation(features, idx):
    """(B,C,N), (B,M,S) -> (B,C,M,S) (differentiable w.r.t. features)."""
    features = _f32(features, "features", 3)
    idx = _i32(idx, "idx", 3)
    B, C, N = features.shape
    # the fused kernel needs an xyz/new_xyz pair; a zero pair makes channels 0:3 zero
    z = torch.zeros((B, N, 3), dtype=torch.float32, device=features.device)
    zc = torch.zeros((B, idx.shape[1], 3), dtype=torch.float32, device=features.device)
    return _Group.apply(z, zc, features, idx, 1.0, False)[..., 3:].permute(0, 3, 1, 2)


# feature gradients of the grouping through the inverse index (ov3d_group_bwd_csr) instead of
# float atomics (ov3d_group_bwd): the masked encoder's interim SA
GATHER_BWD = True


class QueryAndGroup(nn.Module):
    """pointnet2_utils.QueryAndGroup with use_xyz=True (the only mode the
    reference builds: models/model_3detr.py:355-361, 385-391)."""

    def __init__(self, radius, nsample, use_xyz=True, ret_grouped_xyz=False, normalize_xyz=False,
                 sample_uniformly=False, ret_unique_cnt=False):
        super().__init__()
        if not use_xyz or sample_uniformly or ret_unique_cnt:
            raise NotImplementedError("only use_xyz=True grouping is on the reference path")
        self.radius, self.nsample = radius, nsample
        self.use_xyz, self.ret_grouped_xyz, self.normalize_xyz = use_xyz, ret_grouped_xyz, normalize_xyz

    def rows(self, xyz, new_xyz, features=None, idx=None, inverse=None, bf16_rows=False):
        """Grouped features as channels-last rows (B, npoint, nsample, 3+C).  idx: the
        ball-query indices of (xyz, new_xyz) when computed ahead of time; inverse: its
        group_inverse (offsets, rows), likewise.  bf16_rows: bf16 rows padded with zero
        columns to a multiple of 8 (B, npoint, nsample, Cp) for a GEMM (gemm.rows_linear_padk)."""
        if xyz.requires_grad or new_xyz.requires_grad:
            raise NotImplementedError("gradients w.r.t. point coordinates are not on the path")
        if idx is None:
            idx = ball_query(self.radius, self.nsample, xyz, new_xyz)
        elif idx.dtype != torch.int32 or tuple(idx.shape) != (xyz.shape[0], new_xyz.shape[1],
                                                              self.nsample):
            raise ValueError("idx must be int32 (B, npoint, nsample)")
        xyz = _f32(xyz, "xyz", 3)
        new_xyz = _f32(new_xyz, "new_xyz", 3)
        if features is not None:
            if features.dim() != 3:
                raise ValueError("features must be (B, C, N)")
            features = features if features.dtype == torch.float32 else features.float()
            nat.check_device(features, "features")
        inv = None
        if features is not None and features.requires_grad and torch.is_grad_enabled() and \
                (GATHER_BWD or bf16_rows):
            inv = inverse if inverse is not None else group_inverse(idx.contiguous(), xyz.shape[1])
        if bf16_rows and features is not None:
            return _GroupBf16.apply(xyz, new_xyz, features, idx, self.radius, self.normalize_xyz, inv)
        return _Group.apply(xyz, new_xyz, features, idx, self.radius, self.normalize_xyz, inv)

    def forward(self, xyz, new_xyz, features=None):
        """Reference layout: (B, 3+C, npoint, nsample) (a view of the channels-last rows)."""
        out = self.rows(xyz, new_xyz, features).permute(0, 3, 1, 2)
        if self.ret_grouped_xyz:
            return out, out[:, :3]
        return out
