"""Box geometry and 3D GIoU on the ov3d HIP kernels (mirror of the hot-path
parts of reference utils/box_util.py).

``generalized_box3d_iou`` keeps the reference signature (box_util.py:717-724)
and its dispatch: ``needs_grad=False`` -> the Cython semantics
(box_util.py:624-714 + box_intersection.pyx, including the K2 bug, Q1, unless
``k2_bug=False``), ``needs_grad=True`` -> the TorchScript semantics
(box_util.py:517-618) with an analytic HIP backward, axis-aligned and rotated.
Both run on the device (the reference copies rectangles to the host and loops
in Cython, box_util.py:684-698).
"""
import numpy as np
import torch
from torch.autograd import Function

from . import _native as nat


# ----------------------------------------------------------------- geometry
def flip_axis_to_camera_tensor(pc):
    """depth (X right, Y fwd, Z up) -> camera (X right, Y down, Z fwd): (x, -z, y)"""
    return torch.stack([pc[..., 0], -pc[..., 2], pc[..., 1]], dim=-1)


def flip_axis_to_camera_np(pc):
    pc2 = pc.copy()
    pc2[..., [0, 1, 2]] = pc2[..., [0, 2, 1]]
    pc2[..., 1] *= -1
    return pc2


# corner sign pattern of reference get_3d_box_batch_tensor (box_util.py:337-345)
_SX = (1, 1, -1, -1, 1, 1, -1, -1)
_SY = (1, 1, 1, 1, -1, -1, -1, -1)
_SZ = (1, -1, -1, 1, 1, -1, -1, 1)
_SIGN_CACHE = {}


def _corner_signs(dtype, device):
    """(3, 8) sign table, one device copy per (dtype, device): no H2D copy per call, so the
    forward stays capturable in a hipGraph."""
    key = (dtype, device)
    t = _SIGN_CACHE.get(key)
    if t is None:
        t = torch.tensor((_SX, _SY, _SZ), dtype=dtype, device=device)
        _SIGN_CACHE[key] = t
    return t


def get_3d_box_batch_tensor(box_size, angle, center):
    """(…,3) size (l,w,h), (…) yaw about camera Y, (…,3) center -> (…,8,3) corners.

    corner = R_y(angle) @ (sx*l/2, sy*h/2, sz*w/2) + center (box_util.py:313-352)."""
    l = box_size[..., 0:1] / 2
    w = box_size[..., 1:2] / 2
    h = box_size[..., 2:3] / 2
    sx, sy, sz = _corner_signs(box_size.dtype, box_size.device)
    lx, ly, lz = l * sx, h * sy, w * sz
    c = torch.cos(angle)[..., None]
    s = torch.sin(angle)[..., None]
    x = lx * c + lz * s + center[..., 0:1]
    y = ly + center[..., 1:2]
    z = lz * c - lx * s + center[..., 2:3]
    return torch.stack([x, y, z], dim=-1)


def roty_batch_np(t):
    out = np.zeros(tuple(t.shape) + (3, 3))
    c, s = np.cos(t), np.sin(t)
    out[..., 0, 0] = c
    out[..., 0, 2] = s
    out[..., 1, 1] = 1
    out[..., 2, 0] = -s
    out[..., 2, 2] = c
    return out


def get_3d_box_batch_np(box_size, angle, center):
    R = roty_batch_np(angle)
    l, w, h = box_size[..., 0:1], box_size[..., 1:2], box_size[..., 2:3]
    corners = np.zeros(tuple(angle.shape) + (8, 3))
    corners[..., :, 0] = np.concatenate([s * l / 2 for s in _SX], -1)
    corners[..., :, 1] = np.concatenate([s * h / 2 for s in _SY], -1)
    corners[..., :, 2] = np.concatenate([s * w / 2 for s in _SZ], -1)
    nd = len(angle.shape)
    corners = np.matmul(corners, np.transpose(R, tuple(range(nd)) + (nd + 1, nd)))
    return corners + np.expand_dims(center, -2)


# --------------------------------------------------------------------- GIoU
def _prep(corners1, corners2, nums_k2):
    c1 = nat.check(corners1.detach().float().contiguous(), "corners1", torch.float32, 4)
    c2 = nat.check(corners2.detach().float().contiguous(), "corners2", torch.float32, 4)
    if c1.shape[0] != c2.shape[0] or c1.shape[2:] != (8, 3) or c2.shape[2:] != (8, 3):
        raise ValueError("corners must be (B,K,8,3) with matching B")
    nums = None
    if nums_k2 is not None:
        nums = nat.check(nums_k2.to(device=c1.device, dtype=torch.int32).contiguous(), "nums_k2",
                         torch.int32, 1)
    return c1, c2, nums


def giou3d_raw(corners1, corners2, nums_k2, mode, rotated, k2_bug=True):
    """rotated: bool, or a device int32 scalar tensor read by the kernel (no host sync)."""
    c1, c2, nums = _prep(corners1, corners2, nums_k2)
    B, K1 = c1.shape[:2]
    K2 = c2.shape[1]
    out = torch.empty((B, K1, K2), dtype=torch.float32, device=c1.device)
    flag = None
    if isinstance(rotated, torch.Tensor):
        flag = nat.check(rotated.to(device=c1.device, dtype=torch.int32).reshape(1).contiguous(),
                         "rotated", torch.int32, 1)
        rotated = False
    nat.call("ov3d_giou3d", c1, c2, nums, B, K1, K2, int(mode), int(bool(rotated)), flag,
             int(bool(k2_bug)), out, like=c1)
    return out


class _GIoUTensor(Function):
    """differentiable GIoU (box_util.py:517-621, all K2) with the reference's autograd
    gradient w.r.t. corners1: axis-aligned, or rotated -- through the Sutherland-Hodgman
    clip's intersection vertices (box_util.py:387-440, 579-600).  `rotated` is a bool or the
    criterion's device flag (any(gt_box_angles > 0), criterion.py:317-330): read on the
    device, forward and backward, so a captured step needs no host sync."""

    @staticmethod
    def forward(ctx, corners1, corners2, nums_k2, rotated):
        c1, c2, nums = _prep(corners1, corners2, nums_k2)
        flag = rotated if isinstance(rotated, torch.Tensor) else None
        if flag is not None:
            flag = nat.check(flag.to(device=c1.device, dtype=torch.int32).reshape(1).contiguous(),
                             "rotated", torch.int32, 1)
        ctx.save_for_backward(c1, c2, nums if nums is not None else torch.empty(0),
                              flag if flag is not None else torch.empty(0))
        ctx.has_nums = nums is not None
        ctx.rot_host = bool(rotated) if flag is None else False
        return giou3d_raw(c1, c2, nums, nat.OV3D_GIOU_TENSOR,
                          flag if flag is not None else ctx.rot_host)

    @staticmethod
    def backward(ctx, g):
        c1, c2, nums, flag = ctx.saved_tensors
        nums = nums if ctx.has_nums else None
        flag = flag if flag.numel() else None
        g = nat.check(g.float().contiguous(), "grad", torch.float32, 3)
        B, K1, K2 = g.shape
        gc1 = torch.empty_like(c1)
        nat.call("ov3d_giou3d_bwd", c1, c2, nums, B, K1, K2, int(ctx.rot_host), flag, g, gc1, like=g)
        return gc1, None, None, None


def generalized_box3d_iou(corners1, corners2, nums_k2, rotated_boxes=True,
                          return_inter_vols_only=False, needs_grad=False, k2_bug=True):
    """(B,K1,8,3), (B,K2,8,3), (B,) -> (B,K1,K2) generalized IoU.

    rotated_boxes may be a device flag tensor (criterion: any(gt_box_angles > 0))."""
    if return_inter_vols_only:
        raise NotImplementedError("return_inter_vols_only is not on the training path")
    if needs_grad:
        return _GIoUTensor.apply(corners1, corners2, nums_k2, rotated_boxes)
    with torch.no_grad():
        return giou3d_raw(corners1, corners2, nums_k2, nat.OV3D_GIOU_CYTHON, rotated_boxes, k2_bug)
