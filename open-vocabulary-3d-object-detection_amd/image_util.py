"""3D box -> 2D image box projection for the RegionCLIP alignment branch
(mirror of reference utils/image_util.py:117-146, 238-298 as used by
criterion.py:366-396), batched over scenes and decoder layers on the device.

Reference quirk Q4 reproduced: the predicted *full* size is used as the
half-extent (image_util.py:124-127 receives size_unnormalized), and the box is
returned as [min v, min u, max v, max u] (x/y swapped, image_util.py:131-133)
before the [w, h, w, h] clamp of criterion.py:389-391.
"""
import torch


class Boxes:
    """Minimal stand-in for detectron2.structures.Boxes (used only if detectron2 is absent)."""

    def __init__(self, tensor):
        self.tensor = tensor


class Instances:
    """Minimal stand-in for detectron2.structures.Instances."""

    def __init__(self, image_size, **fields):
        self.image_size = image_size
        for k, v in fields.items():
            setattr(self, k, v)


def _structures():
    try:  # the real RegionCLIP stack, when installed
        from detectron2.structures import Boxes as B2, Instances as I2
        return B2, I2
    except Exception:  # pragma: no cover - detectron2 is absent in this image
        return Boxes, Instances


_SIGNS = {}


def _corner_signs(dtype, device):
    """(3, 8) corner sign table, built once per (dtype, device) outside any graph capture."""
    key = (dtype, device)
    if key not in _SIGNS:
        _SIGNS[key] = torch.tensor([[-1, 1, 1, -1, -1, 1, 1, -1], [1, 1, -1, -1, 1, 1, -1, -1],
                                    [1, 1, 1, 1, -1, -1, -1, -1]], dtype=dtype, device=device)
    return _SIGNS[key]


def project_boxes_2d(center, size, heading, Rtilt, K, img_h, img_w):
    """center/size (B,Q,3), heading (B,Q), Rtilt/K (B,3,3), img_h/img_w (B,) -> (B,Q,4).
    On the device: one HIP launch (csrc/project.hip, ov3d_project_box2d); the torch form
    below is the host restatement (CPU parity runs)."""
    if center.is_cuda:
        return _project_device(center, size, heading, Rtilt, K, img_h, img_w)
    c = torch.cos(-heading)[..., None]
    s = torch.sin(-heading)[..., None]
    l, w, h = size[..., 0:1], size[..., 1:2], size[..., 2:3]
    sx, sy, sz = _corner_signs(size.dtype, size.device)
    xc, yc, zc = l * sx, w * sy, h * sz                               # (B,Q,8)
    X = c * xc - s * yc + center[..., 0:1]                            # rotz(-heading) @ corners
    Y = s * xc + c * yc + center[..., 1:2]
    Z = zc + center[..., 2:3]
    P = torch.stack([X, Y, Z], dim=-1)                                # (B,Q,8,3) upright depth
    Rt = Rtilt.float()[:, None, None]                                 # (B,1,1,3,3)
    D = (Rt.transpose(-1, -2) @ P[..., None]).squeeze(-1)             # Rtilt^T @ p
    cam = torch.stack([D[..., 0], -D[..., 2], D[..., 1]], dim=-1)     # flip_axis_to_camera
    uvw = (K.float()[:, None, None] @ cam[..., None]).squeeze(-1)
    u = uvw[..., 0] / uvw[..., 2]
    v = uvw[..., 1] / uvw[..., 2]
    umin, umax = u.min(dim=-1).values, u.max(dim=-1).values
    vmin, vmax = v.min(dim=-1).values, v.max(dim=-1).values
    box = torch.stack([vmin, umin, vmax, umax], dim=-1)               # Q4 swap
    wf = img_w.to(box.dtype)[:, None]
    hf = img_h.to(box.dtype)[:, None]
    lim = torch.stack([wf, hf, wf, hf], dim=-1)
    return torch.minimum(torch.clamp_min(box, 0), lim)


def _project_device(center, size, heading, Rtilt, K, img_h, img_w):
    from . import _native as nat
    B, Q = heading.shape
    f32 = dict(dtype=torch.float32)
    c = nat.check(center.detach().to(**f32).contiguous(), "center", torch.float32, 3)
    s = nat.check(size.detach().to(**f32).contiguous(), "size", torch.float32, 3)
    h = nat.check(heading.detach().to(**f32).contiguous(), "heading", torch.float32, 2)
    rt = Rtilt.detach().to(device=c.device, **f32).contiguous()     # .float() as image_util.py:276
    kk = K.detach().to(device=c.device, **f32).contiguous()
    ih = img_h.to(device=c.device, dtype=torch.int64).contiguous()
    iw = img_w.to(device=c.device, dtype=torch.int64).contiguous()
    if rt.shape != (B, 3, 3) or kk.shape != (B, 3, 3) or ih.shape != (B,) or iw.shape != (B,) \
            or c.shape != (B, Q, 3) or s.shape != (B, Q, 3):
        raise ValueError("project_boxes_2d: center/size (B,Q,3), heading (B,Q), Rtilt/K (B,3,3), "
                         "img_h/img_w (B,)")
    out = torch.empty((B, Q, 4), dtype=torch.float32, device=c.device)
    nat.call("ov3d_project_box2d", c, s, h, B * Q, Q, B, rt, kk, ih, iw, out, like=c)
    return out


def clip_batch(images_1d, img_h, img_w, boxes):
    """Build the per-image list that ``clip.inference`` consumes (criterion.py:371-396):
    image (3,H,W) view of the padded 1-D buffer and Instances(gt_boxes=Boxes(boxes))."""
    B2, I2 = _structures()
    hs = img_h.tolist()
    ws = img_w.tolist()
    out = []
    for b in range(boxes.shape[0]):
        H, W = int(hs[b]), int(ws[b])
        img = images_1d[b, : H * W * 3].view(H, W, 3)
        out.append({"image": img.permute(2, 0, 1).contiguous(),
                    "instances": I2((H, W), gt_boxes=B2(boxes[b]))})
    return out
