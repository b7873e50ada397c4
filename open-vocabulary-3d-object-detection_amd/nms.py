"""3D NMS on the ov3d HIP kernel (replaces reference utils/nms.py:79-162).

* ``nms_3d_faster_samecls(boxes, overlap_threshold, old_type=False)`` and
  ``nms_3d_faster(...)``: same signature and return value (pick list, in pick
  order) as the reference numpy functions for one scene;
* ``nms3d_batched``: all scenes of a batch in one launch, straight from device
  tensors -> (B, K) keep mask, the ``pred_mask`` of ap_calculator.py:153-190.
Float64 arithmetic in the reference's evaluation order; score ties break
towards the larger index (np.argsort(kind="stable") read from the back).
"""
import numpy as np
import torch

from . import _native as nat

MAX_K = 512


def nms3d_batched(boxes, overlap_threshold, old_type=False, samecls=True, valid=None):
    """boxes (B,K,7|8) float64 cuda, valid (B,K) bool/uint8 or None -> keep (B,K) uint8."""
    boxes = nat.check(boxes.to(torch.float64).contiguous(), "boxes", torch.float64, 3)
    B, K, stride = boxes.shape
    if K > MAX_K:
        raise ValueError(f"nms3d supports K <= {MAX_K} boxes per scene")
    v = None
    if valid is not None:
        v = nat.check(valid.to(device=boxes.device, dtype=torch.uint8).contiguous(), "valid",
                      torch.uint8, 2)
    keep = torch.empty((B, K), dtype=torch.uint8, device=boxes.device)
    nat.call("ov3d_nms3d", boxes, v, B, K, stride, float(overlap_threshold), int(bool(old_type)),
             int(bool(samecls)), keep, like=boxes)
    return keep


def nms_boxes_from_corners(corners, obj_prob, sem_cls=None):
    """(B,K,8,3) corners, (B,K) objectness, (B,K) class -> (B,K,8) float64 NMS table
    [xmin,ymin,zmin,xmax,ymax,zmax,obj,cls] (ap_calculator.py:153-187)."""
    c = nat.check(corners.detach().float().contiguous(), "corners", torch.float32, 4)
    B, K = c.shape[:2]
    o = nat.check(obj_prob.detach().float().contiguous(), "obj", torch.float32, 2)
    cl = None
    if sem_cls is not None:
        cl = nat.check(sem_cls.to(torch.int64).contiguous(), "cls", torch.int64, 2)
    out = torch.empty((B, K, 8), dtype=torch.float64, device=c.device)
    nat.call("ov3d_nms_boxes_from_corners", c, o, cl, B, K, out, like=c)
    return out


def _single(boxes, thr, old_type, samecls):
    dev = torch.device("cuda", torch.cuda.current_device())
    b = torch.as_tensor(np.ascontiguousarray(boxes, dtype=np.float64), device=dev)[None]
    keep = nms3d_batched(b, thr, old_type=old_type, samecls=samecls)[0]
    score = b[0, :, 6]
    idx = torch.nonzero(keep).flatten()
    # pick order = descending score, ties -> larger index first
    order = sorted(idx.tolist(), key=lambda i: (-float(score[i]), -i))
    return order


def nms_3d_faster(boxes, overlap_threshold, old_type=False):
    return _single(boxes, overlap_threshold, old_type, samecls=False)


def nms_3d_faster_samecls(boxes, overlap_threshold, old_type=False):
    return _single(boxes, overlap_threshold, old_type, samecls=True)
