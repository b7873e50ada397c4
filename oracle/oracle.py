"""TEST INFRASTRUCTURE ONLY — numpy/ctypes front-end to liboracle_cpu.so.

The oracle is the parity checker for the HIP library: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import
this module.  Every function cites the reference code it restates (see the
header of ``ov3d_oracle.c`` for the file:line map).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

GIOU_MODE_CYTHON = 0   # utils/box_util.py:624-714 (+ box_intersection.pyx:166-198)
GIOU_MODE_TENSOR = 1   # utils/box_util.py:517-618 (TorchScript, all K2)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return os.path.join(HERE, "liboracle_cpu.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle_cpu.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        i = ctypes.c_int
        L.ov3d_fps_cpu.argtypes = [P, i, i, i, P]
        L.ov3d_fps_rank_cpu.argtypes = [i, i]
        L.ov3d_fps_rank_cpu.restype = ctypes.c_uint32
        L.ov3d_ball_query_cpu.argtypes = [P, P, i, i, i, ctypes.c_float, i, P]
        L.ov3d_group_cpu.argtypes = [P, P, i, i, i, i, i, P]
        L.ov3d_giou3d_cpu.argtypes = [P, P, P, i, i, i, i, i, i, P]
        L.ov3d_nms3d_cpu.argtypes = [P, i, i, ctypes.c_double, i, i, P, P]
        L.ov3d_lsap_cpu.argtypes = [P, i, i, i, P]
        L.ov3d_roi_align_cpu.argtypes = [P, i, i, i, i, P, i, i, i, ctypes.c_float, i, i, i, P]
        for f in (L.ov3d_lsap_cpu, L.ov3d_fps_cpu, L.ov3d_ball_query_cpu, L.ov3d_group_cpu,
                  L.ov3d_giou3d_cpu, L.ov3d_nms3d_cpu, L.ov3d_roi_align_cpu):
            f.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def fps(xyz, npoint):
    """furthest_point_sample [upstream pointnet2; SURVEY Appendix A.1] -> int32 (B,npoint)"""
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    B, N, _ = xyz.shape
    out = np.zeros((B, npoint), dtype=np.int32)
    rc = lib().ov3d_fps_cpu(_p(xyz), B, N, npoint, _p(out))
    assert rc == 0, rc
    return out


def fps_rank(k, n):
    return int(lib().ov3d_fps_rank_cpu(k, n))


def ball_query(xyz, new_xyz, radius, nsample):
    """ball_query [upstream; Appendix A.2] -> int32 (B,M,nsample)"""
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    new_xyz = np.ascontiguousarray(new_xyz, dtype=np.float32)
    B, N, _ = xyz.shape
    M = new_xyz.shape[1]
    out = np.zeros((B, M, nsample), dtype=np.int32)
    rc = lib().ov3d_ball_query_cpu(_p(xyz), _p(new_xyz), B, N, M, float(radius), nsample, _p(out))
    assert rc == 0, rc
    return out


def group(features, idx):
    """grouping_operation [upstream; Appendix A.3]: (B,C,N),(B,M,S) -> (B,C,M,S)"""
    features = np.ascontiguousarray(features, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    B, C, N = features.shape
    _, M, S = idx.shape
    out = np.zeros((B, C, M, S), dtype=np.float32)
    lib().ov3d_group_cpu(_p(features), _p(idx), B, C, N, M, S, _p(out))
    return out


def giou3d(corners1, corners2, nums, mode=GIOU_MODE_CYTHON, rotated=True, k2_bug=True):
    """generalized_box3d_iou (box_util.py:717-737), both dispatch targets."""
    c1 = np.ascontiguousarray(corners1, dtype=np.float32)
    c2 = np.ascontiguousarray(corners2, dtype=np.float32)
    B, K1 = c1.shape[:2]
    K2 = c2.shape[1]
    nums = np.ascontiguousarray(nums, dtype=np.int32)
    out = np.zeros((B, K1, K2), dtype=np.float32)
    rc = lib().ov3d_giou3d_cpu(_p(c1), _p(c2), _p(nums), B, K1, K2, int(mode), int(bool(rotated)),
                               int(bool(k2_bug)), _p(out))
    assert rc == 0, rc
    return out


def nms3d(boxes, overlap_threshold, old_type=False, samecls=True):
    """nms_3d_faster(_samecls) (utils/nms.py:79-162) with the stable tie rule.

    Returns (pick list in pick order, keep mask uint8 (K,))."""
    boxes = np.ascontiguousarray(boxes, dtype=np.float64)
    K, stride = boxes.shape
    picks = np.zeros((max(K, 1),), dtype=np.int32)
    keep = np.zeros((max(K, 1),), dtype=np.uint8)
    n = lib().ov3d_nms3d_cpu(_p(boxes), K, stride, float(overlap_threshold), int(bool(old_type)),
                             int(bool(samecls)), _p(picks), _p(keep))
    assert n >= 0, n
    return picks[:n].tolist(), keep[:K]


def lsap(cost):
    """scipy.optimize.linear_sum_assignment restated (criterion.py:79): cost (Q, n) float32
    -> gt_of_q (Q,) int32, -1 where unmatched."""
    c = np.ascontiguousarray(cost, dtype=np.float32)
    nq, ng = c.shape
    out = np.empty(nq, dtype=np.int32)
    rc = lib().ov3d_lsap_cpu(_p(c), nq, ng, ng, _p(out))
    if rc == -1:
        raise ValueError("matrix contains invalid numeric entries")
    if rc:
        raise ValueError("cost matrix is infeasible")
    return out


def roi_align(feat_nhwc, boxes, per_image, nimages, spatial_scale=1.0 / 16, pooled=18,
              sampling_ratio=0, aligned=True):
    """ROIAlignV2 of RegionCLIP's ROI heads [upstream detectron2/torchvision roi_align,
    reached from criterion.py:397]: feat (N,H,W,C) f32, boxes (R,4) -> (R,P,P,C) f32."""
    f = np.ascontiguousarray(feat_nhwc, dtype=np.float32)
    b = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 4)
    N, H, W, C = f.shape
    R = b.shape[0]
    out = np.zeros((R, pooled, pooled, C), dtype=np.float32)
    rc = lib().ov3d_roi_align_cpu(_p(f), N, H, W, C, _p(b), R, per_image, nimages,
                                  float(spatial_scale), pooled, sampling_ratio, int(bool(aligned)),
                                  _p(out))
    assert rc == 0, rc
    return out
