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
        L.ov3d_group_bwd_cpu.argtypes = [P, P, i, i, i, i, i, P]
        L.ov3d_gather_fwd_cpu.argtypes = [P, P, i, i, i, i, P]
        L.ov3d_gather_bwd_cpu.argtypes = [P, P, i, i, i, i, P]
        L.ov3d_project_box2d_cpu.argtypes = [P, P, P, ctypes.c_longlong, i, i, P, P, P, P, P]
        L.ov3d_sa_mlp_fwd_cpu.argtypes = [P, ctypes.c_longlong, i, i, P, P, P, P, ctypes.c_double,
                                          P, P, P, P]
        L.ov3d_sa_mlp_bwd_cpu.argtypes = [P, ctypes.c_longlong, i, i, P, P, P, P, ctypes.c_double,
                                          P, P, P, P]
        for f in (L.ov3d_lsap_cpu, L.ov3d_fps_cpu, L.ov3d_ball_query_cpu, L.ov3d_group_cpu,
                  L.ov3d_giou3d_cpu, L.ov3d_nms3d_cpu, L.ov3d_roi_align_cpu, L.ov3d_group_bwd_cpu,
                  L.ov3d_gather_fwd_cpu, L.ov3d_gather_bwd_cpu, L.ov3d_project_box2d_cpu,
                  L.ov3d_sa_mlp_fwd_cpu, L.ov3d_sa_mlp_bwd_cpu):
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


def group_bwd(grad_out, idx, N):
    """grouping_operation backward: grad_out (B,C,M,S) f32, idx (B,M,S) -> (B,C,N) f32"""
    g = np.ascontiguousarray(grad_out, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    B, C, M, S = g.shape
    out = np.empty((B, C, N), dtype=np.float32)
    assert lib().ov3d_group_bwd_cpu(_p(g), _p(idx), B, C, N, M, S, _p(out)) == 0
    return out


def gather(features, idx):
    """gather_operation (model_3detr.py:174-186, 355-361): (B,C,N) f32, idx (B,M) -> (B,C,M)"""
    f = np.ascontiguousarray(features, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    B, C, N = f.shape
    M = idx.shape[1]
    out = np.empty((B, C, M), dtype=np.float32)
    assert lib().ov3d_gather_fwd_cpu(_p(f), _p(idx), B, C, N, M, _p(out)) == 0
    return out


def gather_bwd(grad_out, idx, N):
    """gather_operation backward: grad_out (B,C,M), idx (B,M) -> (B,C,N) (scatter-add)"""
    g = np.ascontiguousarray(grad_out, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    B, C, M = g.shape
    out = np.empty((B, C, N), dtype=np.float32)
    assert lib().ov3d_gather_bwd_cpu(_p(g), _p(idx), B, C, N, M, _p(out)) == 0
    return out


def project_box2d(center, size, heading, Q, B, Rtilt, K, img_h, img_w):
    """image_util.py:117-134 + :286-298 + criterion.py:386-391 (quirk Q4): rows (n, 3) ordered
    (.., scene, query), Rtilt / K (B, 3, 3), img_h / img_w (B,) -> (n, 4) f32"""
    c = np.ascontiguousarray(center, dtype=np.float32).reshape(-1, 3)
    sz = np.ascontiguousarray(size, dtype=np.float32).reshape(-1, 3)
    hd = np.ascontiguousarray(heading, dtype=np.float32).reshape(-1)
    rt = np.ascontiguousarray(Rtilt, dtype=np.float32)
    kk = np.ascontiguousarray(K, dtype=np.float32)
    ih = np.ascontiguousarray(img_h, dtype=np.int64)
    iw = np.ascontiguousarray(img_w, dtype=np.int64)
    n = c.shape[0]
    out = np.empty((n, 4), dtype=np.float32)
    assert lib().ov3d_project_box2d_cpu(_p(c), _p(sz), _p(hd), n, Q, B, _p(rt), _p(kk), _p(ih),
                                        _p(iw), _p(out)) == 0
    return out


def _sa_args(x0, weights, gammas, betas):
    x0 = np.ascontiguousarray(x0, dtype=np.float32)
    ws = [np.ascontiguousarray(w, dtype=np.float32).reshape(w.shape[0], -1) for w in weights]
    nl = len(ws)
    ch = np.array([x0.shape[1]] + [w.shape[0] for w in ws], dtype=np.int32)
    gs = [None if g is None else np.ascontiguousarray(g, dtype=np.float32) for g in (gammas or [None] * nl)]
    bs = [None if b is None else np.ascontiguousarray(b, dtype=np.float32) for b in (betas or [None] * nl)]
    arr = lambda ts: (ctypes.c_void_p * nl)(*[None if t is None else t.ctypes.data for t in ts])  # noqa: E731
    keep = (x0, ws, gs, bs, ch)
    return x0, nl, ch, arr(ws), arr(gs), arr(bs), keep


def sa_mlp(x0, S, weights, gammas=None, betas=None, eps=1e-5):
    """SharedMLP + max-pool of PointnetSAModuleVotes in train mode (model_3detr.py:353-362),
    float64: x0 (R, cin) centroid-major rows, weights [(c_out, c_in)] -> (out (R/S, C) f32,
    per-layer batch means, biased variances (lists of f64), argmax (R/S, C) int32)"""
    x0, nl, ch, W, G, Bt, keep = _sa_args(x0, weights, gammas, betas)
    R = x0.shape[0]
    C = int(ch[-1])
    out = np.empty((R // S, C), dtype=np.float32)
    tot = int(ch[1:].sum())
    mean, var = np.empty(tot), np.empty(tot)
    amax = np.empty((R // S, C), dtype=np.int32)
    assert lib().ov3d_sa_mlp_fwd_cpu(_p(x0), R, S, nl, _p(ch), W, G, Bt, eps, _p(out), _p(mean),
                                     _p(var), _p(amax)) == 0
    cuts = np.cumsum(ch[1:])[:-1]
    return out, np.split(mean, cuts), np.split(var, cuts), amax


def sa_mlp_bwd(x0, S, weights, dout, gammas=None, betas=None, eps=1e-5):
    """gradients of sum(out * dout) for sa_mlp: ([dW_l], [dgamma_l], [dbeta_l]) f32"""
    x0, nl, ch, W, G, Bt, keep = _sa_args(x0, weights, gammas, betas)
    d = np.ascontiguousarray(dout, dtype=np.float32)
    dW = [np.empty((int(ch[l + 1]), int(ch[l])), dtype=np.float32) for l in range(nl)]
    dg = [np.empty(int(ch[l + 1]), dtype=np.float32) for l in range(nl)]
    db = [np.empty(int(ch[l + 1]), dtype=np.float32) for l in range(nl)]
    arr = lambda ts: (ctypes.c_void_p * nl)(*[t.ctypes.data for t in ts])  # noqa: E731
    assert lib().ov3d_sa_mlp_bwd_cpu(_p(x0), x0.shape[0], S, nl, _p(ch), W, G, Bt, eps, _p(d),
                                     arr(dW), arr(dg), arr(db)) == 0
    return dW, dg, db
