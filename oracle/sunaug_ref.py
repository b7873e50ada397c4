"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference SUN RGB-D loader item.

The checker for ov3d_amd.sunrgbd / csrc/sunaug.hip: only ``tests/`` and ``tools/``
measurement scripts use it.  It restates SunrgbdDetectionDataset.__getitem__
(datasets/sunrgbd.py:256-462, use_color / use_height off) for one raw scan and a numpy
RandomState, vectorised over boxes, with numpy's own dtype rules (so the rounding is the
reference's): support-class filter (:268-270), flip (:311-315), rotz (:317-323), scale
(:345-349), RandomCuboid (utils/random_cuboid.py:38-98), labels (:356-400),
random_sampling (utils/pc_util.py:24-32), normalisations (:402-460).
Pinned against the reference's own outputs by tests/test_sunaug_oracle.py
(tests/golden/sunaug.npz).
"""
import numpy as np

TWO_PI = 2 * np.pi


def _rotz(t):
    c, s = np.cos(t), np.sin(t)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def _aspect_ok(cr, amin):
    pairs = ((0, 1), (0, 2), (1, 2))
    return any(np.min(cr[list(p)]) / np.max(cr[list(p)]) >= amin for p in pairs)


def _cuboid(pc, boxes, rng, min_points, aspect=0.75, lo=0.75, hi=1.0):
    """RandomCuboid.__call__ with box_filter_policy='center' (random_cuboid.py:38-98)"""
    span = np.max(pc[:, 0:3], axis=0) - np.min(pc[:, 0:3], axis=0)
    for _ in range(100):
        cr = lo + rng.rand(3) * (hi - lo)
        if not _aspect_ok(cr, aspect):
            continue
        ctr = pc[rng.choice(len(pc)), 0:3]
        half = span * cr / 2.0
        inside = np.all(pc[:, 0:3] <= ctr + half, 1) & np.all(pc[:, 0:3] >= ctr - half, 1)
        if inside.sum() < min_points:
            continue
        sub = pc[inside, :]
        if boxes.sum() > 0:
            keep = (np.all(boxes[:, 0:3] >= sub[:, 0:3].min(0), 1)
                    & np.all(boxes[:, 0:3] <= sub[:, 0:3].max(0), 1))
            if keep.sum() == 0:
                continue
            boxes = boxes[keep]
        return sub, boxes
    return pc, boxes


def _angle_bin(a, nbin):
    """angle2class (sunrgbd.py:102-120) on a float64 array"""
    per = TWO_PI / float(nbin)
    sh = ((a % TWO_PI) + per / 2) % TWO_PI
    cls = (sh / per).astype(np.int64)
    return cls, sh - (cls * per + per / 2)


def _box_corners_upright(boxes):
    """my_compute_box_3d (sunrgbd.py:153-165) for every box -> (K, 8, 3) float64"""
    out = np.zeros((len(boxes), 8, 3))
    sx = np.array([-1, 1, 1, -1, -1, 1, 1, -1])
    sy = np.array([1, 1, -1, -1, 1, 1, -1, -1])
    sz = np.array([1, 1, 1, 1, -1, -1, -1, -1])
    for i, b in enumerate(boxes):
        loc = np.vstack([sx * b[3], sy * b[4], sz * b[5]])
        out[i] = (np.dot(_rotz(-1 * b[6]), loc) + b[0:3, None]).T
    return out


def _corners_camera(sizes, angles, centers):
    """flip_axis_to_camera_np + get_3d_box_batch_np (box_util.py:255-285)"""
    cam = centers.copy()
    cam[..., [0, 1, 2]] = cam[..., [0, 2, 1]]
    cam[..., 1] *= -1
    c, s = np.cos(angles), np.sin(angles)
    R = np.zeros(angles.shape + (3, 3))
    R[..., 0, 0], R[..., 0, 2], R[..., 1, 1], R[..., 2, 0], R[..., 2, 2] = c, s, 1, -s, c
    l, w, h = (sizes[..., k:k + 1] for k in range(3))
    loc = np.zeros(angles.shape + (8, 3))
    loc[..., 0] = np.concatenate((l / 2, l / 2, -l / 2, -l / 2, l / 2, l / 2, -l / 2, -l / 2), -1)
    loc[..., 1] = np.concatenate((h / 2, h / 2, h / 2, h / 2, -h / 2, -h / 2, -h / 2, -h / 2), -1)
    loc[..., 2] = np.concatenate((w / 2, -w / 2, -w / 2, w / 2, w / 2, -w / 2, -w / 2, w / 2), -1)
    return np.matmul(loc, np.swapaxes(R, -1, -2)) + cam[..., None, :]


def sun_item(pc, boxes, rng, support_class=None, augment=True, use_cuboid=True,
             min_points=30000, num_points=20000, nbin=12, G=64, pseudo_boxes=None):
    """one reference __getitem__ -> dict (numpy).  pc (N, 3) float32|float64, boxes (K, 8);
    pseudo_boxes (use_pbox): appended after the support filter (sunrgbd.py:266-271)."""
    pc = pc[:, 0:3].copy()
    boxes = boxes.copy()
    if support_class is not None:
        boxes = boxes[np.isin(boxes[:, -1], support_class)]
    if pseudo_boxes is not None:
        boxes = np.concatenate([boxes, pseudo_boxes], axis=0)
    if augment:
        if rng.random() > 0.5:
            pc[:, 0] = -1 * pc[:, 0]
            boxes[:, 0] = -1 * boxes[:, 0]
            boxes[:, 6] = np.pi - boxes[:, 6]
        ang = (rng.random() * np.pi / 3) - np.pi / 6
        R = _rotz(ang)
        pc[:, 0:3] = np.dot(pc[:, 0:3], R.T)
        boxes[:, 0:3] = np.dot(boxes[:, 0:3], R.T)
        boxes[:, 6] -= ang
        sc = np.full((1, 3), rng.random() * 0.3 + 0.85)
        pc[:, 0:3] *= sc
        boxes[:, 0:3] *= sc
        boxes[:, 3:6] *= sc
        if use_cuboid:
            pc, boxes = _cuboid(pc, boxes, rng, min_points)
    K = len(boxes)
    present = np.zeros(G)
    present[:K] = 1
    raw_sizes = np.zeros((G, 3), np.float32)
    raw_sizes[:K] = boxes[:, 3:6] * 2
    cls = np.zeros(G, np.float32)
    res = np.zeros(G, np.float32)
    c, r = _angle_bin(boxes[:, 6], nbin)
    cls[:K], res[:K] = c, r
    target = np.zeros((G, 3))
    if K:
        cor = _box_corners_upright(boxes)
        target[:K] = (cor.min(1) + cor.max(1)) / 2
    sel = rng.choice(pc.shape[0], num_points, replace=pc.shape[0] < num_points)
    pc = pc[sel]
    dmin, dmax = pc.min(axis=0), pc.max(axis=0)
    mult = dmax - dmin
    sizes_n = raw_sizes * (1.0 / mult)[None]
    centers = target.astype(np.float32)
    centers_n = ((centers - dmin[None]) * (np.ones(3, np.float32) - np.zeros(3, np.float32))[None]
                 / (dmax - dmin)[None] + np.zeros(3, np.float32)[None]) * present[:, None]
    cls_i = cls.astype(np.int64)
    res = res.astype(np.float32)
    ang = cls_i * (TWO_PI / float(nbin)) + res
    ang[ang > np.pi] = ang[ang > np.pi] - 2 * np.pi
    corners = _corners_camera(raw_sizes[None], ang.astype(np.float32)[None], centers[None])[0]
    semcls = np.zeros(G)
    semcls[:K] = boxes[:, -1]
    return {
        "point_clouds": pc.astype(np.float32),
        "gt_box_corners": corners.astype(np.float32),
        "gt_box_centers": centers,
        "gt_box_centers_normalized": centers_n.astype(np.float32),
        "gt_box_sem_cls_label": semcls.astype(np.int64),
        "gt_box_present": present.astype(np.float32),
        "gt_box_sizes": raw_sizes,
        "gt_box_sizes_normalized": sizes_n.astype(np.float32),
        "gt_box_angles": ang.astype(np.float32),
        "gt_angle_class_label": cls_i,
        "gt_angle_residual_label": res,
        "point_cloud_dims_min": dmin,
        "point_cloud_dims_max": dmax,
    }
