"""Deterministic synthetic SUN RGB-D-like scenes — there is no
network for the real dataset.  Labels follow the reference dataset contract
(datasets/sunrgbd.py:314-461, without augmentation): GT boxes padded to 64
slots, angle (class, residual) coding, normalised centers / sizes, corners in
the camera frame, point-cloud dims.  numpy PCG64, seed = 1000*rank + index.
"""
import numpy as np
import torch

from .dataset_config import SunrgbdDatasetConfig

MAX_NUM_PIXEL = 530 * 730


def _rotz(t):
    c, s = np.cos(t), np.sin(t)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def _box_surface(rng, n, half, heading, center):
    """n points on the surface of a box with half sizes `half`, yaw `heading` (rotz(-heading))."""
    l, w, h = half
    areas = np.array([w * h, w * h, l * h, l * h, l * w, l * w])
    face = rng.choice(6, size=n, p=areas / areas.sum())
    u = rng.uniform(-1, 1, size=(n, 3)) * np.array([l, w, h])
    axis = face // 2
    sign = np.where(face % 2 == 0, 1.0, -1.0)
    u[np.arange(n), axis] = sign * np.array([l, w, h])[axis]
    return u @ _rotz(-heading).T + center


def make_scene(rng, num_points=20000, cfg=None, nobj=None, use_color=False, use_image=False,
               max_num_obj=64, uniform_volume=False):
    """cfg = ScannetDatasetConfig: axis-aligned boxes (heading 0, angle labels 0, as
    datasets/scannet.py:329-378), classes 0..17"""
    cfg = cfg or SunrgbdDatasetConfig()
    aligned = cfg.num_angle_bin == 1
    if nobj is None:
        nobj = int(rng.integers(1, 11))
    half = rng.uniform(0.15, 1.0, size=(nobj, 3))
    heading = rng.uniform(-np.pi, np.pi, size=nobj)
    heading[0] = abs(heading[0]) + 1e-3  # at least one positive angle -> rotated GIoU path
    if aligned:
        heading[:] = 0.0
    centers = np.stack([rng.uniform(-2.4, 2.4, nobj), rng.uniform(1.0, 6.0, nobj), half[:, 2]], 1)
    if uniform_volume:
        pts = np.stack([rng.uniform(-3, 3, num_points), rng.uniform(0.5, 6.5, num_points),
                        rng.uniform(0, 3, num_points)], 1)
    else:
        surf = [36.0, 18.0, 18.0] + [8 * (a * b + b * c + a * c) for a, b, c in half]
        counts = rng.multinomial(num_points, np.array(surf) / np.sum(surf))
        parts = [
            np.stack([rng.uniform(-3, 3, counts[0]), rng.uniform(0.5, 6.5, counts[0]), np.zeros(counts[0])], 1),
            np.stack([rng.uniform(-3, 3, counts[1]), np.full(counts[1], 6.5), rng.uniform(0, 3, counts[1])], 1),
            np.stack([np.full(counts[2], -3.0), rng.uniform(0.5, 6.5, counts[2]), rng.uniform(0, 3, counts[2])], 1),
        ]
        for i in range(nobj):
            parts.append(_box_surface(rng, counts[3 + i], half[i], heading[i], centers[i]))
        pts = np.concatenate(parts, 0)
        pts = pts + rng.normal(0, 0.01, size=pts.shape)
    pts = pts[rng.permutation(num_points)].astype(np.float32)
    if use_color:
        pts = np.concatenate([pts, rng.uniform(-0.5, 0.5, size=(num_points, 3)).astype(np.float32)], 1)

    G = max_num_obj
    ang_cls = np.zeros(G, np.float32)
    ang_res = np.zeros(G, np.float32)
    raw_sizes = np.zeros((G, 3), np.float32)
    present = np.zeros(G, np.float32)
    present[:nobj] = 1
    target = np.zeros((G, 6))
    sem = np.zeros(G, np.int64)
    sem[:nobj] = rng.integers(0, cfg.num_semcls, nobj)
    for i in range(nobj):
        raw_sizes[i] = half[i] * 2
        c, r = (0, 0.0) if aligned else cfg.angle2class(heading[i])
        ang_cls[i], ang_res[i] = c, r
        local = np.array([[sx * half[i, 0], sy * half[i, 1], sz * half[i, 2]]
                          for sx, sy, sz in [(-1, 1, 1), (1, 1, 1), (1, -1, 1), (-1, -1, 1),
                                             (-1, 1, -1), (1, 1, -1), (1, -1, -1), (-1, -1, -1)]])
        corners = local @ _rotz(-heading[i]).T + centers[i]
        mn, mx = corners.min(0), corners.max(0)
        target[i] = np.concatenate([(mn + mx) / 2, mx - mn])
    dmin = pts[:, :3].min(0)
    dmax = pts[:, :3].max(0)
    mult = dmax - dmin
    sizes_n = raw_sizes / mult[None]
    box_centers = target[:, 0:3].astype(np.float32)
    centers_n = ((box_centers - dmin[None]) / mult[None]) * present[:, None]
    ang_cls_i = ang_cls.astype(np.int64)
    raw_angles = (np.zeros(G, np.float32) if aligned else
                  cfg.class2angle_batch(ang_cls_i, ang_res.astype(np.float32)))
    corners = cfg.box_parametrization_to_corners_np(box_centers[None], raw_sizes[None],
                                                   raw_angles.astype(np.float32)[None])[0]
    d = {
        "point_clouds": pts,
        "gt_box_corners": corners.astype(np.float32),
        "gt_box_centers": box_centers,
        "gt_box_centers_normalized": centers_n.astype(np.float32),
        "gt_box_sem_cls_label": sem,
        "gt_box_present": present,
        "gt_box_sizes": raw_sizes,
        "gt_box_sizes_normalized": sizes_n.astype(np.float32),
        "gt_box_angles": raw_angles.astype(np.float32),
        "gt_angle_class_label": ang_cls_i,
        "gt_angle_residual_label": ang_res,
        "point_cloud_dims_min": dmin.astype(np.float32),
        "point_cloud_dims_max": dmax.astype(np.float32),
    }
    if use_image:
        H, W = 530, 730
        img = np.zeros(MAX_NUM_PIXEL * 3, np.float32)
        img[: H * W * 3] = rng.uniform(0, 255, H * W * 3)
        d.update({"image": img, "image_height": np.int64(H), "image_width": np.int64(W),
                  "calib_Rtilt": np.eye(3),
                  "calib_K": np.array([[529.5, 0, 365.0], [0, 529.5, 265.0], [0, 0, 1]])})
    return d


def make_batch(batch_size, seed=0, device="cpu", dataset="sunrgbd", **kw):
    """Collate `batch_size` scenes (seeds seed*1000 + i) into tensors on `device`."""
    if dataset == "scannet":
        from .dataset_config import ScannetDatasetConfig
        kw.setdefault("cfg", ScannetDatasetConfig())
    scenes = [make_scene(np.random.Generator(np.random.PCG64(seed * 1000 + i)), **kw)
              for i in range(batch_size)]
    out = {}
    for k in scenes[0]:
        out[k] = torch.as_tensor(np.stack([s[k] for s in scenes])).to(device)
    return out


def text_embedding(num_classes=21, dim=640, seed=7):
    """(T, 640) rows of normalize(randn) — stand-in for concepts_sunrgbd*.pth."""
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(num_classes, dim, generator=g)
    return t / t.norm(dim=1, keepdim=True)


def make_raw_scene(rng, num_points=50000, nobj=None, num_classes=20, dtype=np.float32):
    """A raw SUN RGB-D v1 scan as the reference loader reads it (sunrgbd.py:260-262):
    pc (N, 3) upright-depth points (the `_pc.npz` "pc" array, colour dropped) and bboxes
    (K, 8) float64 [cx, cy, cz, l/2, w/2, h/2, heading, class] (the `_bbox.npy` array)."""
    if nobj is None:
        nobj = int(rng.integers(0, 16))
    half = rng.uniform(0.15, 1.0, size=(nobj, 3))
    heading = rng.uniform(-np.pi, np.pi, size=nobj)
    centers = np.stack([rng.uniform(-2.4, 2.4, nobj), rng.uniform(1.0, 6.0, nobj), half[:, 2]], 1)
    surf = [36.0, 18.0, 18.0] + [8 * (a * b + b * c + a * c) for a, b, c in half]
    counts = rng.multinomial(num_points, np.array(surf) / np.sum(surf))
    parts = [
        np.stack([rng.uniform(-3, 3, counts[0]), rng.uniform(0.5, 6.5, counts[0]), np.zeros(counts[0])], 1),
        np.stack([rng.uniform(-3, 3, counts[1]), np.full(counts[1], 6.5), rng.uniform(0, 3, counts[1])], 1),
        np.stack([np.full(counts[2], -3.0), rng.uniform(0.5, 6.5, counts[2]), rng.uniform(0, 3, counts[2])], 1),
    ]
    for i in range(nobj):
        parts.append(_box_surface(rng, counts[3 + i], half[i], heading[i], centers[i]))
    pts = np.concatenate(parts, 0) + rng.normal(0, 0.01, size=(num_points, 3))
    pc = pts[rng.permutation(num_points)].astype(dtype)
    cls = rng.integers(0, num_classes, nobj).astype(np.float64)
    bboxes = np.concatenate([centers, half, heading[:, None], cls[:, None]], 1)
    return pc, bboxes
