"""Synthetic inputs of tests/golden/evaldet.npz (shared by make_eval_golden.py and the tests):
regenerated bit-identically from numpy PCG64 seeds."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import synthetic  # noqa: E402
from ov3d_amd.dataset_config import SunrgbdDatasetConfig  # noqa: E402

_DATA = dict(num_batches=3, batch=4, K=64, num_points=4000, num_classes=20, seed=0)
CONFIGS = {
    "exact": dict(data=_DATA, ap=dict(remove_empty_box=True)),                     # evaluate()
    "meter": dict(data=_DATA, ap=dict(remove_empty_box=False)),                    # train meter
    "objectness": dict(data=_DATA, ap=dict(remove_empty_box=True, per_class_proposal=False)),
    "cls_conf": dict(data=_DATA, ap=dict(remove_empty_box=False, per_class_proposal=False,
                                         use_cls_confidence_only=True)),
    "no_nms": dict(data=_DATA, ap=dict(remove_empty_box=True, no_nms=True)),
    "nms_any_class": dict(data=dict(_DATA, seed=1), ap=dict(remove_empty_box=True, cls_nms=False)),
}


def _scene(rng, K, num_points, C):
    cfg = SunrgbdDatasetConfig()
    sc = synthetic.make_scene(rng, num_points=num_points, cfg=cfg)
    nobj = int(sc["gt_box_present"].sum())
    cen = np.zeros((K, 3), np.float32)
    siz = np.zeros((K, 3), np.float32)
    ang = np.zeros(K, np.float32)
    cls = np.zeros(K, np.int64)
    j = 0
    for g in range(nobj):
        for _ in range(int(rng.integers(1, 4))):
            if j >= K:
                break
            cen[j] = sc["gt_box_centers"][g] + rng.normal(0, 0.12, 3)
            siz[j] = sc["gt_box_sizes"][g] * rng.uniform(0.75, 1.25, 3)
            ang[j] = sc["gt_box_angles"][g] + rng.normal(0, 0.15)
            cls[j] = sc["gt_box_sem_cls_label"][g] if rng.random() < 0.8 else rng.integers(0, C)
            j += 1
    while j < K:   # boxes elsewhere in the room (many of them empty)
        cen[j] = [rng.uniform(-2.8, 2.8), rng.uniform(0.7, 6.3), rng.uniform(0.1, 2.5)]
        siz[j] = rng.uniform(0.2, 1.5, 3)
        ang[j] = rng.uniform(-np.pi, np.pi)
        cls[j] = rng.integers(0, C)
        j += 1
    corners = cfg.box_parametrization_to_corners_np(cen[None], siz[None], ang[None])[0]
    logits = rng.normal(0, 1, (K, C))
    logits[np.arange(K), cls] += rng.uniform(1.0, 4.0, K)
    p = np.exp(logits - logits.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    obj = rng.uniform(0, 1, K)
    obj[rng.random(K) < 0.1] = rng.uniform(0, 0.05)
    return {
        "point_clouds": sc["point_clouds"],
        "pred_corners": corners.astype(np.float32),
        "sem_cls_prob": p.astype(np.float32),
        "objectness_prob": obj.astype(np.float32),
        "gt_box_corners": sc["gt_box_corners"],
        "gt_box_sem_cls_label": sc["gt_box_sem_cls_label"],
        "gt_box_present": sc["gt_box_present"],
    }


def make_batches(num_batches, batch, K, num_points, num_classes, seed):
    out = []
    for bi in range(num_batches):
        scenes = [_scene(np.random.Generator(np.random.PCG64(1000 * seed + 10 * bi + i)), K,
                         num_points, num_classes) for i in range(batch)]
        out.append({k: np.stack([s[k] for s in scenes]) for k in scenes[0]})
    return out
