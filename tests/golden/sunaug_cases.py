"""Cases of tests/golden/sunaug.npz (shared by make_sunaug_golden.py and the GPU test):
raw scans are regenerated bit-identically from numpy PCG64 seeds."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import synthetic  # noqa: E402

# case: (split, dtype, num_raw, num_points, augment, cuboid, min_points, seed, indices, per_scene_seeds)
CASES = {
    "train_f32": ("train", np.float32, 6000, 2048, True, True, 3000, 11, [0, 1, 2, 3, 4, 5, 6, 7], False),
    "train_f64": ("train", np.float64, 6000, 2048, True, True, 3000, 3, [2, 0, 5, 1], False),
    "val_f32": ("val", np.float32, 6000, 2048, False, True, 3000, 5, [3, 1, 4, 0], False),
    "train_nocuboid_replace": ("train", np.float32, 6000, 8000, True, False, 3000, 17, [1, 6, 2], False),
    "train_hard_cuboid": ("train", np.float32, 6000, 2048, True, True, 5200, 23, [0, 3, 7, 4], False),
    "train_per_scene": ("train", np.float32, 6000, 2048, True, True, 3000, 29, [4, 2, 6, 0], True),
    "train_pbox": ("train", np.float32, 6000, 2048, True, True, 3000, 31, [0, 5, 3, 7], False),
    "val_image_feat": ("val", np.float32, 6000, 2048, False, True, 3000, 37, [2, 6, 1], False),
    "train_image_pbox": ("train", np.float32, 6000, 2048, True, True, 3000, 41, [7, 1, 4], False),
}
# dataset options per case (sunrgbd.py:185-186, use_image)
OPTS = {
    "train_pbox": dict(use_pbox=True),
    "val_image_feat": dict(use_image=True, use_2d_feature=True),
    "train_image_pbox": dict(use_image=True, use_pbox=True),
}
NSCAN = 8


def raw_scans(dtype, num_raw):
    out = []
    for i in range(NSCAN):
        rng = np.random.Generator(np.random.PCG64(9000 + i))
        nobj = [0, 3, 7, 12, 1, 15, 5, 9][i]
        out.append(synthetic.make_raw_scene(rng, num_points=num_raw, nobj=nobj, dtype=dtype))
    return out




def pseudo_boxes(i):
    """the use_pbox file of scan i (K, 8): classes over all 20 (novel ones included, which
    the support filter would drop if it were applied to them)"""
    rng = np.random.Generator(np.random.PCG64(7000 + i))
    k = [4, 0, 6, 2, 9, 1, 3, 5][i]
    half = rng.uniform(0.15, 1.0, size=(k, 3))
    ctr = np.stack([rng.uniform(-2.4, 2.4, k), rng.uniform(1.0, 6.0, k), half[:, 2]], 1)
    return np.concatenate([ctr, half, rng.uniform(-np.pi, np.pi, (k, 1)),
                           rng.integers(0, 20, (k, 1)).astype(np.float64)], 1)


def image_extras(i):
    """use_image / use_2d_feature inputs of scan i: a BGR uint8 image (ragged sizes up to
    530 x 730), the calib file's two rows, a 2D feature array"""
    rng = np.random.Generator(np.random.PCG64(8000 + i))
    h, w = [(530, 730), (427, 561), (530, 681), (441, 591)][i % 4]
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    rt = np.eye(3) + rng.normal(0, 0.02, (3, 3))
    kk = np.array([[529.5, 0, 365.0], [0, 529.5, 265.0], [0, 0, 1.0]]) + rng.normal(0, 1, (3, 3)) * [[1, 0, 1], [0, 1, 1], [0, 0, 0]]
    feat = rng.standard_normal((16, 640)).astype(np.float32)
    return img, rt, kk, feat


def calib_text(rt, kk):
    """the calib .txt lines (sunrgbd.py:277-279 reads them column-major)"""
    return "\n".join(" ".join(repr(float(x)) for x in m.flatten("F")) for m in (rt, kk)) + "\n"
