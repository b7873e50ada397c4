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
}
NSCAN = 8


def raw_scans(dtype, num_raw):
    out = []
    for i in range(NSCAN):
        rng = np.random.Generator(np.random.PCG64(9000 + i))
        nobj = [0, 3, 7, 12, 1, 15, 5, 9][i]
        out.append(synthetic.make_raw_scene(rng, num_points=num_raw, nobj=nobj, dtype=dtype))
    return out


