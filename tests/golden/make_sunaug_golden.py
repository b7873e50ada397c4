"""Golden batches of the REFERENCE SUN RGB-D loader (datasets/sunrgbd.py:256-462) for the
device pipeline (ov3d_amd.sunrgbd, csrc/sunaug.hip).  Run here, where /root/reference exists:

    python tests/golden/make_sunaug_golden.py      # -> tests/golden/sunaug.npz

Raw scans: ov3d_amd.synthetic.make_raw_scene with numpy PCG64 seeds (regenerated
bit-identically by the test), written as the reference's ``{scan}_pc.npz`` /
``{scan}_bbox.npy`` files into a temporary ``root_dir + "_train"`` / ``"_val"`` directory
and read by the reference's own SunrgbdDetectionDataset.  Each case seeds numpy's global
generator (np.random.seed) exactly as the test seeds the RandomState it passes.
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

from ref_loader import load_reference  # noqa: E402
from sunaug_cases import CASES, raw_scans  # noqa: E402


def main():
    ref = load_reference()
    sun = ref["sunrgbd"]
    cfg = sun.SunrgbdDatasetConfig()
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (split, dt, nraw, npts, aug, cub, minp, seed, inds, per_scene) in CASES.items():
            root = os.path.join(tmp, name, "sun")
            d = root + "_" + split
            os.makedirs(d)
            for i, (pc, bb) in enumerate(raw_scans(dt, nraw)):
                np.savez_compressed(os.path.join(d, "%06d_pc.npz" % i), pc=pc)
                np.save(os.path.join(d, "%06d_bbox.npy" % i), bb)
            ds = sun.SunrgbdDetectionDataset(cfg, split_set=split, root_dir=root, num_points=npts,
                                             augment=aug, use_random_cuboid=cub,
                                             random_cuboid_min_points=minp)
            np.random.seed(seed)
            items = []
            for j, i in enumerate(inds):
                if per_scene:
                    np.random.seed(seed * 100 + j)
                items.append(ds[i])
            for k in items[0]:
                res[f"{name}/{k}"] = np.stack([it[k] for it in items])
    np.savez_compressed(os.path.join(HERE, "sunaug.npz"), **res)
    print("wrote", os.path.join(HERE, "sunaug.npz"), len(res), "arrays")


if __name__ == "__main__":
    main()
