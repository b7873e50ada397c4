"""Golden batches of the REFERENCE SUN RGB-D loader (datasets/sunrgbd.py:256-462) for the
device pipeline (ov3d_amd.sunrgbd, csrc/sunaug.hip).  Run here, where /root/reference exists:

    python tests/golden/make_sunaug_golden.py      # -> tests/golden/sunaug.npz

Raw scans: ov3d_amd.synthetic.make_raw_scene with numpy PCG64 seeds (regenerated
bit-identically by the test), written as the reference's ``{scan}_pc.npz`` /
``{scan}_bbox.npy`` files into a temporary ``root_dir + "_train"`` / ``"_val"`` directory
and read by the reference's own SunrgbdDetectionDataset.  Each case seeds numpy's global
generator (np.random.seed) exactly as the test seeds the RandomState it passes.
"""
import hashlib
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

from ref_loader import load_reference  # noqa: E402
from sunaug_cases import CASES, OPTS, calib_text, image_extras, pseudo_boxes, raw_scans  # noqa: E402


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
            opts = OPTS.get(name, {})
            pdir, fdir, raw = (os.path.join(tmp, name, x) for x in ("pbox", "feat", "raw"))
            for x in (pdir, fdir, os.path.join(raw, "calib"), os.path.join(raw, "image")):
                os.makedirs(x)
            for i, (pc, bb) in enumerate(raw_scans(dt, nraw)):
                np.savez_compressed(os.path.join(d, "%06d_pc.npz" % i), pc=pc)
                np.save(os.path.join(d, "%06d_bbox.npy" % i), bb)
                np.save(os.path.join(pdir, "%06d_bbox.npy" % i), pseudo_boxes(i))
                img, rt, kk, feat = image_extras(i)
                np.save(os.path.join(fdir, "%06d.npy" % i), feat)
                np.save(os.path.join(raw, "image", "%06d.npy" % i), img)
                with open(os.path.join(raw, "calib", "%06d.txt" % i), "w") as f:
                    f.write(calib_text(rt, kk))
            # cv2 is absent here: the stub's imread reads the image array saved beside the
            # .jpg name (the decoder is not what is being pinned)
            sys.modules["cv2"].imread = lambda path: np.load(path[:-4] + ".npy")
            ds = sun.SunrgbdDetectionDataset(cfg, split_set=split, root_dir=root, num_points=npts,
                                             augment=aug, use_random_cuboid=cub,
                                             random_cuboid_min_points=minp, pseudo_box_dir=pdir,
                                             feature_2d_dir=fdir, **opts)
            ds.raw_data_path = raw
            np.random.seed(seed)
            items = []
            for j, i in enumerate(inds):
                if per_scene:
                    np.random.seed(seed * 100 + j)
                items.append(ds[i])
            for k in items[0]:
                v = np.stack([it[k] for it in items])
                if k == "image":   # (B, 530*730*3) float32: kept as its sha256 (IMAGE_DIGEST)
                    v = np.frombuffer(hashlib.sha256(np.ascontiguousarray(v).tobytes()).digest(),
                                      np.uint8).copy()
                    k = "image_sha256"
                res[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "sunaug.npz"), **res)
    print("wrote", os.path.join(HERE, "sunaug.npz"), len(res), "arrays")


if __name__ == "__main__":
    main()
