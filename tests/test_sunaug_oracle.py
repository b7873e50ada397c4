"""The loader oracle (oracle/sunaug_ref.py) against the REFERENCE loader's own batches
(tests/golden/sunaug.npz, datasets/sunrgbd.py:256-462): bit-exact, every array.  CPU only."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))

from sunaug_cases import CASES, OPTS, image_extras, pseudo_boxes, raw_scans  # noqa: E402
import hashlib  # noqa: E402
from oracle import sunaug_ref  # noqa: E402

GOLD = np.load(os.path.join(HERE, "golden", "sunaug.npz"))
SUPPORT = np.arange(10, 20)


def oracle_batch(name):
    split, dt, nraw, npts, aug, cub, minp, seed, inds, per_scene = CASES[name]
    scans = raw_scans(dt, nraw)
    rng = np.random.RandomState(seed)
    items = []
    for j, i in enumerate(inds):
        if per_scene:
            rng = np.random.RandomState(seed * 100 + j)
        pc, bb = scans[i]
        opts = OPTS.get(name, {})
        it = sunaug_ref.sun_item(pc, bb, rng, SUPPORT if split == "train" else None,
                                 augment=aug, use_cuboid=cub, min_points=minp, num_points=npts,
                                 pseudo_boxes=pseudo_boxes(i) if opts.get("use_pbox") else None)
        img, rt, kk, feat = image_extras(i)
        if opts.get("use_2d_feature"):
            it["feature_2d"] = feat
        if opts.get("use_image"):   # sunrgbd.py:281-285, 456-461
            flat = np.zeros(530 * 730 * 3, np.float32)
            flat[: img.size] = img.flatten()
            it.update(image=flat, image_height=img.shape[0], image_width=img.shape[1],
                      calib_Rtilt=rt, calib_K=kk)
        items.append(it)
    out = {k: np.stack([it[k] for it in items]) for k in items[0]}
    if "image" in out:
        out["image_sha256"] = np.frombuffer(hashlib.sha256(out.pop("image").tobytes()).digest(),
                                            np.uint8)
    return out


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_equals_reference_loader(name):
    out = oracle_batch(name)
    for k, got in out.items():
        ref = GOLD[f"{name}/{k}"]
        assert got.dtype == ref.dtype and got.shape == ref.shape, (k, got.dtype, ref.dtype)
        assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (k, np.abs(got - ref).max())
