"""Device SUN RGB-D batches (ov3d_amd.sunrgbd, csrc/sunaug.hip) against the REFERENCE loader's
own outputs (tests/golden/sunaug.npz, made by tests/golden/make_sunaug_golden.py from
datasets/sunrgbd.py:256-462 with the same numpy seeds).

Bar: bit-exact for every array (points, labels, dims, classes, masks) except
gt_box_corners, where the reference's float32 cos / sin come from numpy's SIMD routines
(get_3d_box_batch_np, box_util.py:265-285) and the device's from ocml: <= 4 float32 ulp
of max(|value|, 1).
"""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from sunaug_cases import CASES, OPTS, image_extras, pseudo_boxes, raw_scans  # noqa: E402
from ov3d_amd import sunrgbd  # noqa: E402
from ov3d_amd.dataset_config import SunrgbdDatasetConfig  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(HERE, "golden", "sunaug.npz"))


def _ulp_close(a, b, ulps):
    """|a - b| <= ulps float32 ulp of max(|a|, |b|, 1): a corner is centre + offset, so an
    offset ulp survives the cancellation near 0"""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    mag = np.maximum(np.maximum(np.abs(a), np.abs(b)), np.float32(1.0))
    return bool(np.all(d <= ulps * np.spacing(mag).astype(np.float64)))


def _dataset(split, dt, nraw, npts, aug, cub, minp, use_pbox=False, use_image=False,
             use_2d_feature=False):
    scans = raw_scans(dt, nraw)
    if use_pbox:      # GT boxes, then the pseudo boxes (the count of GT boxes kept beside)
        scans = [(pc, np.concatenate([bb, pseudo_boxes(i)], 0), bb.shape[0])
                 for i, (pc, bb) in enumerate(scans)]
    extras = None
    if use_image or use_2d_feature:
        extras = []
        for i in range(len(scans)):
            img, rt, kk, feat = image_extras(i)
            e = {}
            if use_image:
                # the calib file round trip of the golden (repr -> float) is exact
                e.update(image=img, calib_Rtilt=rt, calib_K=kk)
            if use_2d_feature:
                e["feature_2d"] = feat
            extras.append(e)
    return sunrgbd.SunrgbdDetectionDataset(SunrgbdDatasetConfig(), split_set=split, num_points=npts,
                                           augment=aug, use_random_cuboid=cub,
                                           random_cuboid_min_points=minp, device="cuda",
                                           scans=scans, extras=extras, use_pbox=use_pbox,
                                           use_image=use_image, use_2d_feature=use_2d_feature)


@pytest.mark.parametrize("name", sorted(CASES))
def test_device_batch_equals_reference_loader(name):
    split, dt, nraw, npts, aug, cub, minp, seed, inds, per_scene = CASES[name]
    ds = _dataset(split, dt, nraw, npts, aug, cub, minp, **OPTS.get(name, {}))
    if per_scene:
        out = ds.get_batch(inds, rngs=[np.random.RandomState(seed * 100 + j) for j in range(len(inds))])
    else:
        out = ds.get_batch(inds, rng=np.random.RandomState(seed))
    torch.cuda.synchronize()
    keys = [k.split("/", 1)[1] for k in GOLD.files if k.startswith(name + "/")]
    if "image" in out:   # the golden keeps the (B, 530*730*3) float32 images as a sha256
        digest = hashlib.sha256(out.pop("image").cpu().numpy().tobytes()).digest()
        assert np.frombuffer(digest, np.uint8).tolist() == GOLD[f"{name}/image_sha256"].tolist()
        keys.remove("image_sha256")
    assert set(keys) == set(out), sorted(set(keys) ^ set(out))
    for k in keys:
        ref = GOLD[f"{name}/{k}"]
        got = out[k].cpu().numpy()
        if k == "scan_idx":
            got = np.asarray(inds)
        assert got.shape == ref.shape, (k, got.shape, ref.shape)
        if k == "gt_box_corners":
            assert _ulp_close(got, ref, 4), (k, np.abs(got - ref).max())
        else:
            assert got.dtype == ref.dtype, (k, got.dtype, ref.dtype)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (
                k, np.argwhere(got != ref)[:5], got[got != ref][:5], ref[got != ref][:5])


def test_shared_rng_state_after_batch_matches_reference_draw_count():
    """after a batch, the generator sits exactly where the reference's per-scene draws leave
    it: a second batch from the same generator equals the reference run continued."""
    split, dt, nraw, npts, aug, cub, minp, seed, inds, _ = CASES["train_f32"]
    ds = _dataset(split, dt, nraw, npts, aug, cub, minp)
    r1 = np.random.RandomState(seed)
    a = ds.get_batch(inds[:3], rng=r1)
    b = ds.get_batch(inds[3:], rng=r1)
    r2 = np.random.RandomState(seed)
    full = ds.get_batch(inds, rng=r2)
    for k in ("point_clouds", "gt_box_centers", "gt_box_present"):
        assert torch.equal(torch.cat([a[k], b[k]]), full[k]), k
    assert r1.get_state()[2] == r2.get_state()[2]
    assert np.array_equal(r1.get_state()[1], r2.get_state()[1])


def test_full_size_batch_equals_oracle():
    """BASELINE size: 8 scans of 50000 raw points -> 20000 sampled, RandomCuboid min_points
    30000 (sunrgbd.py:177-184 defaults), against the numpy restatement (oracle/sunaug_ref.py,
    pinned to the reference by tests/test_sunaug_oracle.py)."""
    sys.path.insert(0, os.path.dirname(HERE))
    from oracle import sunaug_ref
    from ov3d_amd import synthetic
    scans = [synthetic.make_raw_scene(np.random.Generator(np.random.PCG64(70 + i)), num_points=50000)
             for i in range(8)]
    ds = sunrgbd.SunrgbdDetectionDataset(SunrgbdDatasetConfig(), split_set="train", augment=True,
                                         device="cuda", scans=scans)
    inds = [5, 2, 7, 0, 1, 6, 3, 4]
    out = ds.get_batch(inds, rng=np.random.RandomState(123))
    rng = np.random.RandomState(123)
    ref = [sunaug_ref.sun_item(*scans[i], rng, np.arange(10, 20)) for i in inds]
    for k in ref[0]:
        r = np.stack([x[k] for x in ref])
        g = out[k].cpu().numpy()
        if k == "gt_box_corners":
            assert _ulp_close(g, r, 4), k
        else:
            assert np.array_equal(g.view(np.uint8), r.view(np.uint8)), k
