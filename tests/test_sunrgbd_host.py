"""The device loader's file reading on the host (no GPU): scan files, use_pbox pseudo boxes
(kept apart from the support-class filter by the per-scan GT count), use_image calib /
image reads and use_2d_feature features, laid out as datasets/sunrgbd.py:256-285 reads them."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from sunaug_cases import calib_text, image_extras, pseudo_boxes, raw_scans  # noqa: E402
from ov3d_amd import sunrgbd  # noqa: E402
from ov3d_amd.dataset_config import SunrgbdDatasetConfig  # noqa: E402


@pytest.fixture()
def tree(tmp_path):
    root = tmp_path / "sun"
    d = tmp_path / "sun_train"
    pdir, fdir, raw = tmp_path / "pbox", tmp_path / "feat", tmp_path / "raw"
    for x in (d, pdir, fdir, raw / "calib", raw / "image"):
        x.mkdir(parents=True)
    scans = raw_scans(np.float32, 3000)[:4]
    for i, (pc, bb) in enumerate(scans):
        np.savez_compressed(d / ("%06d_pc.npz" % i), pc=pc)
        np.save(d / ("%06d_bbox.npy" % i), bb)
        np.save(pdir / ("%06d_bbox.npy" % i), pseudo_boxes(i))
        img, rt, kk, feat = image_extras(i)
        np.save(fdir / ("%06d.npy" % i), feat)
        np.save(raw / "image" / ("%06d.npy" % i), img)
        (raw / "calib" / ("%06d.txt" % i)).write_text(calib_text(rt, kk))
    return dict(root=str(root), pdir=str(pdir), fdir=str(fdir), raw=str(raw), scans=scans)


def test_disk_read_pbox_image_feature(tree):
    ds = sunrgbd.SunrgbdDetectionDataset(
        SunrgbdDatasetConfig(), split_set="train", root_dir=tree["root"], num_points=1024,
        use_pbox=True, pseudo_box_dir=tree["pdir"], use_image=True, use_2d_feature=True,
        feature_2d_dir=tree["fdir"], raw_data_path=tree["raw"], device="cpu",
        image_reader=lambda path: np.load(path[:-4] + ".npy"))
    st = ds.store
    assert ds.scan_names == ["%06d" % i for i in range(4)]
    for i, (pc, bb) in enumerate(tree["scans"]):
        pb = pseudo_boxes(i)
        assert st.ngt[i] == bb.shape[0] and st.k[i] == bb.shape[0] + pb.shape[0]
        np.testing.assert_array_equal(st.boxes[i, : st.k[i]].numpy(), np.concatenate([bb, pb]))
        img, rt, kk, feat = image_extras(i)
        np.testing.assert_array_equal(st.extras["calib_Rtilt"][i].numpy(), rt)
        np.testing.assert_array_equal(st.extras["calib_K"][i].numpy(), kk)
        np.testing.assert_array_equal(st.extras["feature_2d"][i].numpy(), feat)
        flat = st.extras["image"][i]
        assert flat.dtype == torch.uint8 and flat.numel() == sunrgbd.MAX_NUM_PIXEL * 3
        np.testing.assert_array_equal(flat[: img.size].numpy(), img.reshape(-1))
        assert int(flat[img.size:].abs().sum()) == 0
        assert st.extras["image_height"][i] == img.shape[0]
        assert st.extras["image_width"][i] == img.shape[1]


def test_image_without_reader_raises_clearly(tree, monkeypatch):
    monkeypatch.setitem(sys.modules, "cv2", None)    # absent (other tests may stub it)
    with pytest.raises(ImportError, match="image_reader"):
        sunrgbd.SunrgbdDetectionDataset(SunrgbdDatasetConfig(), split_set="train",
                                        root_dir=tree["root"], use_image=True,
                                        raw_data_path=tree["raw"], device="cpu")
