"""Device evaluation (ov3d_amd.ap_calculator, csrc/evaldet.hip) against the REFERENCE
evaluation's own outputs (tests/golden/evaldet.npz from utils/ap_calculator.py,
utils/eval_det.py, utils/box_util.py; made by tests/golden/make_eval_golden.py).

Bars: in-hull point counts, detection masks and per-class scores bit-exact; box3d_iou
<= 1e-12 (shoelace vs Qhull area); per-class AP / recall <= 1e-12, mAP (float32) exact,
AR <= 1e-12.
"""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from eval_cases import CONFIGS, make_batches  # noqa: E402
from ov3d_amd import ap_calculator as apc  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(HERE, "golden", "evaldet.npz"))


class _Cfg:
    def __init__(self, c):
        self.num_semcls = c


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_parse_predictions_equals_reference(name):
    cfg = CONFIGS[name]
    conf = apc.get_ap_config_dict(dataset_config=_Cfg(cfg["data"]["num_classes"]), **cfg["ap"])
    for bi, bt in enumerate(make_batches(**cfg["data"])):
        if conf["remove_empty_box"]:
            cnt = apc.box_points_count(_t(bt["point_clouds"]), _t(bt["pred_corners"])).cpu().numpy()
            assert np.array_equal(cnt, GOLD[f"{name}/b{bi}/counts"]), (bi, np.argwhere(cnt != GOLD[f"{name}/b{bi}/counts"]))
        scores, _ = apc.parse_predictions_device(_t(bt["pred_corners"]), _t(bt["sem_cls_prob"]),
                                                 _t(bt["objectness_prob"]), _t(bt["point_clouds"]), conf)
        sc = scores.cpu().numpy()
        ref = GOLD[f"{name}/b{bi}/scores"]
        assert np.array_equal(np.isfinite(sc).any(-1), GOLD[f"{name}/b{bi}/valid"]), bi
        assert np.array_equal(sc.view(np.uint32), ref.view(np.uint32)), bi


@pytest.mark.parametrize("name", ["exact", "nms_any_class"])
def test_box3d_iou_equals_reference(name):
    cfg = CONFIGS[name]
    bt = make_batches(**cfg["data"])[0]
    B, K = bt["pred_corners"].shape[:2]
    G = bt["gt_box_corners"].shape[1]
    iou = torch.empty((B, K, G), dtype=torch.float64, device="cuda")
    from ov3d_amd import _native as nat
    pv = torch.ones((B, K), dtype=torch.uint8, device="cuda")
    gv = _t((bt["gt_box_present"] == 1).astype(np.uint8))
    nat.call("ov3d_box3d_iou_eval", _t(bt["pred_corners"]), pv, _t(bt["gt_box_corners"]), gv, B, K, G,
             iou, like=pv)
    ref = GOLD[f"{name}/b0/iou"]
    assert (ref > 0.25).sum() > 10 and (ref > 0.5).sum() > 5     # the thresholds are exercised
    np.testing.assert_allclose(iou.cpu().numpy(), ref, rtol=0, atol=1e-12)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_compute_metrics_equals_reference(name):
    cfg = CONFIGS[name]
    conf = apc.get_ap_config_dict(dataset_config=_Cfg(cfg["data"]["num_classes"]), **cfg["ap"])
    calc = apc.APCalculator(_Cfg(cfg["data"]["num_classes"]), ap_iou_thresh=[0.25, 0.5],
                            class2type_map=None, ap_config_dict=conf)
    for bt in make_batches(**cfg["data"]):
        calc.step(_t(bt["pred_corners"]), _t(bt["sem_cls_prob"]), _t(bt["objectness_prob"]),
                  _t(bt["point_clouds"]), _t(bt["gt_box_corners"]), _t(bt["gt_box_sem_cls_label"]),
                  _t(bt["gt_box_present"]))
    met = calc.compute_metrics()
    for th, d in met.items():
        pre = f"{name}/metrics/{th}/"
        keys = [k[len(pre):] for k in GOLD.files if k.startswith(pre)]
        assert list(d.keys()) == sorted(keys, key=lambda k: list(d.keys()).index(k) if k in d else -1)
        assert set(d.keys()) == set(keys)
        for k, v in d.items():
            ref = GOLD[pre + k]
            if k == "mAP":
                assert np.float32(v) == np.float32(ref), (th, v, ref)
            else:
                assert abs(float(v) - float(ref)) <= 1e-12, (th, k, v, ref)
    assert "mAP" in met[0.25] and met[0.25]["mAP"] > 0


def test_parse_predictions_lists_match_reference_layout():
    cfg = CONFIGS["exact"]
    conf = apc.get_ap_config_dict(dataset_config=_Cfg(20), **cfg["ap"])
    bt = make_batches(**cfg["data"])[0]
    lists = apc.parse_predictions(_t(bt["pred_corners"]), _t(bt["sem_cls_prob"]),
                                  _t(bt["objectness_prob"]), _t(bt["point_clouds"]), conf)
    ref = GOLD["exact/b0/scores"]
    for i, lst in enumerate(lists):
        valid = np.isfinite(ref[i])
        assert len(lst) == valid.sum()
        exp = [(c, j) for c in range(20) for j in range(ref.shape[1]) if valid[j, c]]
        for (c, box, s), (ce, je) in zip(lst, exp):
            assert c == ce and s == ref[i, je, c] and np.array_equal(box, bt["pred_corners"][i, je])
