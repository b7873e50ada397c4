"""Golden outputs of the REFERENCE evaluation (utils/ap_calculator.py, utils/eval_det.py,
utils/box_util.py box3d_iou / extract_pc_in_box3d) for the device evaluation path
(ov3d_amd.ap_calculator, csrc/evaldet.hip).  Run here, where /root/reference exists:

    python tests/golden/make_eval_golden.py      # -> tests/golden/evaldet.npz

Inputs are synthetic (tests/golden/eval_cases.py, numpy PCG64): SUN-like scenes with GT
boxes and surface points, predictions = jittered GT boxes (some duplicated, some with the
wrong class) + random boxes in empty space, softmax class probabilities, objectness.
Recorded per batch: the reference's per-box in-hull point counts, the parse_predictions
detections (valid boxes and their per-class scores), every (prediction, GT) box3d_iou of the
first batch, and compute_metrics() at IoU 0.25 / 0.5 over all batches.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

from ref_loader import load_reference  # noqa: E402
from eval_cases import CONFIGS, make_batches  # noqa: E402


def detections_from_lists(batch_pred_map_cls, corners, C):
    """per_class_proposal lists -> (valid (B,K), scores (B,K,C)), boxes located by their
    view's data pointer into the corners array"""
    B, K = corners.shape[:2]
    base = corners.__array_interface__["data"][0]
    valid = np.zeros((B, K), bool)
    scores = np.full((B, K, C), -np.inf, np.float32)
    for i, lst in enumerate(batch_pred_map_cls):
        for cls, box, score in lst:
            off = (box.__array_interface__["data"][0] - base) // (8 * 3 * corners.itemsize)
            b, j = divmod(off, K)
            assert b == i
            valid[b, j] = True
            scores[b, j, cls] = score
    return valid, scores


def main():
    ref = load_reference()
    import utils.ap_calculator as apc
    import utils.box_util as bu
    out = {}
    for name, cfg in CONFIGS.items():
        batches = make_batches(**cfg["data"])
        C = cfg["data"]["num_classes"]

        class Cfg:
            num_semcls = C
        conf = apc.get_ap_config_dict(dataset_config=Cfg(), **cfg["ap"])
        calc = apc.APCalculator(Cfg(), ap_iou_thresh=[0.25, 0.5], class2type_map=None,
                                ap_config_dict=conf)
        for bi, bt in enumerate(batches):
            import torch
            corners = bt["pred_corners"]
            if conf["remove_empty_box"]:
                cnt = np.zeros(corners.shape[:2], np.int32)
                for i in range(corners.shape[0]):
                    for j in range(corners.shape[1]):
                        box = apc.flip_axis_to_depth(corners[i, j])
                        cnt[i, j] = len(bu.extract_pc_in_box3d(bt["point_clouds"][i], box)[0])
                out[f"{name}/b{bi}/counts"] = cnt
            lists = apc.parse_predictions(torch.from_numpy(corners), torch.from_numpy(bt["sem_cls_prob"]),
                                          torch.from_numpy(bt["objectness_prob"]),
                                          torch.from_numpy(bt["point_clouds"]), conf)
            valid, scores = detections_from_lists(lists, corners, C)
            out[f"{name}/b{bi}/valid"] = valid
            out[f"{name}/b{bi}/scores"] = scores
            calc.step(torch.from_numpy(corners), torch.from_numpy(bt["sem_cls_prob"]),
                      torch.from_numpy(bt["objectness_prob"]), torch.from_numpy(bt["point_clouds"]),
                      torch.from_numpy(bt["gt_box_corners"]), torch.from_numpy(bt["gt_box_sem_cls_label"]),
                      torch.from_numpy(bt["gt_box_present"]))
            if bi == 0:
                B, K = corners.shape[:2]
                G = bt["gt_box_corners"].shape[1]
                iou = np.zeros((B, K, G))
                for i in range(B):
                    for j in range(K):
                        for g in range(G):
                            if bt["gt_box_present"][i, g] == 1:
                                iou[i, j, g] = bu.box3d_iou(corners[i, j].astype(float),
                                                            bt["gt_box_corners"][i, g].astype(float))[0]
                out[f"{name}/b0/iou"] = iou
        met = calc.compute_metrics()
        for th, d in met.items():
            for k, v in d.items():
                out[f"{name}/metrics/{th}/{k}"] = np.asarray(v)
        print(name, {th: (float(d["mAP"]), float(d["AR"])) for th, d in met.items()})
    np.savez_compressed(os.path.join(HERE, "evaldet.npz"), **out)
    print("wrote evaldet.npz", len(out))


if __name__ == "__main__":
    main()
