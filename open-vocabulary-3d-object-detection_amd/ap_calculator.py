"""Detection evaluation on the device.

Drop-in for utils/ap_calculator.py (``parse_predictions``, ``get_ap_config_dict``,
``APCalculator``) with utils/eval_det.py's AP underneath, computed by the HIP kernels of
csrc/evaldet.hip and the batched NMS of csrc/nms.hip:

* ``step_meter`` / ``step`` (ap_calculator.py:311-353) keep each batch's detections ON THE
  DEVICE: remove_empty_box as in-hull point counts (one launch), 3D NMS with the non-empty
  mask (one launch), the per-class proposal scores of parse_predictions (:192-238) as a
  (B, K, C) tensor (-inf = not a detection of that class).  No host sync per batch.
* ``compute_metrics`` (:370-407): box3d_iou of every (detection, GT) pair of each scene
  (one launch), the TP / FP walk per (scene, class) (one launch), the per-class descending
  sort (torch.sort) and voc_ap (one launch), for each AP IoU threshold.
* ``parse_predictions`` returns the reference's python lists (for callers that read them);
  it is the device parse plus one copy.

Reference quirks kept: class names come from ``class2type_map[key]`` (SUN's map has 17
names for 20 classes, so compute_metrics raises KeyError there exactly as the reference
does; pass class2type_map=None for numeric names).  Unpinned: tie order among equal
confidences (the reference's np.argsort quicksort order; here: scene order, then box index),
points exactly on a box face (Qhull's find_simplex tolerance), and the clipped polygon's
area (shoelace here, Qhull's ConvexHull.volume in the reference: ~1e-16 relative).
"""
from collections import OrderedDict

import numpy as np
import torch

from . import _native as nat
from . import nms as _nms

# ov3d_ap_match limits (csrc/evaldet.hip): proposals walked per (scene, class), and the
# per-scene "detected" flags of the GT boxes in one 64-bit word
AP_MAX_PROPOSALS = 256
AP_MAX_GT = 64


def get_ap_config_dict(remove_empty_box=True, use_3d_nms=True, nms_iou=0.25, use_old_type_nms=False,
                       cls_nms=True, per_class_proposal=True, use_cls_confidence_only=False,
                       conf_thresh=0.05, no_nms=False, dataset_config=None):
    """ap_calculator.py:241-269"""
    return {"remove_empty_box": remove_empty_box, "use_3d_nms": use_3d_nms, "nms_iou": nms_iou,
            "use_old_type_nms": use_old_type_nms, "cls_nms": cls_nms,
            "per_class_proposal": per_class_proposal,
            "use_cls_confidence_only": use_cls_confidence_only, "conf_thresh": conf_thresh,
            "no_nms": no_nms, "dataset_config": dataset_config}


def box_points_count(point_cloud, corners):
    """points of each scene inside each box's hull: point_cloud (B,N,>=3) f32, corners
    (B,K,8,3) upright camera -> (B,K) int32 (extract_pc_in_box3d, box_util.py:28-31)"""
    pc = nat.check_device(point_cloud.detach().float(), "point_cloud")
    if pc.stride(2) != 1:
        pc = pc.contiguous()
    c = nat.check(corners.detach().float().contiguous(), "corners", torch.float32, 4)
    B, K = c.shape[:2]
    out = torch.empty((B, K), dtype=torch.int32, device=c.device)
    nat.call("ov3d_box_points_count", pc, pc.stride(0), pc.stride(1), pc.shape[1], c, B, K, out,
             like=c)
    return out


def parse_predictions_device(predicted_boxes, sem_cls_probs, objectness_probs, point_cloud,
                             config_dict):
    """ap_calculator.py:39-238 on the device -> (scores (B,K,C) f32 with -inf where a box is
    not a detection of that class, pred_mask (B,K) uint8)."""
    corners = predicted_boxes.detach().float().contiguous()
    probs = sem_cls_probs.detach().float()
    obj = objectness_probs.detach().float().contiguous()
    B, K = corners.shape[:2]
    dev = corners.device
    pred_cls = torch.argmax(probs, -1)             # np.argmax: first maximum
    if config_dict["remove_empty_box"]:
        nonempty = box_points_count(point_cloud[..., 0:3], corners) >= 5
        none = ~nonempty.any(1)                     # all empty -> keep the most objectlike
        first = torch.nn.functional.one_hot(torch.argmax(obj, 1), K).bool()
        nonempty = nonempty | (none[:, None] & first)
    else:
        nonempty = torch.ones((B, K), dtype=torch.bool, device=dev)
    if config_dict.get("no_nms", False):
        pred_mask = nonempty
    elif not config_dict["use_3d_nms"]:
        raise NotImplementedError("2D NMS (use_3d_nms=False) is not on the 3DETR path")
    else:
        boxes = _nms.nms_boxes_from_corners(corners, obj, pred_cls if config_dict["cls_nms"] else None)
        keep = _nms.nms3d_batched(boxes, config_dict["nms_iou"], config_dict["use_old_type_nms"],
                                  samecls=config_dict["cls_nms"], valid=nonempty)
        pred_mask = keep.bool()
    det = pred_mask & (obj > config_dict["conf_thresh"])
    C = config_dict["dataset_config"].num_semcls
    neg = torch.tensor(-float("inf"), device=dev)
    if config_dict["per_class_proposal"]:
        assert config_dict["use_cls_confidence_only"] is False
        scores = torch.where(det[..., None], probs[..., :C] * obj[..., None], neg)
    else:
        val = (torch.gather(probs, -1, pred_cls[..., None])[..., 0]
               if config_dict["use_cls_confidence_only"] else obj)
        Cn = max(C, probs.shape[-1])
        scores = torch.full((B, K, Cn), -float("inf"), device=dev)
        scores.scatter_(-1, pred_cls[..., None], torch.where(det, val, neg)[..., None])
    return scores.contiguous(), pred_mask.to(torch.uint8)


def parse_predictions(predicted_boxes, sem_cls_probs, objectness_probs, point_cloud, config_dict):
    """the reference's return value: per scene a list of (class, corners (8,3), score),
    classes outer / boxes inner for per_class_proposal, boxes in order otherwise"""
    scores, _ = parse_predictions_device(predicted_boxes, sem_cls_probs, objectness_probs,
                                         point_cloud, config_dict)
    sc = scores.cpu().numpy()
    corners = predicted_boxes.detach().cpu().numpy()
    out = []
    for i in range(sc.shape[0]):
        valid = np.isfinite(sc[i])
        if config_dict["per_class_proposal"]:
            out.append([(c, corners[i, j], sc[i, j, c]) for c in range(sc.shape[2])
                        for j in range(sc.shape[1]) if valid[j, c]])
        else:
            out.append([(int(np.argmax(valid[j])), corners[i, j], sc[i, j, np.argmax(valid[j])])
                        for j in range(sc.shape[1]) if valid[j].any()])
    return out


def _first_appearance(mask):
    """(C, M) bool -> per class the flat index of its first True (M if none)"""
    M = mask.shape[1]
    ar = torch.arange(M, device=mask.device).expand_as(mask)
    return torch.where(mask, ar, torch.full_like(ar, M)).min(1).values


def eval_det_device(scores, corners, gt_corners, gt_cls, gt_present, ovthresh_list):
    """eval_det_multiprocessing (eval_det.py:214-272) for every threshold at once.
    scores (S,K,C) f32 (-inf: none), corners (S,K,8,3), gt_* (S,G,...).  Returns, per
    threshold, {class: (ap, rec_last)} in the reference's gt.keys() order, plus the npos."""
    S, K, C = scores.shape
    G = gt_corners.shape[1]
    if K > AP_MAX_PROPOSALS or G > AP_MAX_GT:
        # ov3d_ap_match keeps one 64-bit "detected" word per GT block and walks <= 256
        # proposals per (scene, class) thread
        raise ValueError(f"device AP supports <= {AP_MAX_PROPOSALS} proposals and <= {AP_MAX_GT} "
                         f"GT boxes per scene (got K={K}, G={G}); nqueries / max_num_obj too large")
    dev = scores.device
    det = torch.isfinite(scores)
    pvalid = det.any(-1).to(torch.uint8).contiguous()
    gvalid = (gt_present == 1).to(torch.uint8).contiguous()
    gcls = gt_cls.to(torch.int64).contiguous()
    iou = torch.empty((S, K, G), dtype=torch.float64, device=dev)
    nat.call("ov3d_box3d_iou_eval", corners.contiguous(), pvalid, gt_corners.float().contiguous(),
             gvalid, S, K, G, iou, like=scores)
    # global descending-confidence order per class (stable: scene, then box index)
    flat = scores.permute(2, 0, 1).reshape(C, S * K)
    order = torch.sort(flat, dim=1, descending=True, stable=True).indices
    nvalid = det.permute(2, 0, 1).reshape(C, S * K).sum(1).to(torch.int32)
    gmask = gvalid.bool()
    maxcls = int(max(C, int(gcls[gmask].max().item()) + 1 if gmask.any() else 0))
    npos_all = torch.bincount(gcls[gmask], minlength=maxcls)
    npos = npos_all[:C].to(torch.int32).contiguous()
    tp_cap = max(1, int(npos.max().item()) if C else 1)
    # the reference's class order: predicted classes by first appearance, then GT-only
    pred_first = _first_appearance(det.reshape(S * K, C).t())
    gt_first = _first_appearance(torch.stack([(gcls == c) & gmask for c in range(maxcls)]).reshape(maxcls, -1))
    res = {}
    for th in ovthresh_list:
        tp = torch.zeros((S, K, C), dtype=torch.uint8, device=dev)
        nat.call("ov3d_ap_match", iou, scores.contiguous(), gcls, gvalid, S, K, G, C, float(th), tp,
                 like=scores)
        tps = torch.gather(tp.permute(2, 0, 1).reshape(C, S * K), 1, order).contiguous()
        ap = torch.empty(C, dtype=torch.float64, device=dev)
        rec = torch.empty(C, dtype=torch.float64, device=dev)
        pos = torch.empty((C, tp_cap), dtype=torch.int32, device=dev)
        nat.call("ov3d_ap_curve", tps, S * K, nvalid, npos, C, pos, tp_cap, ap, rec, like=scores)
        res[th] = (ap, rec)
    # host: class order and the per-class values (a few dozen numbers)
    nv = nvalid.cpu().numpy()
    pf = pred_first.cpu().numpy()
    gf = gt_first.cpu().numpy()
    in_pred = [c for c in range(C) if nv[c] > 0]
    keys = sorted(in_pred, key=lambda c: pf[c])
    keys += sorted([c for c in range(maxcls) if gf[c] < S * G and c not in in_pred], key=lambda c: gf[c])
    out = {}
    for th, (ap, rec) in res.items():
        a, r = ap.cpu().numpy(), rec.cpu().numpy()
        out[th] = OrderedDict((c, (a[c], r[c]) if c in in_pred else (0, None)) for c in keys)
    return out


class APCalculator:
    """ap_calculator.py:272-450 with the detections kept on the device."""

    def __init__(self, dataset_config, ap_iou_thresh=[0.25, 0.5], class2type_map=None,
                 exact_eval=True, ap_config_dict=None):
        self.ap_iou_thresh = ap_iou_thresh
        if ap_config_dict is None:
            ap_config_dict = get_ap_config_dict(dataset_config=dataset_config,
                                                remove_empty_box=exact_eval)
        self.ap_config_dict = ap_config_dict
        self.class2type_map = class2type_map
        self.reset()

    def step_meter(self, outputs, targets):
        if "outputs" in outputs:
            outputs = outputs["outputs"]
        self.step(predicted_box_corners=outputs["box_corners"],
                  sem_cls_probs=outputs["sem_cls_prob"],
                  objectness_probs=outputs["objectness_prob"],
                  point_cloud=targets["point_clouds"],
                  gt_box_corners=targets["gt_box_corners"],
                  gt_box_sem_cls_labels=targets["gt_box_sem_cls_label"],
                  gt_box_present=targets["gt_box_present"])

    def step(self, predicted_box_corners, sem_cls_probs, objectness_probs, point_cloud,
             gt_box_corners, gt_box_sem_cls_labels, gt_box_present):
        scores, _ = parse_predictions_device(predicted_box_corners, sem_cls_probs,
                                             objectness_probs, point_cloud, self.ap_config_dict)
        self._scores.append(scores)
        self._corners.append(predicted_box_corners.detach().float().contiguous())
        self._gt.append((gt_box_corners.detach().float(), gt_box_sem_cls_labels.detach(),
                         gt_box_present.detach()))
        self.scan_cnt += scores.shape[0]

    def compute_metrics(self):
        scores = torch.cat(self._scores)
        corners = torch.cat(self._corners)
        gtc = torch.cat([g[0] for g in self._gt])
        gcl = torch.cat([g[1] for g in self._gt])
        gpr = torch.cat([g[2] for g in self._gt])
        per = eval_det_device(scores, corners, gtc, gcl, gpr, self.ap_iou_thresh)
        overall = OrderedDict()
        for th in self.ap_iou_thresh:
            ap = {c: v[0] for c, v in per[th].items()}
            rec = {c: v[1] for c, v in per[th].items()}
            ret = OrderedDict()
            for key in sorted(ap.keys()):
                name = self.class2type_map[key] if self.class2type_map else str(key)
                ret["%s Average Precision" % name] = ap[key]
            vals = np.array(list(ap.values()), dtype=np.float32)
            vals[np.isnan(vals)] = 0
            ret["mAP"] = vals.mean()
            rl = []
            for key in sorted(ap.keys()):
                name = self.class2type_map[key] if self.class2type_map else str(key)
                r = rec[key] if rec[key] is not None else 0
                ret["%s Recall" % name] = r
                rl.append(r)
            ret["AR"] = np.mean(rl)
            overall[th] = ret
        return overall

    def __str__(self):
        return self.metrics_to_str(self.compute_metrics())

    def metrics_to_str(self, overall_ret, per_class=True):
        """ap_calculator.py:398-436"""
        mAP_strs, AR_strs, per_class_metrics = [], [], []
        for th in self.ap_iou_thresh:
            mAP_strs.append(f"{overall_ret[th]['mAP'] * 100:.2f}")
            AR_strs.append(f"{overall_ret[th]['AR'] * 100:.2f}")
            if per_class:
                per_class_metrics += ["-" * 5, f"IOU Thresh={th}"]
                for x in overall_ret[th]:
                    if x not in ("mAP", "AR"):
                        per_class_metrics.append(f"{x}: {overall_ret[th][x] * 100:.2f}")
        s = ", ".join(f"mAP{x:.2f}" for x in self.ap_iou_thresh) + ": " + ", ".join(mAP_strs) + "\n"
        s += ", ".join(f"AR{x:.2f}" for x in self.ap_iou_thresh) + ": " + ", ".join(AR_strs)
        if per_class:
            s += "\n" + "\n".join(per_class_metrics)
        return s

    def metrics_to_dict(self, overall_ret):
        d = {}
        for th in self.ap_iou_thresh:
            d[f"mAP_{th}"] = overall_ret[th]["mAP"] * 100
            d[f"AR_{th}"] = overall_ret[th]["AR"] * 100
        return d

    def reset(self):
        self._scores, self._corners, self._gt = [], [], []
        self.scan_cnt = 0
