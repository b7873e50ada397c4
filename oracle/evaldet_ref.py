"""TEST INFRASTRUCTURE ONLY — numpy / scipy restatement of the reference detection evaluation.

The checker (and CPU baseline) for ov3d_amd.ap_calculator / csrc/evaldet.hip; only tests/
and tools/ use it.  Restates utils/ap_calculator.py parse_predictions (:39-238, 3D NMS
variants) + APCalculator.compute_metrics (:370-407) and utils/eval_det.py eval_det_cls
(:66-155) + voc_ap (:20-52), with box3d_iou (utils/box_util.py:116-141: Sutherland-Hodgman
clip + scipy ConvexHull area) and in_hull (box_util.py:22-31: scipy Delaunay).  Pinned
against the reference's own outputs by tests/test_evaldet_oracle.py (tests/golden/evaldet.npz).
"""
from collections import OrderedDict

import numpy as np
from scipy.spatial import ConvexHull, Delaunay


def _to_depth(c):
    d = c[..., [0, 2, 1]].copy()
    d[..., 2] *= -1
    return d


def inside_counts(pc, corners):
    """(N,3) points, (K,8,3) upright-camera corners -> (K,) points inside each hull"""
    return np.array([(Delaunay(_to_depth(c)).find_simplex(pc[:, 0:3]) >= 0).sum() for c in corners])


def _nms3d(boxes, thr, old_type, samecls):
    """nms_3d_faster(_samecls) (utils/nms.py:79-162): greedy, ascending argsort popped from the end"""
    x1, y1, z1, x2, y2, z2, score = (boxes[:, i] for i in range(7))
    area = (x2 - x1) * (y2 - y1) * (z2 - z1)
    I = np.argsort(score)
    pick = []
    while I.size:
        i = I[-1]
        pick.append(i)
        rest = I[:-1]
        xx1, yy1, zz1 = (np.maximum(a[i], a[rest]) for a in (x1, y1, z1))
        xx2, yy2, zz2 = (np.minimum(a[i], a[rest]) for a in (x2, y2, z2))
        l, w, h = (np.maximum(0, b - a) for a, b in ((xx1, xx2), (yy1, yy2), (zz1, zz2)))
        inter = l * w * h
        o = inter / np.minimum(area[i], area[rest]) if old_type else inter / (area[i] + area[rest] - inter)
        drop = o > thr
        if samecls:
            drop &= boxes[i, 7] == boxes[rest, 7]
        I = rest[~drop]
    return pick


def detections(corners, probs, obj, pc, cfg, num_semcls):
    """parse_predictions -> scores (B,K,C) float32, -inf where not a detection"""
    B, K = corners.shape[:2]
    cls = np.argmax(probs, -1)
    keep_ne = np.ones((B, K), bool)
    if cfg["remove_empty_box"]:
        for i in range(B):
            keep_ne[i] = inside_counts(pc[i], corners[i]) >= 5
            if not keep_ne[i].any():
                keep_ne[i, obj[i].argmax()] = True
    mask = np.zeros((B, K), bool)
    for i in range(B):
        if cfg.get("no_nms", False):
            mask[i] = keep_ne[i]
            continue
        tab = np.concatenate([corners[i].min(1), corners[i].max(1), obj[i][:, None], cls[i][:, None]], 1)
        idx = np.where(keep_ne[i])[0]
        pick = _nms3d(tab[idx].astype(np.float64), cfg["nms_iou"], cfg["use_old_type_nms"], cfg["cls_nms"])
        mask[i, idx[pick]] = True
    det = mask & (obj > cfg["conf_thresh"])
    scores = np.full((B, K, num_semcls), -np.inf, np.float32)
    for i in range(B):
        for j in np.where(det[i])[0]:
            if cfg["per_class_proposal"]:
                scores[i, j] = probs[i, j, :num_semcls] * obj[i, j]
            elif cfg["use_cls_confidence_only"]:
                scores[i, j, cls[i, j]] = probs[i, j, cls[i, j]]
            else:
                scores[i, j, cls[i, j]] = obj[i, j]
    return scores


def _clip(subject, clip):
    """Sutherland-Hodgman (box_util.py:34-80 semantics), python floats"""
    def inside(p, a, b):
        return (b[0] - a[0]) * (p[1] - a[1]) > (b[1] - a[1]) * (p[0] - a[0])

    def cross(a, b, s, e):
        dc = (a[0] - b[0], a[1] - b[1])
        dp = (s[0] - e[0], s[1] - e[1])
        n1 = a[0] * b[1] - a[1] * b[0]
        n2 = s[0] * e[1] - s[1] * e[0]
        n3 = 1.0 / (dc[0] * dp[1] - dc[1] * dp[0])
        return ((n1 * dp[0] - n2 * dc[0]) * n3, (n1 * dp[1] - n2 * dc[1]) * n3)

    out = list(subject)
    a = clip[-1]
    for b in clip:
        inp, out = out, []
        s = inp[-1]
        for e in inp:
            if inside(e, a, b):
                if not inside(s, a, b):
                    out.append(cross(a, b, s, e))
                out.append(e)
            elif inside(s, a, b):
                out.append(cross(a, b, s, e))
            s = e
        a = b
        if not out:
            return None
    return out


def iou3d(c1, c2):
    c1 = c1.astype(float)
    c2 = c2.astype(float)
    r1 = [(c1[i, 0], c1[i, 2]) for i in (3, 2, 1, 0)]
    r2 = [(c2[i, 0], c2[i, 2]) for i in (3, 2, 1, 0)]
    poly = _clip(r1, r2)
    area = ConvexHull(poly).volume if poly is not None else 0.0
    h = max(0.0, min(c1[0, 1], c2[0, 1]) - max(c1[4, 1], c2[4, 1]))

    def vol(c):
        return (np.sqrt(np.sum((c[0] - c[1]) ** 2)) * np.sqrt(np.sum((c[1] - c[2]) ** 2))
                * np.sqrt(np.sum((c[0] - c[4]) ** 2)))
    inter = area * h
    return inter / (vol(c1) + vol(c2) - inter)


def _voc_ap(rec, prec):
    mrec = np.concatenate(([0.0], rec, [1.0]))
    mpre = np.concatenate(([0.0], prec, [0.0]))
    mpre = np.maximum.accumulate(mpre[::-1])[::-1]
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1])


def compute_metrics(scores, corners, gt_corners, gt_cls, gt_present, thresholds, per_class=True):
    """-> {thresh: OrderedDict(AP per class, mAP, Recall per class, AR)} (class names = str)"""
    S, K, C = scores.shape
    pred, gt = {}, {}
    # the reference's dict construction order (eval_det.py:234-252): scenes in order, each
    # scene's list class-outer / box-inner (per_class_proposal) or box order
    for s in range(S):
        ks = [(c, j) for c in range(C) for j in range(K) if np.isfinite(scores[s, j, c])]
        if not per_class:
            ks.sort(key=lambda t: t[1])
        for c, j in ks:
            pred.setdefault(c, {}).setdefault(s, []).append((corners[s, j], scores[s, j, c]))
            gt.setdefault(c, {}).setdefault(s, [])
    for s in range(S):
        for g in range(gt_corners.shape[1]):
            if gt_present[s, g] == 1:
                gt.setdefault(int(gt_cls[s, g]), {}).setdefault(s, []).append(gt_corners[s, g])
    out = OrderedDict()
    for th in thresholds:
        ap, rec = {}, {}
        for c in gt:
            if c not in pred:
                ap[c], rec[c] = 0, None
                continue
            ids, conf, boxes = [], [], []
            for s, lst in pred[c].items():
                for b, sc in lst:
                    ids.append(s)
                    conf.append(sc)
                    boxes.append(b)
            srt = np.argsort(-np.array(conf), kind="stable")
            det = {s: [False] * len(v) for s, v in gt[c].items()}
            npos = sum(len(v) for v in gt[c].values())
            tp = np.zeros(len(srt))
            fp = np.zeros(len(srt))
            for d, k in enumerate(srt):
                s = ids[k]
                ovmax, jmax = -np.inf, -1
                for jj, g in enumerate(gt[c].get(s, [])):
                    v = iou3d(boxes[k], g)
                    if v > ovmax:
                        ovmax, jmax = v, jj
                if ovmax > th and not det[s][jmax]:
                    tp[d] = 1
                    det[s][jmax] = True
                else:
                    fp[d] = 1
            tp, fp = np.cumsum(tp), np.cumsum(fp)
            r = tp / float(npos) if npos else np.zeros_like(tp)
            p = tp / np.maximum(tp + fp, np.finfo(np.float64).eps)
            ap[c], rec[c] = _voc_ap(r, p), r[-1]
        d = OrderedDict()
        for c in sorted(ap):
            d["%s Average Precision" % c] = ap[c]
        v = np.array(list(ap.values()), dtype=np.float32)
        v[np.isnan(v)] = 0
        d["mAP"] = v.mean()
        rl = []
        for c in sorted(ap):
            r = rec[c] if rec[c] is not None else 0
            d["%s Recall" % c] = r
            rl.append(r)
        d["AR"] = np.mean(rl)
        out[th] = d
    return out
