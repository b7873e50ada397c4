"""Throughput of the device detection evaluation (ov3d_amd.ap_calculator) vs the CPU
restatement of the reference evaluation (oracle/evaldet_ref.py: scipy Delaunay in-hull,
numpy NMS, python box3d_iou + ConvexHull, eval_det_cls), SUN RGB-D sizes: 20000-point
scenes, 128 proposals, 20 classes, the exact_eval config of engine.evaluate.
Prints one JSON object.

    python tools/bench_eval.py [--batches 32] [--cpu-scenes 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from eval_cases import _scene  # noqa: E402
from ov3d_amd import ap_calculator as apc  # noqa: E402


class _Cfg:
    num_semcls = 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=32)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--cpu-scenes", type=int, default=8)
    a = ap.parse_args()
    scenes = [_scene(np.random.Generator(np.random.PCG64(i)), 128, 20000, 20) for i in range(a.batch * 4)]
    stack = lambda sl: {k: torch.from_numpy(np.stack([s[k] for s in sl])).cuda() for k in sl[0]}
    dev_batches = [stack(scenes[i * a.batch:(i + 1) * a.batch]) for i in range(4)]
    conf = apc.get_ap_config_dict(dataset_config=_Cfg(), remove_empty_box=True)

    def run(nb):
        calc = apc.APCalculator(_Cfg(), ap_iou_thresh=[0.25, 0.5], ap_config_dict=conf)
        for k in range(nb):
            bt = dev_batches[k % 4]
            calc.step(bt["pred_corners"], bt["sem_cls_prob"], bt["objectness_prob"], bt["point_clouds"],
                      bt["gt_box_corners"], bt["gt_box_sem_cls_label"], bt["gt_box_present"])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        m = calc.compute_metrics()
        torch.cuda.synchronize()
        return m, t1
    run(2)
    t0 = time.perf_counter()
    m, t1 = run(a.batches)
    t2 = time.perf_counter()
    n = a.batches * a.batch
    res = {"workload": "SUN RGB-D eval: %d scenes x 128 proposals x 20 classes, 20000 pts, "
                       "remove_empty_box + 3D NMS + per-class proposals + AP@0.25/0.5" % n,
           "device": {"scenes_per_s": round(n / (t2 - t0), 1), "step_ms_per_batch": round((t1 - t0) / a.batches * 1e3, 3),
                      "compute_metrics_ms": round((t2 - t1) * 1e3, 2), "mAP@0.25": float(m[0.25]["mAP"])}}
    sys.path.insert(0, ROOT)
    from oracle import evaldet_ref as R
    sl = scenes[:a.cpu_scenes]
    cb = {k: np.stack([s[k] for s in sl]) for k in sl[0]}
    t0 = time.perf_counter()
    sc = R.detections(cb["pred_corners"], cb["sem_cls_prob"], cb["objectness_prob"], cb["point_clouds"], conf, 20)
    R.compute_metrics(sc, cb["pred_corners"], cb["gt_box_corners"], cb["gt_box_sem_cls_label"],
                      cb["gt_box_present"], [0.25, 0.5])
    dt = time.perf_counter() - t0
    res["cpu_reference_restatement"] = {"scenes_per_s": round(a.cpu_scenes / dt, 2), "cores": 1,
                                        "sample": f"{a.cpu_scenes} scenes, parse + metrics, one process"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
