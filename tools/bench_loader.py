"""Throughput of the device SUN RGB-D batch pipeline (ov3d_amd.sunrgbd) vs the reference's
per-scene numpy loader work (oracle/sunaug_ref.py restatement, pinned to the reference), at
the BASELINE sizes: 50000-point raw scans resident in HBM, batches of 8, 20000 points,
RandomCuboid min_points 30000.  Prints one JSON object.

    python tools/bench_loader.py [--batches 20] [--scans 64]
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
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import sunrgbd, synthetic  # noqa: E402
from ov3d_amd.dataset_config import SunrgbdDatasetConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--scans", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--cpu-scenes", type=int, default=16)
    a = ap.parse_args()
    scans = [synthetic.make_raw_scene(np.random.Generator(np.random.PCG64(i)), num_points=50000)
             for i in range(a.scans)]
    ds = sunrgbd.SunrgbdDetectionDataset(SunrgbdDatasetConfig(), split_set="train", augment=True,
                                         device="cuda", scans=scans)
    order = np.random.RandomState(0).permutation(a.scans)
    res = {"workload": "SUN RGB-D train batch: 50000-pt raw scans in HBM -> %d x 20000 pts + labels "
                       "(flip/rotz/scale, RandomCuboid, random_sampling)" % a.batch}
    for mode in ("shared_rng", "per_scene_rng"):
        rng = np.random.RandomState(1)
        def one(k):
            inds = [int(order[(k * a.batch + j) % a.scans]) for j in range(a.batch)]
            if mode == "shared_rng":
                return ds.get_batch(inds, rng=rng)
            return ds.get_batch(inds, rngs=[np.random.RandomState(k * 100 + j) for j in range(a.batch)])
        for k in range(3):
            one(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.batches):
            one(k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[mode] = {"scenes_per_s": round(a.batches * a.batch / dt, 1),
                     "ms_per_batch": round(dt / a.batches * 1e3, 3)}
    sys.path.insert(0, ROOT)
    from oracle import sunaug_ref
    rng = np.random.RandomState(2)
    t0 = time.perf_counter()
    for k in range(a.cpu_scenes):
        sunaug_ref.sun_item(*scans[int(order[k % a.scans])], rng, np.arange(10, 20))
    dt = time.perf_counter() - t0
    res["cpu_numpy_restatement"] = {"scenes_per_s": round(a.cpu_scenes / dt, 1), "cores": 1,
                                    "sample": f"{a.cpu_scenes} scenes, one process (the reference "
                                              "runs 4 such DataLoader workers, main.py:452-458)"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
