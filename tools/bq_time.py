"""Ball query: the cell index (ov3d_ball_query_cells, the product path) vs the index-order scan
(ov3d_ball_query) on the steps' shapes, HIP events, equal outputs asserted.

    python tools/bq_time.py        # (GPU) one JSON line per shape
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import _native as nat, pointnet2_utils as pu, synthetic  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for (B, N, M, r, S, shuffle) in [(8, 20000, 2048, 0.2, 64, False), (8, 40000, 2048, 0.2, 64, False),
                                     (8, 2048, 1024, 0.4, 32, False), (8, 20000, 2048, 0.2, 64, True)]:
        xyz = synthetic.make_batch(B, seed=1, num_points=N, device="cuda")["point_clouds"][..., :3].contiguous()
        if shuffle:   # the same scenes in random point order
            xyz = xyz[:, torch.randperm(N, device="cuda")].contiguous()
        _, cen = pu.furthest_point_sample_gather(xyz, M)
        idx = torch.empty((B, M, S), dtype=torch.int32, device="cuda")
        scan = lambda: nat.call("ov3d_ball_query", xyz, cen, B, N, M, r, S, idx, like=xyz)
        t_scan = timed(scan)
        ref = idx.clone()
        nbytes = int(nat.load().ov3d_ball_query_ws_bytes(B, N))
        ws = torch.empty((nbytes,), dtype=torch.uint8, device="cuda")
        cells = lambda: nat.call("ov3d_ball_query_cells", xyz, cen, B, N, M, r, S, idx, ws, nbytes,
                                 like=xyz)
        idx.zero_()
        t_cells = timed(cells)
        print(json.dumps({"shuffled": shuffle, "B": B, "N": N, "M": M, "r": r, "S": S, "scan_us": round(t_scan, 2),
                          "cells_us": round(t_cells, 2), "equal": bool(torch.equal(idx, ref))}),
              flush=True)


if __name__ == "__main__":
    main()
