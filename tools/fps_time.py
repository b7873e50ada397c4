"""FPS launch times (HIP events) on the steps' shapes: B=8, N=20000 -> 2048 (SUN pre-encoder),
2048 -> 128 (query FPS), N=40000 -> 2048 (ScanNet, the two-workgroup kernel).

    python tools/fps_time.py      # (GPU) one JSON line per shape: ms per launch, us per iteration
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import pointnet2_utils as pu, synthetic  # noqa: E402


def main():
    for (B, N, M) in [(8, 20000, 2048), (8, 2048, 128), (8, 40000, 2048)]:
        xyz = synthetic.make_batch(B, seed=2, num_points=N, device="cuda")["point_clouds"][..., :3].contiguous()
        pu.furthest_point_sample(xyz, M)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pu.furthest_point_sample(xyz, M)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[len(ts) // 2]
        print(json.dumps({"B": B, "N": N, "M": M, "ms": round(ms, 4),
                          "us_per_iter": round(ms * 1e3 / (M - 1), 4)}), flush=True)


if __name__ == "__main__":
    main()
