"""Time ov3d_fps (HIP events, median) at the SUN (B=8, N=20000) and ScanNet (B=8, N=40000)
pre-encoder shapes, M=2048: ms per launch and us per sampling iteration."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import pointnet2_utils as pu, synthetic  # noqa: E402
from bench_kernels import timeit  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for n in (20000, 40000):
        xyz = synthetic.make_batch(8, seed=1, num_points=n, device=dev)["point_clouds"][..., :3].contiguous()
        ms = timeit(lambda: pu.furthest_point_sample_gather(xyz, 2048), reps=10, warm=2)
        res[f"fps_B8_N{n}_M2048"] = {"ms": round(ms, 3), "us_per_iter": round(ms * 1e3 / 2048, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
