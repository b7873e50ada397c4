"""Ball-query launch time at the workloads' sizes (HIP events, 20 launches each); the
centroids-per-wave choice comes from OV3D_BQ_CPW.  python tools/bq_time.py  (GPU)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ov3d_import  # noqa: E402


def main():
    ov3d_import.load()
    from ov3d_amd import pointnet2_utils as pu
    from ov3d_amd import synthetic
    dev = torch.device("cuda")
    cases = [("sun pre-encoder", 8, 20000, 2048, 0.2, 64),
             ("scannet pre-encoder", 8, 40000, 2048, 0.2, 64),
             ("scannet interim", 8, 2048, 1024, 0.4, 32)]
    for name, B, N, M, r, S in cases:
        xyz = synthetic.make_batch(B, seed=1, device=dev, num_points=N)["point_clouds"][..., :3] \
            if N != 2048 else torch.rand(B, N, 3, device=dev) * 4
        xyz = xyz.contiguous()
        _, cen = pu.furthest_point_sample_gather(xyz, M)
        for _ in range(3):
            pu.ball_query(r, S, xyz, cen)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            pu.ball_query(r, S, xyz, cen)
        e1.record()
        torch.cuda.synchronize()
        print(f"cpw={os.environ.get('OV3D_BQ_CPW', 'default')} {name:22s} "
              f"{e0.elapsed_time(e1) / 20 * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
