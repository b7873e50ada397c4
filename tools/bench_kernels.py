"""Per-kernel microbenchmarks of libov3d_hip.so at the BASELINE shapes (HIP events,
median of R launches) with the algorithmic-bytes roofline of SURVEY.md §8d."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import nms, pointnet2_utils as pu, synthetic  # noqa: E402
from ov3d_amd.box_util import giou3d_raw  # noqa: E402

HBM = 8000.0


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda", 0)
    res = {}
    batch = synthetic.make_batch(8, seed=1, device=dev)
    xyz = batch["point_clouds"]
    B, N = xyz.shape[:2]
    for (n, m) in ((N, 2048), (2048, 128)):
        x = xyz if n == N else pu.furthest_point_sample_gather(xyz, 2048)[1]
        ms = timeit(lambda: pu.furthest_point_sample_gather(x, m))
        algo = B * m * n * 16.0
        res[f"fps_{n}_{m}"] = {"ms": ms, "GB/s(algo)": algo / ms / 1e6, "frac": algo / ms / 1e6 / HBM,
                               "us_per_iter": ms * 1e3 / m}
    _, nx = pu.furthest_point_sample_gather(xyz, 2048)
    ms = timeit(lambda: pu.ball_query(0.2, 64, xyz, nx))
    algo = B * 2048 * N * 12.0
    res["ball_query_0.2_64"] = {"ms": ms, "GB/s(algo)": algo / ms / 1e6, "frac": algo / ms / 1e6 / HBM}
    grouper = pu.QueryAndGroup(0.2, 64, ret_grouped_xyz=True, normalize_xyz=True)
    idx = pu.ball_query(0.2, 64, xyz, nx)
    out = torch.empty(B, 3, 2048, 64, device=dev)
    from ov3d_amd import _native as nat
    ms = timeit(lambda: nat.call("ov3d_group_fwd", xyz, nx, None, idx, B, 0, N, 2048, 64, 0.2, 1, out, like=xyz))
    algo = out.numel() * 4 + idx.numel() * 4
    res["group_fwd_xyz"] = {"ms": ms, "GB/s(algo)": algo / ms / 1e6, "frac": algo / ms / 1e6 / HBM}
    c1 = batch["gt_box_corners"].repeat(8, 2, 1, 1)[:, :128].contiguous()
    c2 = batch["gt_box_corners"].repeat(8, 1, 1, 1).contiguous()
    nums = batch["gt_box_present"].sum(1).int().repeat(8)
    ms = timeit(lambda: giou3d_raw(c1, c2, nums, 0, True))
    pairs = c1.shape[0] * 128 * 64
    res["giou_8x8x128x64"] = {"ms": ms, "pairs/us": pairs / ms / 1e3,
                              "GB/s(algo)": pairs * (2 * 96 + 4) / ms / 1e6}
    boxes = nms.nms_boxes_from_corners(c1[:8], torch.rand(8, 128, device=dev), batch["gt_box_sem_cls_label"][:, :1].repeat(1, 128))
    ms = timeit(lambda: nms.nms3d_batched(boxes, 0.25))
    res["nms_8x128"] = {"ms": ms}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
