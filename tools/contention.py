"""Does the side-stream FPS (8 workgroups holding 8 CUs for ~2.5 ms) slow the step's
kernels?  Times a few step kernels alone and while an FPS launch runs on another stream."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import attention as A, pointnet2_utils as pu, synthetic  # noqa: E402


def timed(fn, n):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def main():
    dev = torch.device("cuda", 0)
    xyz = synthetic.make_batch(8, seed=1, device=dev)["point_clouds"][..., :3].contiguous()
    qkv = (torch.randn(2048, 8, 768, device=dev)).to(torch.bfloat16)
    q, k, v = (t.contiguous() for t in qkv.chunk(3, dim=-1))
    x = torch.randn(16384, 256, device=dev).to(torch.bfloat16)
    w = torch.randn(768, 256, device=dev).to(torch.bfloat16)
    from ov3d_amd.gemm import rows_linear
    qd = (torch.randn(128, 8, 256, device=dev)).to(torch.bfloat16)
    xr = torch.randn(1024, 256, device=dev).to(torch.bfloat16)
    wr = torch.randn(256, 256, device=dev)
    br = torch.randn(256, device=dev)
    kern = {"attn_fwd_L2048": lambda: A.attention(q, k, v, 4, dropout_p=0.1, site=1),
            "gemm_16384x256x768": lambda: torch.mm(x, w.t()),
            "dec_cross_attn_128x2048": lambda: A.attention(qd, k, v, 4, dropout_p=0.1, site=2),
            "dec_self_attn_128": lambda: A.attention(qd, qd, qd, 4, dropout_p=0.1, site=3),
            "rows_linear_1024x256": lambda: rows_linear(xr, wr, br)}
    side = torch.cuda.Stream()
    res = {}
    for name, fn in kern.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        alone = timed(fn, 20)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            pu.furthest_point_sample_gather(xyz, 2048)   # ~2.5 ms on 8 CUs
        with_fps = timed(fn, 20)
        torch.cuda.synchronize()
        res[name] = {"alone_us": round(alone, 1), "beside_fps_us": round(with_fps, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    with torch.no_grad():
        main()
