"""Weight-gradient variants on the hot path's linear shapes: split-K bmm + sum (gemm.py),
plain GEMM with fp32 output, and the bias reduction.  python tools/wgrad_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def t(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ov3d_import.load()
    from ov3d_amd import gemm
    for R, N, K in [(16384, 768, 256), (16384, 256, 256), (16384, 128, 256), (16384, 256, 128),
                    (8192, 256, 256), (8192, 640, 256), (8192, 3, 256), (1024, 256, 256), (1024, 768, 256), (1000, 12, 100)]:
        dy = torch.randn(R, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
        a = t(lambda: gemm.weight_grad(dy, x))
        b = t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        c = t(lambda: torch.sum(dy, dim=0, dtype=torch.float32))
        d = t(lambda: torch.mm(dy.t(), x))
        f = t(lambda: gemm.fused_weight_grad(dy, x, True))
        dw, db = gemm.fused_weight_grad(dy, x, True)
        ref = dy.float().t() @ x.float()
        err = ((dw - ref).norm() / ref.norm()).item()
        berr = ((db - dy.float().sum(0)).norm() / dy.float().sum(0).norm()).item()
        print(f"R={R:6d} N={N:4d} K={K:4d}: splitK {a:6.1f} us  mm_f32out {b:6.1f} us  "
              f"bias_sum {c:5.1f} us | fused {f:6.1f} us (err {err:.1e}, {berr:.1e})", flush=True)


if __name__ == "__main__":
    main()
