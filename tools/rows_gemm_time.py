"""rowsgemm vs the library GEMM on the decoder / encoder row shapes.
python tools/rows_gemm_time.py"""
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
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ov3d_import.load()
    from ov3d_amd import gemm
    bf = torch.bfloat16
    for M, N, K in ((1024, 256, 256), (1024, 512, 256), (1024, 256, 512), (4096, 256, 256),
                    (16384, 256, 256), (16384, 768, 256), (16384, 128, 256), (16384, 256, 128)):
        a = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf)
        wt = torch.randn(K, N, device="cuda", dtype=bf)
        b = torch.randn(N, device="cuda", dtype=bf)
        gemm.ROWS_GEMM_MAX_M = 1 << 30
        r = [t(lambda: torch.nn.functional.linear(a, w, b)), t(lambda: gemm.rows_gemm(a, w, b)),
             t(lambda: a @ wt), t(lambda: gemm.rows_gemm(a, wt, trans_b=False))]
        print(f"M={M:6d} N={N:4d} K={K:4d}: linear lib {r[0]:6.2f} us rows {r[1]:6.2f} us | "
              f"dgrad lib {r[2]:6.2f} us rows {r[3]:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
