"""hipBLASLt (torch) time of the step's large M = 16384 GEMMs in several equivalent layouts.
python tools/gemm_layouts.py   (GPU)"""
import torch
import torch.nn.functional as F


def t(fn, iters=30):
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
    dev = "cuda"
    bf = torch.bfloat16
    for M, K, N in [(16384, 256, 2048), (16384, 256, 768), (16384, 256, 256), (16384, 2048, 256)]:
        x = torch.randn(M, K, device=dev, dtype=bf)
        W = torch.randn(N, K, device=dev, dtype=bf)
        Wt = W.t().contiguous()
        b = torch.randn(N, device=dev, dtype=bf)
        fl = 2.0 * M * N * K
        res = {
            "addmm(b, x, W.t())": t(lambda: torch.addmm(b, x, W.t())),
            "F.linear(x, W, b)": t(lambda: F.linear(x, W, b)),
            "x @ W.t()": t(lambda: x @ W.t()),
            "x @ Wt (KxN contig)": t(lambda: x @ Wt),
            "addmm(b, x, Wt)": t(lambda: torch.addmm(b, x, Wt)),
            "(W @ x.t()).t() [N x M]": t(lambda: W @ x.t()),
        }
        out_mb = M * N * 2 / 1e6
        print(f"M={M} K={K} N={N} ({fl / 1e9:.1f} GFLOP, out {out_mb:.0f} MB):")
        for k, us in res.items():
            print(f"   {k:28s} {us:7.1f} us  {fl / us / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
