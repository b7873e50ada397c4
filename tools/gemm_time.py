"""Isolated per-call time of the long row-block GEMMs of the SUN step (profiles/r03_gemm_census.txt
shapes) on csrc/tilegemm.hip vs the library GEMM, same operands, back-to-back launches timed with
events; max |diff| against the fp32 product.  python tools/gemm_time.py [--reps 200]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

# (M, N, K, trans_b, bias): trans_b = 1 is F.linear(x (M,K), w (N,K)), 0 is dy (M,K) @ w (K,N)
SHAPES = [(16384, 768, 256, 1, 1), (16384, 256, 256, 1, 1), (16384, 256, 256, 1, 0),
          (16384, 128, 256, 1, 1), (16384, 256, 128, 1, 1), (16384, 2048, 256, 1, 1),
          (16384, 256, 256, 0, 0), (16384, 256, 768, 0, 0), (16384, 256, 128, 0, 0),
          (16384, 128, 256, 0, 0), (16384, 256, 2048, 0, 0), (8192, 1280, 256, 1, 0),
          (8192, 256, 1280, 0, 0), (8192, 256, 640, 0, 0)]


def timeit(fn, reps):
    """per-call device time: `reps` calls captured in one graph (no host launch overhead),
    the replay timed with events"""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (3 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--eager", action="store_true", help="no graph (profilers): 3 plain calls each")
    ap.add_argument("--only", default=None, help="comma list of shape indices")
    a = ap.parse_args()
    ov3d_import.load()
    from ov3d_amd import gemm
    gemm.TILE_GEMM = True
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    tot_lib = tot_own = 0.0
    for si, (M, N, K, tb, hb) in enumerate(SHAPES):
        if a.only is not None and str(si) not in a.only.split(","):
            continue
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) if tb else
             torch.randn(K, N, device=dev, generator=g)).div(K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16) if hb else None
        if tb:
            lib = lambda: torch.nn.functional.linear(x, w, b)
        else:
            lib = lambda: x @ w
        own = lambda: gemm.tile_gemm(x, w, b, trans_b=bool(tb))
        ref = (x.float() @ (w.float().t() if tb else w.float())) + (b.float() if hb else 0)
        d_own = (own().float() - ref).abs().max().item()
        d_lib = (lib().float() - ref).abs().max().item()
        if a.eager:
            for _ in range(3):
                lib()
                own()
            torch.cuda.synchronize()
            continue
        t_lib, t_own = timeit(lib, a.reps), timeit(own, a.reps)
        tot_lib += t_lib
        tot_own += t_own
        mb = (M * K + M * N) * 2 / 1e6
        print(f"M={M:6d} N={N:5d} K={K:5d} tb={tb} bias={hb}  lib {t_lib:7.2f} us  own {t_own:7.2f} us"
              f"  ({mb / t_own * 1e3:5.0f} GB/s of A+C)  maxdiff own {d_own:.3g} lib {d_lib:.3g}", flush=True)
    print(f"sum lib {tot_lib:.1f} us  own {tot_own:.1f} us")


if __name__ == "__main__":
    main()
