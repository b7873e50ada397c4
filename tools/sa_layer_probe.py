"""Occupancy sweep of the fused SA layer kernels (csrc/sa_mlp.hip) at the BASELINE shape
(R = 8*2048*64 rows): workgroup count vs time and HBM rate.  python tools/sa_layer_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def t(f, n):
    """average microseconds of f() over n launches (after one warm-up)"""
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    ov3d_import.load()
    from ov3d_amd import _native as nat
    dev = torch.device("cuda")
    R, S = 8 * 2048 * 64, 64
    P = R // S
    for K, N in ((64, 128), (128, 256)):
        y = torch.randn(R, K, device=dev).bfloat16()
        sc = torch.rand(K, device=dev) + 0.5
        sh = torch.randn(K, device=dev) * 0.1
        W = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
        z = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
        yo = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        pmax = torch.empty(P, N, device=dev)
        pmin = torch.empty(P, N, device=dev)
        imax = torch.empty(P, N, device=dev, dtype=torch.uint8)
        imin = torch.empty(P, N, device=dev, dtype=torch.uint8)
        gsel = torch.randn(P, N, device=dev)
        cA, cB, cC = (torch.randn(N, device=dev) for _ in range(3))
        for nparts in (256, 512, 768, 1024, 2048):
            parts = torch.empty(nparts, 2, N, device=dev, dtype=torch.float64)
            res = []
            if K == 64:
                f = lambda: nat.call("ov3d_sa_layer_fwd", y, sc, sh, W, R, K, N, z, yo, parts, nparts, like=y)  # noqa
                us = t(f, 10)
                res.append(("store", us, R * (2 * K + 2 * K + 2 * N)))
            else:
                gam = torch.randn(N, device=dev)
                f = lambda: nat.call("ov3d_sa_layer_pool_fwd", y, sc, sh, W, R, K, N, S, None, pmax, pmin,  # noqa
                                     imax, imin, gam, parts, nparts, like=y)
                us = t(f, 10)
                res.append(("pool", us, R * (2 * K + 2 * K)))
                f = lambda: nat.call("ov3d_sa_layer_dy", y, sc, sh, W, R, K, N, S, gsel, imax, cA, cB, cC,  # noqa
                                     yo, nparts, like=y)
                us = t(f, 10)
                res.append(("dy", us, R * (2 * K + 2 * N)))
            print(f"K={K} N={N} nparts={nparts}: " + "  ".join(
                f"{m} {us:7.1f} us {b / us / 1e3:7.1f} GB/s" for m, us, b in res), flush=True)


if __name__ == "__main__":
    main()
