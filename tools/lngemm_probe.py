"""Per-launch time of the fused decoder boundary kernels (csrc/lngemm.hip) against the
resnorm + rows-GEMM launches they replace, back to back on one stream (HIP events), at the
decoder's R = 1024 rows: python tools/lngemm_probe.py"""
import ctypes
import sys

import torch

sys.path.insert(0, "tests")
from helpers import ov3d  # noqa: E402,F401
from ov3d_amd import _native, gemm  # noqa: E402
from ov3d_amd import attention as flash  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


def main():
    dev = torch.device("cuda:0")
    R, C = 1024, 256
    bf = torch.bfloat16
    flash.next_step(dev)
    seed = flash._seed(dev)
    src = torch.randn(R, C, device=dev)
    y = torch.randn(R, C, device=dev).to(bf)
    pos = torch.randn(R, C, device=dev)
    ga, ba, gb, bb = (torch.ones(C, device=dev), torch.zeros(C, device=dev),
                      torch.ones(C, device=dev), torch.zeros(C, device=dev))
    s = torch.empty(R, C, device=dev)
    mean, rstd = torch.empty(R, device=dev), torch.empty(R, device=dev)
    xa, xap = torch.empty(R, C, device=dev, dtype=bf), torch.empty(R, C, device=dev, dtype=bf)
    xb = torch.empty(R, C, device=dev)
    res = {}
    for N in (256, 768):
        W = (0.05 * torch.randn(N, C, device=dev)).to(bf)
        b = torch.zeros(N, device=dev, dtype=bf)
        o = torch.empty(R, N, device=dev, dtype=bf)
        arr = (gemm._LnProblem * 1)(gemm._LnProblem(W.data_ptr(), C, b.data_ptr(), o.data_ptr(), N, N, 1))

        def fused(wb=True):
            _native.call("ov3d_lngemm_fwd", R, src, 0, y, 0.1, seed, 3, ga, ba, pos, 0,
                         gb if wb else None, bb if wb else None, 1e-5, s, mean, rstd,
                         xa if wb else None, xap if wb else None, xb if wb else None, 0, 0, 0, 0,
                         1, ctypes.addressof(arr), 0, 0.0, None, 0, like=s)

        def rn_only():
            _native.call("ov3d_resnorm_fwd", R, C, src, 0, y, 1, 0.1, seed, 3, ga, ba, pos, 0, gb,
                         bb, 1e-5, s, mean, rstd, xa, xap, xb, 0, 0, 0, 0, like=s)

        def gemm_only():
            _native.call("ov3d_rows_gemm_act", R, N, C, xap, C, W, C, 1, b, 0, 0.0, None, 0, None,
                         0, o, N, like=s)

        res[f"fwd N={N} fused"] = timeit(fused)
        res[f"fwd N={N} fused, no extra outputs"] = timeit(lambda: fused(False))
        res[f"fwd N={N} resnorm"] = timeit(rn_only)
        res[f"fwd N={N} rows_gemm"] = timeit(gemm_only)
        res[f"fwd N={N} resnorm+rows_gemm"] = timeit(lambda: (rn_only(), gemm_only()))
    ds = torch.randn(R, C, device=dev)
    dxa = torch.randn(R, C, device=dev).to(bf)
    dxap = torch.randn(R, C, device=dev).to(bf)
    Wy = (0.05 * torch.randn(C, C, device=dev)).to(bf)
    dsrc, dpos = torch.empty(R, C, device=dev), torch.empty(R, C, device=dev)
    dy = torch.empty(R, C, device=dev, dtype=bf)
    dx = torch.empty(R, C, device=dev, dtype=bf)
    part = torch.empty(R // 8, 4, C, device=dev)

    def bfused():
        _native.call("ov3d_lngemm_bwd", R, s, mean, rstd, ds, dxa, dxap, None, 0, 0, 0, 0, ga,
                     None, 0.1, seed, 3, dsrc, dy, dpos, 0, part, 0, Wy, C, C, 0, 0.0, None, 0,
                     dx, C, like=s)

    def brn():
        _native.call("ov3d_resnorm_bwd", R, C, s, mean, rstd, ds, dxa, dxap, None, 0, 0, 0, 0, ga,
                     None, 0.1, seed, 3, dsrc, dy, 1, dpos, 0, part, R // 8, None, None, None,
                     None, 0, like=s)

    def bgemm():
        _native.call("ov3d_rows_gemm_act", R, C, C, dy, C, Wy, C, 0, None, 0, 0.0, None, 0, None,
                     0, dx, C, like=s)

    res["bwd fused"] = timeit(bfused)
    res["bwd resnorm"] = timeit(brn)
    res["bwd rows_gemm"] = timeit(bgemm)
    res["bwd resnorm+rows_gemm"] = timeit(lambda: (brn(), bgemm()))
    for k, v in res.items():
        print(f"{k:40s} {v:7.2f} us")
    # phase clocks of one forward launch per shape (s_memtime cycles, per wave)
    lib = _native.load()
    for N in (256, 768):
        W = (0.05 * torch.randn(N, C, device=dev)).to(bf)
        b = torch.zeros(N, device=dev, dtype=bf)
        o = torch.empty(R, N, device=dev, dtype=bf)
        arr = (gemm._LnProblem * 1)(gemm._LnProblem(W.data_ptr(), C, b.data_ptr(), o.data_ptr(), N, N, 1))
        bn = 64 if N <= 256 else 128
        nw = (R // (16 if bn == 64 else 32)) * (N // bn) * 8
        st = torch.zeros(nw * 8, dtype=torch.int64, device=dev)
        for arm in (True, False):
            lib.ov3d_lngemm_stamps_arm(st.data_ptr() if arm else None)
            _native.call("ov3d_lngemm_fwd", R, src, 0, y, 0.1, seed, 3, ga, ba, pos, 0, gb, bb,
                         1e-5, s, mean, rstd, xa, xap, xb, 0, 0, 0, 0, 1, ctypes.addressof(arr), 0,
                         0.0, None, 0, like=s)
            torch.cuda.synchronize()
        t8 = st.view(nw, 8).double()
        med = lambda x: x.median().item()   # noqa: E731
        print(f"N={N} phase cycles (median over waves): loads + W to LDS {med(t8[:, 5] - t8[:, 0]):.0f}, "
              f"row arithmetic {med(t8[:, 6] - t8[:, 5]):.0f}, row outputs {med(t8[:, 7] - t8[:, 6]):.0f}, "
              f"barrier {med(t8[:, 2] - t8[:, 1]):.0f}, mfma {med(t8[:, 3] - t8[:, 2]):.0f}, "
              f"epilogue {med(t8[:, 4] - t8[:, 3]):.0f}; total max {(t8[:, 4] - t8[:, 0]).max().item():.0f}")


if __name__ == "__main__":
    main()
