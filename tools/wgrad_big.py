"""Time the weight gradient dW = dy^T x of the ScanNet (C4) set-abstraction layers (R = 2^20
and 2^18 rows) on the grouped stream-K kernel (ov3d_wgrad_group, one problem), the
single-problem kernel (ov3d_wgrad) and the split-K bmm path (gemm.weight_grad)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402

ov3d_import.load()
from ov3d_amd import _native, gemm  # noqa: E402
from bench_kernels import timeit  # noqa: E402


def grouped(dy, x, dw):
    R, N = dy.shape
    K = x.shape[1]
    p = gemm._WgProblem(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), R, N, K,
                        gemm._wg_group_splits(R), dw.data_ptr(), dw.stride(0), None)
    arr = (gemm._WgProblem * 1)(p)
    n = _native.load().ov3d_wgrad_group_workspace(ctypes.addressof(arr), 1)
    ws = torch.empty((max(n, 1),), dtype=torch.float32, device=dy.device)
    return lambda: _native.call("ov3d_wgrad_group", ctypes.addressof(arr), 1, ws, like=ws)


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for R, N, K in ((1 << 20, 256, 128), (1 << 20, 128, 64), (1 << 20, 64, 6), (1 << 18, 256, 259),
                    (1 << 18, 256, 256)):
        dy = torch.randn(R, N, device=dev).to(torch.bfloat16)
        x = torch.randn(R, K, device=dev).to(torch.bfloat16)
        dw = torch.empty(N, K, device=dev)
        gf = 2.0 * R * N * K / 1e9
        gb = R * (N + K) * 2 / 1e9
        t = {"grouped": timeit(grouped(dy, x, dw), reps=10),
             "single": timeit(lambda: gemm.fused_weight_grad(dy, x, bias=False), reps=10),
             "bmm": timeit(lambda: gemm.weight_grad(dy, x), reps=10)}
        ref = (dy.float().t() @ x.float())
        grouped(dy, x, dw)()
        err = float((dw - ref).abs().max() / ref.abs().max())
        res[f"R{R}_N{N}_K{K}"] = {k: {"us": round(v * 1e3, 1), "TF/s": round(gf / v, 1),
                                      "GB/s": round(gb / v * 1e3, 0)} for k, v in t.items()}
        res[f"R{R}_N{N}_K{K}"]["rel_err_grouped"] = err
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
