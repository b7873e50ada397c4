"""Isolated timing of csrc/rows256.hip against gemm256 on the masked encoder's interim SA product
(2^18 x 256 rows, W 256 x 256): python tools/rows256_probe.py [reps]   (GPU; prints one JSON line;
run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE for the HBM bytes per launch)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def main():
    ov3d_import.load()
    from ov3d_amd import _native, gemm
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = 1 << 18
    x = torch.randn(M, 256, device=dev).to(torch.bfloat16)
    w = (0.06 * torch.randn(256, 256, device=dev)).to(torch.bfloat16)
    y = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
    res = {}

    def run_rows():
        _native.call("ov3d_rows256", x, 256, 256, 256, w, 256, y, 256, M, gemm._rows256_counters(dev), like=x)

    def run_g256():
        gemm.gemm256(x, w, out=y)

    for name, fn in (("rows256", run_rows), ("gemm256", run_g256)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[name] = {"us": round(us, 1), "tb_s": round(2 * M * 256 * 2 / us / 1e6, 2)}
    run_rows()
    a = y.clone()
    run_g256()
    res["bitexact"] = bool(torch.equal(a, y))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
