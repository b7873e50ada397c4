"""Split-count sweep of the one-launch weight gradient (csrc/wgrad.hip) on the short-R
(decoder: 1024 rows) shapes, against hipBLASLt mm + bias sum.  python tools/wgrad_split_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402
from wgrad_probe import t  # noqa: E402


def main():
    ov3d_import.load()
    from ov3d_amd import gemm
    orig = gemm._wg_splits
    for R, N, K in [(1024, 256, 256), (1024, 512, 256), (1024, 768, 256), (1024, 1280, 256),
                    (8192, 256, 256), (16384, 256, 256), (16384, 768, 256)]:
        dy = torch.randn(R, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
        res = []
        for ns in (1, 2, 4, 8, 16, 32):
            gemm._wg_splits = lambda R_, N_, K_, ns=ns: ns
            res.append((ns, t(lambda: gemm.fused_weight_grad(dy, x, True))))
        gemm._wg_splits = orig
        cur = t(lambda: gemm.fused_weight_grad(dy, x, True))
        mm = t(lambda: (torch.mm(dy.t(), x, out_dtype=torch.float32), torch.sum(dy, 0, dtype=torch.float32)))
        print(f"R={R:6d} N={N:4d} K={K:4d}: current {cur:6.1f} | " +
              " ".join(f"ns{n}={v:5.1f}" for n, v in res) + f" | mm+sum {mm:5.1f}", flush=True)


if __name__ == "__main__":
    main()
