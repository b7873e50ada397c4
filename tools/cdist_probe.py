"""Which arithmetic gives torch.cdist's matmul-form squared distances bit for bit on this
device (transformer.euclid_sq)?  Builds on tools/cdist/libcdist_probe.so (hipcc, see the .hip)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "open-vocabulary-3d-object-detection_amd", ".."))
sys.path.insert(0, "tests")
from helpers import ov3d  # noqa: E402,F401
from ov3d_amd.transformer import euclid_sq  # noqa: E402


def main():
    lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "cdist", "libcdist_probe.so"))
    dev = torch.device("cuda:0")
    for trial, (B, L, scale) in enumerate([(8, 2048, 3.0), (8, 1024, 3.0), (2, 2048, 0.5)]):
        g = torch.Generator(device=dev).manual_seed(trial)
        x = (torch.rand(B, L, 3, device=dev, generator=g) * 2 - 1) * scale
        ref = euclid_sq(x)
        xn = x.pow(2).sum(-1).contiguous()
        for mode, name in ((0, "fma chain"), (1, "mfma 16x16x4 x2"), (2, "mul + add chain")):
            out = torch.empty(B, L, L, device=dev)
            rc = lib.cdist_probe(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(xn.data_ptr()), B, L,
                                 mode, ctypes.c_void_p(out.data_ptr()))
            torch.cuda.synchronize()
            neq = (out != ref).sum().item()
            print(f"B={B} L={L} scale={scale} {name:18s} rc={rc} mismatches {neq} of {out.numel()}"
                  f" max|d| {(out - ref).abs().max().item():.3g}")


if __name__ == "__main__":
    main()
