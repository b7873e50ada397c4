"""Run the encoder-shape flash-attention forward (and backward with --bwd) a few times,
for rocprofv3 --pmc passes.  python tools/attn_pmc.py [--bwd] [--drop 0.1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--bwd", action="store_true")
    p.add_argument("--drop", type=float, default=0.1)
    p.add_argument("--iters", type=int, default=3)
    a = p.parse_args()
    ov3d_import.load()
    from ov3d_amd import attention as A
    B, H, L = 8, 4, 2048
    E = H * 64
    x = torch.randn(L, B, 3 * E, device="cuda", dtype=torch.bfloat16, requires_grad=a.bwd)
    for _ in range(a.iters):
        o = A.attention_packed([x], ((0, 0), (0, E), (0, 2 * E)), L, L, H, a.drop, site=1)
        if a.bwd:
            o.backward(torch.ones_like(o))
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
