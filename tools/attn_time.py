"""Time the HIP flash attention on the encoder shape (B=8, H=4, L=2048, d=64) and the decoder
cross shape (128 queries x 2048 keys), forward and backward, with and without dropout.
python tools/attn_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def run(Lq, Lk, drop, iters=20):
    from ov3d_amd import attention as A
    B, H = 8, 4
    E = H * 64
    q = torch.randn(Lq, B, E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    kv = torch.randn(Lk, B, 2 * E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(Lq, B, E, device="cuda", dtype=torch.bfloat16)
    spec = ((0, 0), (1, 0), (1, E))
    for _ in range(3):
        o = A.attention_packed([q, kv], spec, Lq, Lk, H, drop, site=1)
        o.backward(g)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(iters):
        ev[0].record()
        o = A.attention_packed([q, kv], spec, Lq, Lk, H, drop, site=1)
        ev[1].record()
        o.backward(g)
        ev[2].record()
        torch.cuda.synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    fl = 4 * B * H * Lq * Lk * 64
    tf, tb = tf / iters * 1e3, tb / iters * 1e3
    print(f"Lq={Lq} Lk={Lk} p={drop}: fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF/s)  "
          f"bwd {tb:7.1f} us ({2.5 * fl / tb / 1e6:6.1f} TF/s)", flush=True)


def main():
    ov3d_import.load()
    for Lq, Lk in ((2048, 2048), (128, 2048)):
        for p in (0.0, 0.1):
            run(Lq, Lk, p)


if __name__ == "__main__":
    main()
