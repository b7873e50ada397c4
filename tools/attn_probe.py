"""Time SDPA fwd+bwd on the 3DETR attention shapes for each ROCm flash-attention library
(aotriton / ck).  python tools/attn_probe.py"""
import time
import torch
import torch.nn.functional as F


def bench(B, H, Lq, Lk, d=64, drop=0.1, iters=20):
    dev = "cuda"
    q = torch.randn(B, H, Lq, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, H, Lk, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, H, Lk, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, H, Lq, d, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=drop)
        o.backward(g)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(iters):
        e[0].record()
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=drop)
        e[1].record()
        o.backward(g)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    return tf / iters * 1e3, tb / iters * 1e3


def bench_ov3d(B, H, Lq, Lk, d=64, drop=0.1, iters=20):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import ov3d_import
    ov3d_import.load()
    from ov3d_amd import attention as A
    dev = "cuda"
    E = H * d
    q = torch.randn(Lq, B, E, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(Lk, B, E, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(Lk, B, E, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(Lq, B, E, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        A.attention(q, k, v, H, drop, site=1).backward(g)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(iters):
        e[0].record()
        o = A.attention(q, k, v, H, drop, site=1)
        e[1].record()
        o.backward(g)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    return tf / iters * 1e3, tb / iters * 1e3


for shp in [(8, 4, 2048, 2048), (8, 4, 128, 2048), (8, 4, 128, 128)]:
    for drop in (0.0, 0.1):
        f, b = bench_ov3d(*shp, drop=drop)
        fl = 4.0 * shp[0] * shp[1] * shp[2] * shp[3] * 64
        print(f"ov3d      {shp} drop={drop}: fwd {f:7.1f} us ({fl / f / 1e6:6.1f} TF/s)  "
              f"bwd {b:7.1f} us ({2.5 * fl / b / 1e6:6.1f} TF/s)", flush=True)

for lib in ("aotriton",):
    try:
        torch.backends.cuda.preferred_rocm_fa_library(lib)
    except Exception as ex:
        print(lib, "unavailable", ex)
        continue
    for shp in [(8, 4, 2048, 2048), (8, 4, 128, 2048), (8, 4, 128, 128)]:
        for drop in (0.0, 0.1):
            try:
                f, b = bench(*shp, drop=drop)
                print(f"{lib:9s} {shp} drop={drop}: fwd {f:7.1f} us  bwd {b:7.1f} us", flush=True)
            except Exception as ex:
                print(lib, shp, drop, "error", repr(ex)[:200], flush=True)
