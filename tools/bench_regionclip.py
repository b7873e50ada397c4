"""Time the RegionCLIP ROI-feature path of one C5 training step (SURVEY §8d C5:
B=4 scenes/GPU, Q=128, L=8 decoder layers, 530x730 images, RN50x4 bf16).

    python tools/bench_regionclip.py [--B 4] [--Q 128] [--L 8] [--iters 5] [--stages]

Prints a JSON line: ms per call of region_features (all L*B*Q ROIs, one backbone
pass) and its algorithmic TFLOP/s; --stages adds per-stage HIP-event timings.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def flops(m, B, H, W, R):
    """matmul/conv FLOPs of the product formulation (backbone once, reassociated pool)."""
    tot = {"backbone": 0.0, "res5": 0.0, "attnpool": 0.0}
    hooks = []

    def conv_hook(name):
        def f(mod, inp, out):
            k = mod.kernel_size[0] * mod.kernel_size[1]
            tot[name] += 2.0 * out.numel() * mod.in_channels * k
        return f
    bb = m.backbone
    for n, mod in bb.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            hooks.append(mod.register_forward_hook(conv_hook("res5" if n.startswith("layer4") else "backbone")))
    with torch.no_grad():
        x = torch.zeros(1, 3, H, W, device="meta")
        r4 = bb.to("meta")(x)["res4"]
        bb.layer4(torch.zeros(1, r4.shape[1], 18, 18, device="meta"))
    for h in hooks:
        h.remove()
    tot["backbone"] *= B
    tot["res5"] *= R
    C = bb.attnpool.q_proj.in_features
    T = 82
    Hh = bb.attnpool.num_heads
    d = C // Hh
    out = bb.attnpool.c_proj.out_features
    tot["attnpool"] = R * (2.0 * C * C + 2 * Hh * d * C * 2 + 2 * Hh * T * C * 2 + 2 * C * out)
    return tot


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--B", type=int, default=4)
    p.add_argument("--Q", type=int, default=128)
    p.add_argument("--L", type=int, default=8)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--stages", action="store_true")
    a = p.parse_args()
    ov3d_import.load()
    from ov3d_amd import regionclip as rc
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    m, _ = rc.build_regionclip(compute_dtype=dt)
    fl = flops(rc.RegionCLIP(compute_dtype=dt), a.B, 530, 730, a.L * a.B * a.Q)
    m = m.to(dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    H, W = 530, 730
    img = (torch.rand(a.B, H * W * 3, generator=g) * 255).to(dev)
    x1 = torch.rand(a.L, a.B, a.Q, generator=g) * W * 0.8
    y1 = torch.rand(a.L, a.B, a.Q, generator=g) * H * 0.8
    bw = torch.rand(a.L, a.B, a.Q, generator=g) * W * 0.4 + 4
    bh = torch.rand(a.L, a.B, a.Q, generator=g) * H * 0.4 + 4
    boxes = torch.stack([x1, y1, (x1 + bw).clamp(max=W), (y1 + bh).clamp(max=H)], -1).to(dev)
    hs = [H] * a.B
    ws = [W] * a.B
    for i in range(2):
        t1 = time.perf_counter()
        m.region_features(img, hs, ws, boxes)
        torch.cuda.synchronize()
        print(f"warmup {i}: {time.perf_counter() - t1:.2f} s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        out = m.region_features(img, hs, ws, boxes)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    total = sum(fl.values())
    res = {"what": "RegionCLIP region_features (backbone once + all L*B*Q ROIs)",
           "B": a.B, "Q": a.Q, "L": a.L, "rois": a.L * a.B * a.Q, "dtype": a.dtype,
           "ms": round(ms, 3), "tflop": round(total / 1e12, 3),
           "tflops_achieved": round(total / (ms * 1e-3) / 1e12, 1),
           "flop_split_tflop": {k: round(v / 1e12, 3) for k, v in fl.items()},
           "finite": bool(torch.isfinite(out).all().item())}
    if a.stages:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        x = m._preprocess_1d(img, hs, ws, H, W)
        f = m._features(x)
        ev[1].record()
        P = m.pooler_resolution
        R = boxes.numel() // 4
        from ov3d_amd import _native
        roi = torch.empty((R, P, P, f.shape[-1]), dtype=f.dtype, device=dev)
        bx = boxes.reshape(-1, 4).contiguous()
        _native.call("ov3d_roi_align_fwd", f, int(f.dtype == torch.bfloat16), f.shape[0], f.shape[1],
                     f.shape[2], f.shape[3], bx, R, a.Q, a.B, 1.0 / 16, P, 0, 1, roi, like=f)
        ev[2].record()
        y = m._res_layer(roi, "layer4")
        ev[3].record()
        e4 = torch.cuda.Event(enable_timing=True)
        m._attnpool(y)
        e4.record()
        torch.cuda.synchronize()
        res["stages_ms"] = {"preprocess+backbone": round(ev[0].elapsed_time(ev[1]), 3),
                            "roi_align": round(ev[1].elapsed_time(ev[2]), 3),
                            "res5": round(ev[2].elapsed_time(ev[3]), 3),
                            "attnpool": round(ev[3].elapsed_time(e4), 3)}
        roi_bytes = roi.numel() * roi.element_size()
        res["roi_align_out_GBs"] = round(roi_bytes / (ev[1].elapsed_time(ev[2]) * 1e-3) / 1e9, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
