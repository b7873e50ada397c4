"""Which python lines (forward) / autograd nodes (backward) launch the torch glue kernels
(fills, copies, casts, cats, elementwise) in one eager training step, with their device time.
python tools/glue_census.py [--workload sunrgbd|scannet]"""
import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ov3d_import  # noqa: E402


def _where(ev):
    """the product source line (forward) or the autograd node (backward) of a profiler event"""
    for f in ev.stack or []:
        if "ov3d" in f or "open-vocabulary" in f or "bench.py" in f or "torch/nn/utils" in f \
                or "torch/optim" in f:
            return f
    p = ev.cpu_parent
    while p is not None:
        if p.name.startswith("autograd::engine::evaluate_function"):
            return p.name.split(":")[-1].strip()
        p = p.cpu_parent
    return "?"

GLUE = ("at::native", "rocclr", "Memcpy", "Memset", "elementwise", "Fill", "Copy", "copy")


def _kernel_events(ev, out):
    for k in getattr(ev, "kernels", []) or []:
        out.append(k)
    for c in ev.cpu_children:
        _kernel_events(c, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    ov3d_import.load()
    from ov3d_amd import gemm, synthetic
    from bench import build, default_args, train_step
    gemm.DEFER_WGRAD = True
    args = default_args()
    dev = torch.device("cuda")
    model, crit, opt = build(args, dev)
    batch = synthetic.make_batch(8, seed=1, device=dev)
    for _ in range(2):
        train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        train_step(model, crit, opt, batch, args, torch.bfloat16)
        torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if not ev.name.startswith("aten::") or (ev.cpu_parent is not None and
                                                ev.cpu_parent.name.startswith("aten::")):
            continue
        ks = []
        _kernel_events(ev, ks)
        for k in ks:
            if not any(g in k.name for g in GLUE):
                continue
            shapes = str(ev.input_shapes)[:70] if ev.input_shapes else ""
            key = (ev.name, _where(ev), shapes, k.name[:60])
            agg[key][0] += 1
            agg[key][1] += getattr(k, "duration", 0.0)
    tot = sum(v[1] for v in agg.values())
    print(f"glue kernels in one eager step: {sum(v[0] for v in agg.values())}, {tot:.1f} us")
    for (name, frame, shp, kn), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{us:7.1f}us {c:3d}  {name:22s} {frame[-80:]}  {shp}  [{kn}]")


if __name__ == "__main__":
    main()
