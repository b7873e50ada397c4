"""Library GEMMs (aten mm / addmm / bmm / linear -> hipBLASLt) of one eager SUN training step:
operand shapes, kernel names and device time, largest first.  python tools/gemm_census.py"""
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
from glue_census import _kernel_events  # noqa: E402


def main():
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
        if ev.name not in ("aten::mm", "aten::addmm", "aten::bmm", "aten::linear", "aten::matmul",
                           "aten::_addmm_activation", "aten::baddbmm"):
            continue
        if ev.cpu_parent is not None and ev.cpu_parent.name in ("aten::linear", "aten::matmul"):
            continue
        ks = []
        _kernel_events(ev, ks)
        for k in ks:
            key = (ev.name, _where(ev), str(ev.input_shapes)[:80], k.name[:50])
            agg[key][0] += 1
            agg[key][1] += getattr(k, "duration", 0.0)
    tot = sum(v[1] for v in agg.values())
    print(f"library GEMM kernels in one eager step: {sum(v[0] for v in agg.values())}, {tot:.1f} us")
    for (name, frame, shp, kn), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{us:7.1f}us {c:3d}  {name:14s} {frame[-60:]}  {shp}  [{kn}]")


if __name__ == "__main__":
    main()
