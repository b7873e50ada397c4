"""Which python lines (forward) / autograd nodes (backward) launch the most device kernels
in one eager training step (torch.profiler with stacks).
python tools/op_census.py [--top 60]"""
import argparse
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ov3d_import  # noqa: E402


def _kernels(ev):
    n = len(getattr(ev, "kernels", []) or [])
    for c in ev.cpu_children:
        n += _kernels(c)
    return n


def _where(ev):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    ov3d_import.load()
    from ov3d_amd import synthetic
    from bench import build, default_args, train_step
    from ov3d_amd import gemm
    gemm.DEFER_WGRAD = True   # as bench.py's captured step
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
    by_line = Counter()
    total = 0
    for ev in prof.events():
        if not ev.name.startswith("aten::") or (ev.cpu_parent is not None and
                                                ev.cpu_parent.name.startswith("aten::")):
            continue
        k = _kernels(ev)
        if k == 0:
            continue
        total += k
        shapes = str(ev.input_shapes)[:60] if ev.input_shapes else ""
        by_line[(ev.name, _where(ev), shapes)] += k
    print("device kernels launched by aten ops in one step:", total)
    for (name, frame, shp), c in by_line.most_common(a.top):
        print(f"{c:5d}  {name:28s} {frame[-90:]}  {shp}")


if __name__ == "__main__":
    main()
