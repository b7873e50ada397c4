"""Which python lines launch the most device ops in one eager training step (torch.profiler
with stacks).  python tools/op_census.py [--top 60]"""
import argparse
import os
import sys
from collections import Counter, defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ov3d_import  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    ov3d = ov3d_import.load()
    from ov3d_amd import synthetic
    from ov3d_amd.dataset_config import SunrgbdDatasetConfig
    from bench import build, default_args, train_step
    args = default_args()
    dev = torch.device("cuda")
    model, crit, opt = build(args, dev)
    batch = synthetic.make_batch(8, seed=1, device=dev)
    for _ in range(2):
        train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        train_step(model, crit, opt, batch, args, torch.bfloat16)
        torch.cuda.synchronize()
    by_line = Counter()
    by_op = Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.cpu_parent is not None and \
                ev.cpu_parent.name.startswith("aten::"):
            continue
        frame = "?"
        for f in ev.stack or []:
            if "ov3d" in f or "open-vocabulary" in f or "bench.py" in f or "torch/nn/utils" in f \
                    or "torch/optim" in f or "autograd" in f:
                frame = f
                break
        by_line[(ev.name, frame)] += 1
        by_op[ev.name] += 1
    print("top-level aten ops in one step:", sum(by_op.values()))
    for (name, frame), c in by_line.most_common(a.top):
        print(f"{c:5d}  {name:32s} {frame[-110:]}")


if __name__ == "__main__":
    main()
