"""Step time of the captured SUN step with and without the side-stream sampling plan work
(diagnostic only: without it every step reuses the first plan).  Separates the graph's own
time from its contention with the plan."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def main():
    ov3d_import.load()
    import bench
    from ov3d_amd import gemm, synthetic
    from ov3d_amd.graphs import StepGraph
    dev = torch.device("cuda", 0)
    args = bench.default_args()
    model, crit, opt = bench.build(args, dev)
    gemm.DEFER_WGRAD = True
    pool = [synthetic.make_batch(8, seed=i, device=dev) for i in range(4)]
    g = StepGraph(model, crit, opt, pool[0], amp_dtype=torch.bfloat16, clip=args.clip_gradient)
    res = {}
    for mode in ("plan", "no_plan", "plan", "no_plan"):
        if mode == "no_plan":
            g._sample = lambda pc: g.plan_cur      # no side-stream work at all
        else:
            g.__dict__.pop("_sample", None)
        for i in range(5):
            g.step(pool[i % 4], pool[(i + 1) % 4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 30
        for i in range(n):
            g.step(pool[i % 4], pool[(i + 1) % 4])
        torch.cuda.synchronize()
        res.setdefault(mode, []).append(round((time.perf_counter() - t0) * 1e3 / n, 3))
    res["split"] = g.split
    print(json.dumps(res))




def host_launch_cost():
    """host time of graph.replay() (the launch call only) vs the GPU time of the step"""
    ov3d_import.load()
    import bench
    from ov3d_amd import gemm, synthetic
    from ov3d_amd.graphs import StepGraph
    dev = torch.device("cuda", 0)
    args = bench.default_args()
    model, crit, opt = bench.build(args, dev)
    gemm.DEFER_WGRAD = True
    pool = [synthetic.make_batch(8, seed=i, device=dev) for i in range(2)]
    g = StepGraph(model, crit, opt, pool[0], amp_dtype=torch.bfloat16, clip=args.clip_gradient)
    for i in range(3):
        g.step(pool[i % 2], pool[(i + 1) % 2])
    torch.cuda.synchronize()
    out = {}
    for name, gr in (("graph_A", g.graph), ("graph_B", g.graph2)):
        if gr is None:
            continue
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gr.replay()
            ts.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        out[name + "_host_ms"] = round(sorted(ts)[2], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "host":
        host_launch_cost()
    else:
        main()
