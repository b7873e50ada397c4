"""Every long row-block GEMM launch (csrc/tilegemm.hip entry points) of one eager SUN training
step: entry point, leading int arguments (M, N, K / batch, M, N) and event-timed duration.
python tools/tile_census.py"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ov3d_import  # noqa: E402

NAMES = ["ov3d_tile_gemm", "ov3d_tile_gemm_act", "ov3d_tile_gemm2", "ov3d_tile_gemm_batched"]


def main():
    ov3d_import.load()
    from ov3d_amd import _native, gemm, synthetic
    from bench import build, default_args, train_step
    gemm.DEFER_WGRAD = True
    args = default_args()
    dev = torch.device("cuda")
    model, crit, opt = build(args, dev)
    batch = synthetic.make_batch(8, seed=1, device=dev)
    for _ in range(2):
        train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    _native.timing_enable(NAMES)
    train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    recs = _native.timing_collect()
    agg = collections.defaultdict(list)
    for n, rs in recs.items():
        for r in rs:
            agg[(n, r["shape"])].append(r["ms"] * 1e3)
    tot = 0.0
    for (n, shape), us in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(us)
        print(f"{sum(us):8.1f} us  {len(us):2d} x {sum(us) / len(us):6.1f}  {n:24s} {shape}")
    print(f"total {tot:.1f} us (eager, event-timed: includes launch gaps)")


if __name__ == "__main__":
    main()
