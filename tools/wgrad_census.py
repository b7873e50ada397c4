"""List the deferred weight-gradient problems of one bench training step (R, N, K, nsplit,
GFLOP) in launch order.  python tools/wgrad_census.py [sun|scannet]   (GPU)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ov3d_import  # noqa: E402


def main():
    ov3d_import.load()
    import bench
    from ov3d_amd import _native, gemm, synthetic
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "sun"]
    args = bench.default_args(**wl["args"])
    ds = wl.get("dataset", "sunrgbd")
    model, crit, opt = bench.build(args, dev, dataset=ds)
    gemm.DEFER_WGRAD = True
    kw = {"num_points": wl["points"]} if "points" in wl else {}
    kw["use_color"] = bool(getattr(args, "use_color", False))
    batch = synthetic.make_batch(wl["batch"], seed=1, device=dev, dataset=ds, **kw)
    seen = []
    orig = _native.call

    def spy(name, *a, **k):
        if name == "ov3d_wgrad_group":
            import ctypes
            arr = ctypes.cast(a[0], ctypes.POINTER(gemm._WgProblem))
            for i in range(a[1]):
                p = arr[i]
                seen.append((p.R, p.N, p.K, p.nsplit, p.db is not None))
        return orig(name, *a, **k)

    _native.call = spy
    bench.train_step(model, crit, opt, batch, args, torch.bfloat16)
    torch.cuda.synchronize()
    _native.call = orig
    tot = 0.0
    rows = []
    for R, N, K, ns, hb in seen:
        gf = 2.0 * R * N * K / 1e9
        tot += gf
        rows.append({"R": R, "N": N, "K": K, "nsplit": ns, "bias": hb, "gflop": round(gf, 3)})
    print(json.dumps({"problems": len(rows), "gflop_total": round(tot, 2), "list": rows}))


if __name__ == "__main__":
    main()
