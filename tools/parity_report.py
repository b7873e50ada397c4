"""Print the error distribution of the product against the float64 reference fixtures
(tests/full_fixture.py) for fp32 and bf16 autocast: quantiles and worst entries per group.
python tools/parity_report.py [--amp bf16|fp32]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import full_fixture as F  # noqa: E402


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--amp", default="bf16")
    a.add_argument("--floor", type=float, default=1e-4)
    args = a.parse_args()
    amp = torch.bfloat16 if args.amp == "bf16" else None
    for name, ds in F.CASES:
        reps = {}
        for mode in ("hip", "torch") if amp is not None else ("hip",):
            if mode == "torch":
                with F.torch_bf16_path():
                    rep = F.run(name, ds, torch.device("cuda", 0), amp=amp, grad_floor=args.floor)
            else:
                rep = F.run(name, ds, torch.device("cuda", 0), amp=amp, grad_floor=args.floor)
            reps[mode] = rep
            print("==", name, args.amp, mode)
            for g, v in rep.items():
                e = np.array([x for x, _ in v])
                print("  %-9s n=%4d  q50 %.2e q90 %.2e q99 %.2e max %.2e" % (
                    g, len(e), *np.quantile(e, [0.5, 0.9, 0.99]), e.max()),
                    [("%.2e" % x, k) for x, k in v[:3]])
        if len(reps) == 2:
            print("== hip / torch, largest ratios (hip err, torch err, key)")
            for g in reps["hip"]:
                t = {k: x for x, k in reps["torch"][g]}
                r = sorted(((x / max(t[k], 1e-3), x, t[k], k) for x, k in reps["hip"][g]),
                           reverse=True)[:6]
                print("  %-9s" % g, ["%.1fx %.1e/%.1e %s" % q for q in r])


if __name__ == "__main__":
    main()
