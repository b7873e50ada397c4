"""Average duration per (kernel, grid) from a rocprofv3 --kernel-trace CSV: the roofline
kernel's rocprof figure for one launch shape (the kernel-stats CSV averages all shapes).
python tools/trace_kernel_avg.py <run_kernel_trace.csv> [name-substring ...] > out.json
--steps K --marker NAME: only the last K steps, a step = the interval between consecutive
launches of the kernel whose name contains NAME (one launch per step), so warmup / capture
launches are left out and `per_step_us` is the steady-state cost per step."""
import argparse
import collections
import csv
import json
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("pats", nargs="*")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--marker", default="sa_dy8_kernel")
    a = ap.parse_args()
    pats = a.pats or ["attn_"]
    rows = list(csv.DictReader(open(a.csv)))
    lo = hi = None
    if a.steps:
        marks = sorted(int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"])
        if len(marks) > a.steps:
            lo, hi = marks[-a.steps - 1], marks[-1]
    d = collections.defaultdict(list)
    for r in rows:
        t0 = int(r["Start_Timestamp"])
        if lo is not None and not (lo <= t0 < hi):
            continue
        if any(p in r["Kernel_Name"] for p in pats):
            nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            key = "%s grid=(%s,%s,%s) wg=%s" % (nm.split("(")[0], r["Grid_Size_X"],
                                                r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
            d[key].append((int(r["End_Timestamp"]) - t0) / 1e3)
    nst = a.steps if lo is not None else None
    out = {k: {"launches": len(v), "avg_us": round(sum(v) / len(v), 2), "min_us": round(min(v), 2),
               "max_us": round(max(v), 2),
               **({"per_step_us": round(sum(v) / nst, 2)} if nst else {})}
           for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))}
    res = {"source": a.csv, "kernels": out}
    if nst:
        res["steps"] = nst
        res["window_us"] = (hi - lo) / 1e3
        res["kernel_us_per_step"] = round(sum(sum(v) for v in d.values()) / nst, 1)
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
