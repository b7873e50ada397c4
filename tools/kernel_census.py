"""Kernel launches per training step by kernel type (rocprofv3 kernel trace), using one
per-step marker kernel.  python tools/kernel_census.py trace.csv [--marker NAME] [--top 45]"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="fps_cull_kernel<2>")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--by-time", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    marks = [i for i, k in enumerate(ks) if a.marker in k[2]]
    lo, hi = marks[-(a.steps + 1)], marks[-1]
    cnt, tm = defaultdict(int), defaultdict(int)
    pat = (r"(\w+Functor\w*|\w+_kernel_cuda\w*|launch_clamp_scalar|direct_copy\w*|"
           r"(?:anonymous namespace\)::)\w+|^\w+|Cijk\w{0,30})")
    for s, e, name in ks[lo:hi]:
        m = re.findall(pat, name)
        key = name[:55] + " | " + " ".join(dict.fromkeys(m[:3]))[:70]
        cnt[key] += 1
        tm[key] += e - s
    print(f"kernels/step {sum(cnt.values()) / a.steps:.0f}, kernel time/step "
          f"{sum(tm.values()) / a.steps / 1e6:.2f} ms")
    order = (lambda k: -tm[k]) if a.by_time else (lambda k: -cnt[k])
    for k in sorted(cnt, key=order)[: a.top]:
        print(f"{cnt[k] / a.steps:7.1f}/step {tm[k] / a.steps / 1e3:8.1f} us/step  {k}")


if __name__ == "__main__":
    main()
