"""Per-(kernel, grid) time of a rocprofv3 kernel trace: python tools/grid_breakdown.py trace.csv [steps] [regex]"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 16
pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if pat and not pat.search(n):
        continue
    m = re.search(r"::(\w+(<[^>]*>)?)\(", n)
    key = (m.group(1) if m else n[:50], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(k, len(v), f"{sum(v) / len(v) / 1e3:.1f}us", f"per-step={sum(v) / steps / 1e3:.1f}us")
