"""Average duration per (kernel, grid) from a rocprofv3 --kernel-trace CSV: the roofline
kernel's rocprof figure for one launch shape (the kernel-stats CSV averages all shapes).
python tools/trace_kernel_avg.py <run_kernel_trace.csv> [name-substring ...] > out.json"""
import collections
import csv
import json
import sys


def main():
    path, pats = sys.argv[1], sys.argv[2:] or ["attn_"]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if any(p in r["Kernel_Name"] for p in pats):
            nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            key = "%s grid=(%s,%s,%s) wg=%s" % (nm.split("(")[0], r["Grid_Size_X"],
                                                r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {k: {"launches": len(v), "avg_us": round(sum(v) / len(v), 2), "min_us": round(min(v), 2),
               "max_us": round(max(v), 2)} for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))}
    json.dump({"source": path, "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
