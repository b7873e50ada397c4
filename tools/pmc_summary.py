"""Per-kernel (name, grid) mean of each PMC counter per dispatch from rocprofv3 --pmc
counter_collection CSVs.  python tools/pmc_summary.py out.json file.csv [file.csv ...]"""
import collections
import csv
import json
import sys


def main():
    out_path, paths = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        per = collections.defaultdict(float)   # (dispatch, kernel key, counter) -> value
        for r in csv.DictReader(open(path)):
            nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            grid = r.get("Grid_Size") or "%s,%s,%s" % (r.get("Grid_Size_X"), r.get("Grid_Size_Y"),
                                                        r.get("Grid_Size_Z"))
            key = "%s grid=%s" % (nm, grid)
            per[(r.get("Dispatch_Id", r.get("Correlation_Id")), key, r["Counter_Name"])] += \
                float(r["Counter_Value"])
        for (_, key, cn), v in per.items():
            acc[key][cn].append(v)
    res = {k: {cn: {"mean": sum(v) / len(v), "n": len(v)} for cn, v in sorted(c.items())}
           for k, c in sorted(acc.items())}
    json.dump(res, open(out_path, "w"), indent=1)
    for k, c in res.items():
        print(k[:100], {cn: "%.4g" % x["mean"] for cn, x in c.items()})


if __name__ == "__main__":
    main()
