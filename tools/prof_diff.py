"""Per-kernel total-time difference of two rocprofv3 kernel_stats.csv files (B - A), largest
first: python tools/prof_diff.py A.csv B.csv [top]"""
import csv
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"].replace('"', "")
        out[n] = (float(r["TotalDurationNs"]) / 1e3, int(r["Calls"]))
    return out


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    ta, tb = sum(v[0] for v in a.values()), sum(v[0] for v in b.values())
    print(f"total us: A {ta:.0f}  B {tb:.0f}  B-A {tb - ta:+.0f}")
    keys = set(a) | set(b)
    rows = sorted(keys, key=lambda k: -abs(b.get(k, (0, 0))[0] - a.get(k, (0, 0))[0]))
    for k in rows[:top]:
        (xa, ca), (xb, cb) = a.get(k, (0, 0)), b.get(k, (0, 0))
        print(f"{xb - xa:+9.1f} us  A {xa:9.1f} ({ca:4d})  B {xb:9.1f} ({cb:4d})  {k[:100]}")


if __name__ == "__main__":
    main()
