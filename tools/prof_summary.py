"""Summarise a rocprofv3 --kernel-trace --stats CSV (kernel_stats.csv): top kernels by total time."""
import csv
import sys


def short(n, w=60):
    n = n.replace('"', "")
    return n if len(n) <= w else n[: w - 3] + "..."


def main(path, steps=None, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print(f"total kernel time {tot/1e6:.2f} ms" + (f" ({tot/1e6/steps:.2f} ms/step over {steps} steps)" if steps else ""))
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'%':>6s}")
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{short(r['Name']):60s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.1f} {t/1e6:9.2f} {100*t/tot:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
