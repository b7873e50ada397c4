"""Per-kernel per-step difference of two steady-trace summaries (tools/trace_kernel_avg.py output):
    python tools/trace_cmp.py A.json B.json [--top 25] [--grep attn]"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--grep", default="")
    o = ap.parse_args()
    a = json.load(open(o.a))["kernels"]
    b = json.load(open(o.b))["kernels"]

    def short(n):
        g = n.split("grid=")[1].split(" ")[0] if "grid=" in n else ""
        return n.split(" grid")[0].replace("(anonymous namespace)::", "")[:64] + " " + g
    rows = []
    for n in set(a) | set(b):
        if o.grep and o.grep not in n:
            continue
        x = a.get(n, {}).get("per_step_us", 0.0)
        y = b.get(n, {}).get("per_step_us", 0.0)
        rows.append((y - x, x, y, n))
    rows.sort()
    sel = rows if o.grep else rows[:o.top] + rows[-o.top // 2:]
    for d, x, y, n in sel:
        print("%8.1f %8.1f %8.1f %s" % (d, x, y, short(n)))
    print("total %.1f -> %.1f us per step" % (sum(v["per_step_us"] for v in a.values()),
                                              sum(v["per_step_us"] for v in b.values())))


if __name__ == "__main__":
    main()
