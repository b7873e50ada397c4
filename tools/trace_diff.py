"""Per-kernel per-step difference of two steady-state traces (tools/trace_kernel_avg.py output):
python tools/trace_diff.py base.json new.json [--top 14]"""
import json
import sys


def main():
    a, b = (json.load(open(p)) for p in sys.argv[1:3])
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 14
    print("window_us", a["window_us"], "->", b["window_us"], " kernel_us_per_step",
          a["kernel_us_per_step"], "->", b["kernel_us_per_step"])
    ka, kb = a["kernels"], b["kernels"]
    rows = []
    for n in set(ka) | set(kb):
        x, y = ka.get(n, {}), kb.get(n, {})
        steps_a = x.get("launches", 0) * x.get("per_step_us", 0) / max(x.get("avg_us", 1e-9) * 1.0, 1e-9) if x else 0
        rows.append((y.get("per_step_us", 0) - x.get("per_step_us", 0), n[:80],
                     x.get("per_step_us", 0), y.get("per_step_us", 0)))
    rows.sort()
    for r in rows[:top] + [None] + rows[-top:]:
        print("-" * 20 if r is None else "%8.1f  %-80s %8.1f -> %8.1f" % r)


if __name__ == "__main__":
    main()
