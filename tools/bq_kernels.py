"""per-launch kernel times of tools/bq_time.py's trace (gpurun_out/bq_prof), by kernel and grid"""
import collections
import csv
import glob

f = glob.glob("gpurun_out/bq_prof/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "bq_" in n or "ball_query" in n:
        agg[(n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0], r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in agg.items():
    print(f"{n:42s} grid={g:>8s} n={len(v):3d} avg_us={sum(v) / len(v):8.2f}")
