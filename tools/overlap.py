"""How much of each FPS launch overlaps other kernels (rocprofv3 kernel trace)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
fps = [k for k in ks if "fps_cull_kernel<20>" in k[2]]
others = [k for k in ks if "fps_cull_kernel<20>" not in k[2]]
for s, e, _ in fps[-8:]:
    cov, end = 0, s
    for os_, oe, _ in others:
        if oe <= s or os_ >= e:
            continue
        a, b = max(os_, end), min(oe, e)
        if b > a:
            cov += b - a
            end = b
    print(f"fps {(e - s) / 1e3:8.1f} us, overlapped by other kernels {cov / 1e3:8.1f} us")
