"""Per-step timeline of a rocprofv3 kernel trace (run_kernel_trace.csv).

Steps are delimited by the pre-encoder FPS launch (one per training step).  For
the last `--steps` complete steps prints wall span, GPU-busy time (union of
kernel intervals), idle time, the largest idle gaps with the kernels on either
side, and per-kernel-family time per step.

    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv --steps 8
"""
import argparse
import csv
import re
from collections import defaultdict


def family(name):
    n = name.replace('"', "")
    for pat, fam in [(r"fps_", "ov3d_fps"), (r"ball_query", "ov3d_ball_query"), (r"group_", "ov3d_group"),
                     (r"giou", "ov3d_giou"), (r"hungarian", "ov3d_hungarian"), (r"nms", "ov3d_nms"),
                     (r"attn_fwd", "attention fwd"), (r"bwd_kernel|bwd_preprocess", "attention bwd"),
                     (r"batch_norm", "batch_norm"), (r"layer_norm", "layer_norm"),
                     (r"^Cijk|gemm|Gemm", "GEMM (hipBLASLt)"), (r"reduce_kernel", "reduce"),
                     (r"elementwise|unrolled_elementwise", "elementwise"), (r"rocclr_copy", "copy"),
                     (r"rocclr_fill", "fill"), (r"cat|CatArray", "cat"), (r"index|gather|scatter", "index"),
                     (r"adam|Adam|multi_tensor", "optimizer"), (r"softmax|Softmax|log_softmax|nll", "softmax/nll")]:
        if re.search(pat, n):
            return fam
    return "other: " + n[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--gaps", type=int, default=12)
    ap.add_argument("--marker", default="fps_cull_kernel<20>")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    marks = [i for i, k in enumerate(ks) if a.marker in k[2]]
    if len(marks) < 2:
        raise SystemExit("not enough step markers")
    marks = marks[-(a.steps + 1):]
    n = len(marks) - 1
    span = ks[marks[-1]][0] - ks[marks[0]][0]
    busy, gaps = 0, []
    fam = defaultdict(int)
    end = ks[marks[0]][0]
    for i in range(marks[0], marks[-1]):
        s, e, name = ks[i]
        if s > end:
            gaps.append((s - end, ks[i - 1][2] if i else "", name))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        fam[family(name)] += e - s
    print(f"{n} steps: {span / n / 1e6:.3f} ms/step wall, {busy / n / 1e6:.3f} ms/step GPU busy, "
          f"{(span - busy) / n / 1e6:.3f} ms/step idle, {(marks[-1] - marks[0]) / n:.0f} kernels/step")
    print("largest idle gaps (us, per occurrence):")
    for g, prev, nxt in sorted(gaps, reverse=True)[: a.gaps]:
        print(f"  {g / 1e3:8.1f}  after {prev.replace(chr(34), '')[:60]}  before {nxt.replace(chr(34), '')[:60]}")
    tot_gap = sum(g for g, _, _ in gaps)
    small = sum(g for g, _, _ in gaps if g < 20000)
    print(f"gaps: {len(gaps) / n:.0f}/step, {tot_gap / n / 1e6:.3f} ms/step total, "
          f"{small / n / 1e6:.3f} ms/step in gaps < 20 us")
    print("kernel time per step by family (ms):")
    for f, t in sorted(fam.items(), key=lambda x: -x[1]):
        print(f"  {t / n / 1e6:8.3f}  {f}")


if __name__ == "__main__":
    main()
