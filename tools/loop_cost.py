"""Per-block instruction issue cost of a kernel's loop bodies in a hipcc -S file.

    python tools/loop_cost.py file.s KERNEL_SYMBOL

Prints every basic block that belongs to a loop (the compiler's "in Loop: Header=" notes)
with its instruction count and an estimated vector issue cost in cycles for one wave on one
SIMD (MI355X_MICROARCH.md 'Per-instruction cycle constants': transcendental 8, plain VALU 4,
quarter-rate integer multiplies 16, MFMA 8 of issue, s_nop N = 4(N+1)); scalar, LDS and memory
instructions are listed by count only.  Rarely taken blocks (tails, rescales) are shown
separately so the steady-state cost can be read off.
"""
import re
import sys
from collections import Counter, OrderedDict

TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32")
QUARTER = ("v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mad_i64_i32", "v_mul_hi_i32")


def cost(op, line):
    if op.startswith("v_mfma"):
        return 8
    if op.startswith(TRANS):
        return 8
    if op.startswith(QUARTER):
        return 16
    if op == "s_nop":
        n = int(line.split()[1], 0)
        return 4 * (n + 1)
    if op.startswith("v_"):
        return 4
    return 0


def main():
    path, sym = sys.argv[1], sys.argv[2]
    s = open(path).read()
    start = s.index(sym + ":")
    end = s.index(".Lfunc_end", start)
    blocks = OrderedDict()
    cur, inloop = "entry", False
    for line in s[start:end].split("\n"):
        t = line.strip()
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?\s*(;.*)?$", t)
        if m:
            cur = m.group(1)
            note = m.group(2) or ""
            inloop = "Loop" in note
            continue
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        if not inloop:
            continue
        op = t.split()[0]
        b = blocks.setdefault(cur, {"n": 0, "cyc": 0, "ops": Counter()})
        b["n"] += 1
        b["cyc"] += cost(op, t)
        b["ops"][op] += 1
    tot_n = tot_c = 0
    for name, b in blocks.items():
        kinds = Counter()
        for op, c in b["ops"].items():
            k = ("mfma" if op.startswith("v_mfma") else "trans" if op.startswith(TRANS) else
                 "quarter" if op.startswith(QUARTER) else "ds" if op.startswith("ds_") else
                 "vmem" if op.startswith(("global_", "buffer_")) else "valu" if op.startswith("v_") else
                 "salu")
            kinds[k] += c
        print(f"{name:12s} n={b['n']:4d} issue~{b['cyc']:5d} cyc  " +
              " ".join(f"{k}={v}" for k, v in sorted(kinds.items())))
        tot_n += b["n"]
        tot_c += b["cyc"]
    print(f"all loop blocks: n={tot_n} issue~{tot_c} cyc")


if __name__ == "__main__":
    main()
