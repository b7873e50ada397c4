"""Instruction histogram of one kernel in a hipcc -S assembly file.
python tools/isa_hist.py file.s KERNEL_SYMBOL [--top 40]"""
import sys
from collections import Counter


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 45
    s = open(path).read()
    start = s.index(sym + ":")
    end = s.index(".Lfunc_end", start)
    c = Counter()
    for line in s[start:end].split("\n"):
        t = line.strip()
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        c[t.split()[0]] += 1
    print("instructions", sum(c.values()))
    for k, v in c.most_common(top):
        print(f"{v:6d} {k}")


if __name__ == "__main__":
    main()
