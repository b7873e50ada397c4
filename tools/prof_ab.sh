#!/bin/bash
# rocprofv3 kernel stats of bench.py for the ab_base/ build and this tree (same box), and a
# per-kernel comparison of the two (tools/prof_diff.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for side in base head; do
  if [ $side = base ]; then d=ab_base; else d=.; fi
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$side -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$side.json 2> $OUT/prof_$side.err) || { tail -5 $OUT/prof_$side.err; exit 1; }
done
python tools/prof_diff.py $(find $OUT/prof_base -name '*kernel_stats.csv' | head -1) $(find $OUT/prof_head -name '*kernel_stats.csv' | head -1)
