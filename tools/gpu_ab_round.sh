#!/bin/bash
# same-box A/B: the build at ab_base/ (a git worktree of an earlier commit, built in place) vs
# this tree, alternating, 30 steps each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do
  for side in base head; do
    if [ $side = base ]; then d=ab_base; else d=.; fi
    (cd $d && timeout -k 10 300 python bench.py --workload ${WORKLOAD:-sun} --steps 30 --warmup 5 --no-cpu-baseline > $OUT/ab_${side}_$i.json 2> $OUT/ab_${side}_$i.err) || { tail -3 $OUT/ab_${side}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab_${side}_$i.json')); print('$side', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
