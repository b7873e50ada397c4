#!/bin/bash
# Selected GPU tests (-k expression in $1), then the C4 bench; each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$1" > $OUT/sel.log 2>&1
rc=$?; tail -25 $OUT/sel.log; [ $rc -eq 0 ] || exit $rc
if [ "${2:-}" != "" ]; then
  timeout -k 10 300 python bench.py --workload $2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/sel_bench.json 2> $OUT/sel_bench.err
  rc=$?; cat $OUT/sel_bench.json; tail -3 $OUT/sel_bench.err; exit $rc
fi
