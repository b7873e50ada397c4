#!/bin/bash
# bench (with cpu_baseline) + rocprofv3 kernel-trace stats of the same command; each GPU
# step under its own time limit, chained so the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03}
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -5 $OUT/prof_$TAG.err; exit 1; }
  cat $OUT/prof_bench_$TAG.json
fi
echo done
