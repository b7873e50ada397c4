#!/bin/bash
# glue census (SUN eager step) and a steady-state kernel trace of the C4 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03h}
timeout -k 10 300 python tools/glue_census.py > $OUT/glue_$TAG.txt 2>&1 || { tail -5 $OUT/glue_$TAG.txt; exit 1; }
head -45 $OUT/glue_$TAG.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_c4_$TAG.json 2> $OUT/prof_$TAG.err || { tail -5 $OUT/prof_$TAG.err; exit 1; }
f=$(ls $OUT/prof_$TAG/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_$TAG/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_c4_$TAG.json
rm -f $f
cut -c1-300 $OUT/prof_c4_$TAG.json
echo done
