#!/bin/bash
# interim SA on bf16 padded group rows: every GPU test, C4 bench + steady trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03n}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4_$TAG.json 2> $OUT/c4_$TAG.err || { tail -5 $OUT/c4_$TAG.err; exit 1; }
cut -c1-330 $OUT/c4_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_c4_$TAG.json 2> $OUT/prof_$TAG.err || { tail -5 $OUT/prof_$TAG.err; exit 1; }
f=$(ls $OUT/prof_$TAG/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_$TAG/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_c4_$TAG.json
rm -f $f
echo done
