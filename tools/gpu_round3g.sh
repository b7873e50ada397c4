#!/bin/bash
# full check (smoke, every GPU test, bench as the driver runs it), then the FPS shapes and C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03g}
PMC=0 PROFILE=0 bash tools/gpu_check.sh || exit $?
timeout -k 10 200 python tools/fps_time.py > $OUT/fps_$TAG.json 2> $OUT/fps_$TAG.err || { tail -5 $OUT/fps_$TAG.err; exit 1; }
cat $OUT/fps_$TAG.json
timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4_$TAG.json 2> $OUT/c4_$TAG.err || { tail -5 $OUT/c4_$TAG.err; exit 1; }
cut -c1-400 $OUT/c4_$TAG.json
timeout -k 10 300 python tools/glue_census.py > $OUT/glue_$TAG.txt 2>&1; head -50 $OUT/glue_$TAG.txt
echo done
