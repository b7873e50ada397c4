#!/bin/bash
# full check after the glue changes: smoke, every GPU test, bench, glue probe + census
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03j}
PMC=0 PROFILE=0 bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python tools/glue_probe.py > $OUT/glueprobe_$TAG.txt 2>&1 || { tail -5 $OUT/glueprobe_$TAG.txt; exit 1; }
head -40 $OUT/glueprobe_$TAG.txt
timeout -k 10 300 python tools/glue_census.py > $OUT/glue_$TAG.txt 2>&1 || { tail -5 $OUT/glue_$TAG.txt; exit 1; }
head -40 $OUT/glue_$TAG.txt
echo done
