#!/bin/bash
# FPS kernel tests + timing after the exchange change, glue probe (python call sites)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03i}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k fps --timeout 120 --timeout-method thread > $OUT/t_$TAG.log 2>&1
rc=$?; tail -3 $OUT/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/fps_time.py > $OUT/fps_$TAG.json 2> $OUT/fps_$TAG.err || { tail -5 $OUT/fps_$TAG.err; exit 1; }
cat $OUT/fps_$TAG.json
timeout -k 10 300 python tools/glue_probe.py > $OUT/glueprobe_$TAG.txt 2>&1 || { tail -5 $OUT/glueprobe_$TAG.txt; exit 1; }
head -70 $OUT/glueprobe_$TAG.txt
echo done
