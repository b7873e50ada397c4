#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "== parity report"
timeout -k 10 300 python tools/parity_report.py > $OUT/pr.log 2>&1 || { tail -30 $OUT/pr.log; exit 1; }
cut -c1-600 $OUT/pr.log
echo "== dp world 2"
timeout -k 10 400 python -u -m pytest tests/test_dp_world2_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/dp2.log 2>&1
rc=$?; tail -30 $OUT/dp2.log; [ $rc -le 1 ] || exit $rc
echo "== bench + prof"
TAG=r03a bash tools/gpu_bench_prof.sh
