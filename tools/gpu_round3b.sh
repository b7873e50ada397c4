#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "== kernel tests"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_gpu.py tests/test_project_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/t3b.log 2>&1
rc=$?; tail -15 $OUT/t3b.log; [ $rc -eq 0 ] || exit $rc
echo "== fps timing (pair / two-cluster)"
OV3D_FPS_PAIR=1 timeout -k 10 120 python tools/fps_time.py > $OUT/fps_pair.json 2>&1 && cat $OUT/fps_pair.json || exit 1
OV3D_FPS_PAIR=0 timeout -k 10 120 python tools/fps_time.py > $OUT/fps_old.json 2>&1 && cat $OUT/fps_old.json || exit 1
echo "== dp world 2"
timeout -k 10 400 python -u -m pytest tests/test_dp_world2_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/dp2.log 2>&1
rc=$?; tail -12 $OUT/dp2.log; [ $rc -le 1 ] || exit $rc
echo "== parity report"
timeout -k 10 400 python tools/parity_report.py > $OUT/pr2.log 2>&1 || { tail -30 $OUT/pr2.log; exit 1; }
grep -E "==|grad|out|loss" $OUT/pr2.log | cut -c1-300
echo "== bench"
PROFILE=0 TAG=r03b bash tools/gpu_bench_prof.sh
TAG=r03c timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4.json 2>$OUT/bench_c4.err; cat $OUT/bench_c4.json | cut -c1-400
