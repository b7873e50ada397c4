#!/bin/bash
# pair FPS with the published Morton order (stress, both exchange paths), every GPU test,
# attention / FPS timing, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/fps_pair_stress.py 40 > $OUT/fps_stress.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/fps_stress.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
OV3D_FPS_XCH=mem timeout -k 10 300 python tools/fps_pair_stress.py 40 > $OUT/fps_stress_mem.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/fps_stress_mem.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/attn_time.py > $OUT/attn_time.log 2>&1; tail -8 $OUT/attn_time.log
timeout -k 10 200 python tools/fps_time.py
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_k.json 2> $OUT/bench_k.err || { tail -5 $OUT/bench_k.err; exit 1; }
cut -c1-400 $OUT/bench_k.json
echo done
