#!/bin/bash
# pair-FPS diagnosis: the previous fps.hip (e96b460) and the one-workgroup kernel on the same data
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/fps_pair_stress.py 40 tools/libfps_old.so > $OUT/fps_stress_old.log 2>&1; echo "old rc=$?"
grep -v amdgpu.ids $OUT/fps_stress_old.log | cut -c1-200
OV3D_FPS_PAIR=0 timeout -k 10 300 python tools/fps_pair_stress.py 10 > $OUT/fps_stress_one.log 2>&1; echo "one-wg rc=$?"
grep -v amdgpu.ids $OUT/fps_stress_one.log | cut -c1-200
true
