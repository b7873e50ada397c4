#!/bin/bash
# Long row-block GEMM check on the GPU box: parity tests, graph-timed per-shape comparison with the
# library GEMM for the default tiles and each VARIANTS entry (env assignments), then PMC passes
# of three shapes (PMC=0 skips them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/tg_test.log gpurun_out/gt_*.log gpurun_out/gpmc.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tile_gemm_gpu.py > gpurun_out/tg_test.log 2>&1 || { tail -30 gpurun_out/tg_test.log; exit 1; }
timeout -k 10 200 python tools/gemm_time.py > gpurun_out/gt_def.log 2>&1 || exit 1
i=0
for v in ${VARIANTS:-}; do
  i=$((i+1))
  env $v timeout -k 10 200 python tools/gemm_time.py > gpurun_out/gt_v$i.log 2>&1 || exit 1
  sed -i "1i $v" gpurun_out/gt_v$i.log
done
[ "${PMC:-1}" = 1 ] || exit 0
PMC_RE="tile_gemm_kernel" PMC_CMD="tools/gemm_time.py --eager --only ${PMC_ONLY:-1,5,7}" timeout -k 10 400 bash tools/gpu_pmc.sh > gpurun_out/gpmc.log 2>&1
