#!/bin/bash
# library GEMM census; the DP collectives path at world 1 (graph capture with RCCL)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/gemm_census.py > $OUT/gemm_census.txt 2>&1; rc=$?; grep -v amdgpu $OUT/gemm_census.txt | head -45; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --dp-collectives > $OUT/bench_dp.json 2> $OUT/bench_dp.err || { tail -5 $OUT/bench_dp.err; exit 1; }
cut -c1-300 $OUT/bench_dp.json
echo done
