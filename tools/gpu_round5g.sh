# round-5: the interim SA's 2^18-row GEMMs on gemm256 with K padded to 320: tests, C4 A/B
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_parity_full.py tests/test_wgrad_defer_gpu.py tests/test_gemm256_gpu.py > $O/r5g2_tests.log 2>&1 || { tail -30 $O/r5g2_tests.log; exit 1; }
tail -2 $O/r5g2_tests.log
for cfg in "X=1" "OV3D_GEMM256_MIN_M=1000000000 OV3D_GROUP_ROW_ALIGN=8" "OV3D_GROUP_ROW_ALIGN=8" "OV3D_GEMM256_MIN_M=1000000000"; do
  env $cfg timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_g.json 2> $O/c4_g.err || { tail -5 $O/c4_g.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_g.json')); print('C4 $cfg', d['value'], d['ms_per_step_median'])"
done
