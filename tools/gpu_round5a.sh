# round-5 check: C5 tests + bench + trace (tools/c5_quick.sh), the SUN step with the decoder K/V
# pair persistent vs one tile per workgroup, ROI statistics of the C5 step, gemm256 shape timings
set -u
bash tools/c5_quick.sh || exit 1
cd ${GRAFT_REPO_ROOT}; O=gpurun_out
for pp in 0 1; do
  OV3D_GEMM256_PAIR_PERSIST=$pp timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_pp$pp.json 2>$O/sun_pp$pp.err || exit 1
  python -c "import json; d=json.load(open('$O/sun_pp$pp.json')); print('SUN pp=$pp', d['value'], d['ms_per_step_median'])"
done
OV3D_ROI_STATS=1 timeout -k 10 300 python bench.py --workload sun_image --steps 1 --warmup 0 --no-cpu-baseline --no-graph > $O/roistats.json 2> $O/roistats.err
grep ROI_STATS $O/roistats.json $O/roistats.err | head -3
timeout -k 10 300 python -u tools/gemm256_time.py --reps 5 --json $O/g256.json > $O/g256.log 2>&1 || { tail -5 $O/g256.log; exit 1; }
cat $O/g256.log
