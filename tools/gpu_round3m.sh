#!/bin/bash
# new FPS regression test; C5 with / without the im2col overlap; C4; SUN steady-state trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03m}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "two_workgroup or fps_bit" --timeout 120 --timeout-method thread > $OUT/t_$TAG.log 2>&1
rc=$?; tail -2 $OUT/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
for ov in 1 0; do
  OV3D_CONV_OVERLAP=$ov timeout -k 10 500 python bench.py --workload sun_image --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5_ov${ov}_$TAG.json 2> $OUT/c5_ov${ov}_$TAG.err || { tail -5 $OUT/c5_ov${ov}_$TAG.err; exit 1; }
  echo "overlap=$ov"; cut -c1-200 $OUT/c5_ov${ov}_$TAG.json
done
timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4_$TAG.json 2> $OUT/c4_$TAG.err || { tail -5 $OUT/c4_$TAG.err; exit 1; }
cut -c1-300 $OUT/c4_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -5 $OUT/prof_$TAG.err; exit 1; }
f=$(ls $OUT/prof_$TAG/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_$TAG/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_all_$TAG.json
rm -f $f
cut -c1-300 $OUT/prof_bench_$TAG.json
echo done
