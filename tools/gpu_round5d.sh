# round-5: colour SA layer-2 backward on sa_dy2_fused (stored y1), ROIAlign image-affine XCD
# order: their tests, the C4 / C5 bench lines and a C4 kernel trace
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_regionclip_gpu.py tests/test_parity_full.py > $O/r5d_tests.log 2>&1 || { tail -30 $O/r5d_tests.log; exit 1; }
tail -2 $O/r5d_tests.log
timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_bench3.json 2> $O/c4_bench3.err || { tail -5 $O/c4_bench3.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_bench3.json')); print('C4', d['value'], d['ms_per_step_median'])"
for aff in 1 0; do
  OV3D_ROI_AFFINE=$aff timeout -k 10 300 python bench.py --workload sun_image --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_aff$aff.json 2> $O/c5_aff$aff.err || { tail -5 $O/c5_aff$aff.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_aff$aff.json')); print('C5 affine=$aff', d['value'], d['ms_per_step_median'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4_prof3 -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_prof3.json 2> $O/c4_prof3.err || { tail -5 $O/c4_prof3.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/c4_prof3 -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy8_kernel > $O/c4_trace_steady3.json
