# round-5: decoder norm + linear boundaries in one launch each way (csrc/lngemm.hip): the
# resnorm / decoder tests, then the SUN bench line with and without, and a SUN kernel trace
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnorm_gpu.py > $O/r5e_tests.log 2>&1 || { tail -40 $O/r5e_tests.log; exit 1; }
tail -2 $O/r5e_tests.log
for lg in 1 0; do
  OV3D_LNGEMM=$lg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_lg$lg.json 2> $O/sun_lg$lg.err || { tail -5 $O/sun_lg$lg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sun_lg$lg.json')); print('SUN lngemm=$lg', d['value'], d['ms_per_step_median'])"
done


timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sun_prof5 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sun_prof5.json 2> $O/sun_prof5.err || { tail -5 $O/sun_prof5.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/sun_prof5 -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy8_kernel > $O/sun_trace_steady5.json
