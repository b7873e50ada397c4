# C4 check: the SA / parity / model GPU tests, then the ScanNet bench and its kernel trace
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_parity_full.py tests/test_model_gpu.py > $O/c4chk_tests.log 2>&1 || { tail -30 $O/c4chk_tests.log; exit 1; }
tail -2 $O/c4chk_tests.log
timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_bench2.json 2> $O/c4_bench2.err || { tail -5 $O/c4_bench2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_bench2.json')); print('C4', d['value'], d['ms_per_step_median'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4_prof2 -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_prof2.json 2> $O/c4_prof2.err || { tail -5 $O/c4_prof2.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/c4_prof2 -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy8_kernel > $O/c4_trace_steady2.json
