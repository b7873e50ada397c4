# round-5: BN row passes with several rows a thread: their tests, SUN / C4 bench, C4 trace
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_heads_gpu.py tests/test_sa_fused_gpu.py tests/test_parity_full.py > $O/r5h_tests.log 2>&1 || { tail -30 $O/r5h_tests.log; exit 1; }
tail -2 $O/r5h_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_h.json 2> $O/sun_h.err || { tail -5 $O/sun_h.err; exit 1; }
python -c "import json; d=json.load(open('$O/sun_h.json')); print('SUN', d['value'], d['ms_per_step_median'])"
timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_h.json 2> $O/c4_h.err || { tail -5 $O/c4_h.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_h.json')); print('C4', d['value'], d['ms_per_step_median'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4_prof5 -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_prof5.json 2> $O/c4_prof5.err || { tail -5 $O/c4_prof5.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/c4_prof5 -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy8_kernel > $O/c4_trace_steady5.json
