# C5 quick check: RegionCLIP GPU tests (or $TESTS), the C5 bench, a C5 kernel trace (per-step
# steady figures in gpurun_out/c5_steady.json).  SKIP_TESTS=1 / SKIP_PROF=1 skip those parts.
set -u
cd ${GRAFT_REPO_ROOT:-.}; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_regionclip_gpu.py tests/test_c5_step_gpu.py tests/test_gemm256_gpu.py} > $O/c5q_tests.log 2>&1 || { tail -30 $O/c5q_tests.log; exit 1; }
  tail -2 $O/c5q_tests.log
fi
timeout -k 10 300 python bench.py --workload sun_image --steps 10 --warmup 3 --no-cpu-baseline > $O/c5q_bench.json 2> $O/c5q_bench.err || { tail -20 $O/c5q_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5q_bench.json')); print('C5', d['value'], d['ms_per_step_median'])"
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5q_prof -o run --output-format csv -- python bench.py --workload sun_image --steps 5 --warmup 2 --no-cpu-baseline > $O/c5q_prof.json 2> $O/c5q_prof.err || { tail -5 $O/c5q_prof.err; exit 1; }
  python tools/trace_kernel_avg.py $(find $O/c5q_prof -name '*kernel_trace.csv' | head -1) "" --steps 4 --marker roi_align > $O/c5_steady.json
fi
