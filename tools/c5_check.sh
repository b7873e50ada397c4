set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_regionclip_gpu.py tests/test_c5_step_gpu.py > $O/c5_tests.log 2>&1 || { tail -30 $O/c5_tests.log; exit 1; }
timeout -k 10 300 python bench.py --workload sun_image --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_bench.json 2> $O/c5_bench.err || { tail -20 $O/c5_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5_prof -o run --output-format csv -- python bench.py --workload sun_image --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_prof.json 2> $O/c5_prof.err || { tail -5 $O/c5_prof.err; exit 1; }
python tools/prof_summary.py $(find $O/c5_prof -name '*kernel_stats.csv' | head -1) 7 > $O/c5_prof_summary.txt
