# quick GPU check: selected test files, then optional timing tool and SUN bench.
#   TESTS="tests/a.py tests/b.py" TIME=1 BENCH=1 bash tools/quick_check.sh
set -u
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $O/qc_tests.log 2>&1 || { tail -40 $O/qc_tests.log; exit 1; }
  tail -3 $O/qc_tests.log
fi
if [ "${TIME:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/gemm256_time.py --reps 5 --json $O/qc_g256.json > $O/qc_g256.log 2>&1 || { tail -20 $O/qc_g256.log; exit 1; }
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/qc_bench.json 2> $O/qc_bench.err || { tail -20 $O/qc_bench.err; exit 1; }
  cat $O/qc_bench.json
fi
