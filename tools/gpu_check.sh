#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop() { echo "STOP after $1 (rc=$2)"; exit "$2"; }
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

echo "== smoke"; timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || stop smoke $rc

echo "== pytest -m gpu"; timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log; if fatal $rc; then stop pytest $rc; fi

echo "== bench"; timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; [ $rc -eq 0 ] || stop bench $rc

if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
  rc=$?; tail -3 $OUT/prof.err; [ $rc -eq 0 ] || stop rocprof $rc
  find $OUT/prof -name '*stats*' | head
fi
if [ "${PMC:-1}" = "1" ]; then
  # HBM traffic of the FPS kernel: FETCH_SIZE and WRITE_SIZE need separate passes on gfx950
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $c"
    timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex fps -d $OUT/pmc_$c -o run --output-format csv -- \
        python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-graph > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err
    rc=$?; tail -2 $OUT/pmc_$c.err; [ $rc -eq 0 ] || stop pmc_$c $rc
  done
fi
echo "== done"
