#!/bin/bash
# One GPU-box session, steps chosen by name (replaces round 5's one-off gpu_round5*/gpu_close5*):
#   bash tools/gpu_session.sh smoke tests bench sun_trace c4 c4_trace c5 pmc
#   TESTS="tests/test_x.py" bash tools/gpu_session.sh tests        (a subset of the GPU suite)
#   TAG=r6a: output names under gpurun_out/ carry the tag.  PMC_RE: kernels for the pmc step.
# Every GPU step runs under its own time limit; the first failure (fault, abort, timeout) ends the
# script, so nothing else touches the GPU after it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
T=${TAG:-s}
fail() { echo "STOP after $1 (rc=$2)"; tail -30 "$3"; exit "$2"; }
for step in "$@"; do
  echo "== $step"
  case $step in
    smoke)
      timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || fail smoke $? $O/${T}_smoke.log
      tail -1 $O/${T}_smoke.log ;;
    tests)
      timeout -k 10 1500 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1 || fail tests $? $O/${T}_pytest.log
      tail -2 $O/${T}_pytest.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/${T}_bench.json 2> $O/${T}_bench.err || fail bench $? $O/${T}_bench.err
      python -c "import json; d=json.load(open('$O/${T}_bench.json')); r=d.get('roofline') or {}; print('SUN', d['value'], d['ms_per_step_median'], r.get('frac'), (d.get('cpu_baseline') or {}).get('value'))" ;;
    quick)
      for rep in 1 2; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/${T}_quick$rep.json 2> $O/${T}_quick$rep.err || fail quick $? $O/${T}_quick$rep.err
        python -c "import json; d=json.load(open('$O/${T}_quick$rep.json')); print('quick', d['value'], d['ms_per_step_median'])"
      done ;;
    sun_trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${T}_sun_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/${T}_sun_prof.json 2> $O/${T}_sun_prof.err || fail sun_trace $? $O/${T}_sun_prof.err
      python tools/trace_kernel_avg.py $(find $O/${T}_sun_prof -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy9_kernel > $O/${T}_sun_trace_steady.json ;;
    c4)
      timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_c4_bench.json 2> $O/${T}_c4_bench.err || fail c4 $? $O/${T}_c4_bench.err
      python -c "import json; d=json.load(open('$O/${T}_c4_bench.json')); print('C4', d['value'], d['ms_per_step_median'])" ;;
    c4_trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${T}_c4_prof -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/${T}_c4_prof.json 2> $O/${T}_c4_prof.err || fail c4_trace $? $O/${T}_c4_prof.err
      python tools/trace_kernel_avg.py $(find $O/${T}_c4_prof -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy9_kernel > $O/${T}_c4_trace_steady.json ;;
    c5)
      SKIP_TESTS=1 bash tools/c5_quick.sh || exit 1 ;;
    pmc)
      PMC_RE="${PMC_RE:-attn_fwd_kernel|attn_bwd|sa_dy9_kernel|sa_layer_kernel|sa_dy2_fused_kernel|lngemm_bwd_kernel}" bash tools/gpu_pmc.sh || exit 1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
