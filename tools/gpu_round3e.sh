#!/bin/bash
# attention tests, then a steady-state trace of the bench and the PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_headsout_gpu.py -q --timeout 300 --timeout-method thread > $OUT/t3e.log 2>&1
rc=$?; tail -3 $OUT/t3e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_e -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/tr_e.json 2> $OUT/tr_e.err || { tail -5 $OUT/tr_e.err; exit 1; }
f=$(ls $OUT/tr_e/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/tr_e/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_all_e.json
rm -f $f
cut -c1-200 $OUT/tr_e.json
bash tools/gpu_pmc.sh
