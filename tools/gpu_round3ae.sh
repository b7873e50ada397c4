#!/bin/bash
# set-criterion kernels on 16 lanes per row: set-loss tests, model parity, bench, trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03ae}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_parity_full.py tests/test_attention_gpu.py -q -x --timeout 200 --timeout-method thread > $OUT/t_$TAG.log 2>&1
rc=$?; tail -5 $OUT/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -5 $OUT/bench_$TAG.err; exit 1; }
cut -c1-300 $OUT/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -5 $OUT/prof_$TAG.err; exit 1; }
f=$(ls $OUT/prof_$TAG/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_$TAG/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_all_$TAG.json
python tools/trace_kernel_avg.py $f add_cast Fill > $OUT/tr_sl_$TAG.json
rm -f $f
cat $OUT/tr_sl_$TAG.json | head -30
echo done
