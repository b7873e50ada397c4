#!/bin/bash
# tests of the changed kernels, the bench as the driver runs it, and rocprofv3 kernel stats +
# a steady-state trace of the same bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03f}
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_headsout_gpu.py tests/test_heads_gpu.py tests/test_sa_fused_gpu.py tests/test_model_gpu.py -q --timeout 300 --timeout-method thread > $OUT/t_$TAG.log 2>&1
rc=$?; tail -3 $OUT/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -5 $OUT/bench_$TAG.err; exit 1; }
cut -c1-300 $OUT/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -5 $OUT/prof_$TAG.err; exit 1; }
f=$(ls $OUT/prof_$TAG/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_$TAG/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_all_$TAG.json
python tools/trace_kernel_avg.py $f attn_fwd attn_bwd > $OUT/tr_attn_$TAG.json
rm -f $f
cut -c1-300 $OUT/prof_bench_$TAG.json
echo done
