#!/bin/bash
# dp world-2 test, the bf16 / fp32 full-shape parity tests, heads tests; then a bench trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_dp_world2_gpu.py tests/test_attention_gpu.py tests/test_parity_full.py tests/test_headsout_gpu.py tests/test_heads_gpu.py tests/test_model_gpu.py -v -s --timeout 300 --timeout-method thread > $OUT/t3d.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|checked|hip/torch|q50|flip" $OUT/t3d.log | cut -c1-250 | tail -40; [ $rc -eq 0 ] || exit $rc
echo "== trace"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_d -o run -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/tr_d.json 2> $OUT/tr_d.err || { tail -5 $OUT/tr_d.err; exit 1; }
f=$(ls $OUT/tr_d/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/tr_d/run_kernel_trace.csv)
python tools/trace_kernel_avg.py $f attn_ fps_ sa_ wgrad heads_out --steps 8 > $OUT/tr_avg_d.json
python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_all_d.json
rm -f $f
cut -c1-200 $OUT/tr_d.json
echo done
