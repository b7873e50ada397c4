#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
echo "== attention tests"
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_headsout_gpu.py tests/test_heads_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/attn.log 2>&1
rc=$?; tail -3 $OUT/attn.log; [ $rc -eq 0 ] || exit $rc
echo "== dp world 2"
timeout -k 10 400 python -u -m pytest tests/test_dp_world2_gpu.py -x -q -s --timeout 300 --timeout-method thread > $OUT/dp2.log 2>&1
rc=$?; grep -E "checked|passed|failed|Error" $OUT/dp2.log | tail -5; [ $rc -le 1 ] || exit $rc
echo "== parity report"
timeout -k 10 400 python tools/parity_report.py --floor 1e-6 > $OUT/pr3.log 2>&1 || { tail -30 $OUT/pr3.log; exit 1; }
echo "== traces dropgen on / off"
for v in on off; do
  if [ $v = off ]; then export OV3D_ATTN_DROPGEN_MIN=2000000000; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$v -o run -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/tr_$v.json 2> $OUT/tr_$v.err || { tail -5 $OUT/tr_$v.err; exit 1; }
  f=$(ls $OUT/tr_$v/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/tr_$v/run_kernel_trace.csv)
  python tools/trace_kernel_avg.py $f attn_ fps_ sa_ wgrad heads_out > $OUT/tr_avg_$v.json
  python tools/trace_kernel_avg.py $f "" > $OUT/tr_all_$v.json
  rm -f $f
  cut -c1-200 $OUT/tr_$v.json
done
echo done
