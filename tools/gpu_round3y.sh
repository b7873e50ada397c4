#!/bin/bash
# drop bits ahead of the encoder forward (attn_dropgen_kernel over 4 key-tile ranges): attention
# tests, then the trace with and without the pre-pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03y}
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 200 --timeout-method thread > $OUT/t_$TAG.log 2>&1
rc=$?; tail -3 $OUT/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
for mode in -1 1048576; do
  OV3D_ATTN_DROPGEN_MIN=$mode timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_${TAG}_$mode.json 2> $OUT/bench_${TAG}_$mode.err || { tail -5 $OUT/bench_${TAG}_$mode.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${TAG}_$mode.json')); print('$mode', d['value'], d['ms_per_step_median'])"
  OV3D_ATTN_DROPGEN_MIN=$mode timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_$mode -o run -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> $OUT/prof_${TAG}_$mode.err || { tail -5 $OUT/prof_${TAG}_$mode.err; exit 1; }
  f=$(ls $OUT/prof_${TAG}_$mode/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_${TAG}_$mode/run_kernel_trace.csv)
  python tools/trace_kernel_avg.py $f "" --steps 8 > $OUT/tr_all_${TAG}_$mode.json
  python tools/trace_kernel_avg.py $f attn_ Fill > $OUT/tr_attn_${TAG}_$mode.json
  rm -f $f
  python - <<PY
import json
d=json.load(open('$OUT/tr_attn_${TAG}_$mode.json'))
for k,v in d['kernels'].items():
    if 'grid=(4096,32' in k: print('  ', round(v['avg_us'],1), k[:70])
PY
done
