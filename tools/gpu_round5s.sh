# round-5: layer-3 forward with column block 0's epilogue in block 1's MFMA shadow: SA tests,
# forward probe, kernel times, SUN bench
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_parity_full.py > $O/r5s_tests.log 2>&1 || { tail -30 $O/r5s_tests.log; exit 1; }
tail -2 $O/r5s_tests.log
timeout -k 10 200 python tools/sa_probe.py run fwd > $O/saprobe_fwd4.json 2> $O/saprobe_fwd4.err || { tail -5 $O/saprobe_fwd4.err; exit 1; }
python -c "import json; d=json.load(open('$O/saprobe_fwd4.json')); print('pool1', d['total_cycles_per_tile'], d['cycles_per_tile_by_phase'])"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_s.json 2> $O/sun_s.err || { tail -5 $O/sun_s.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sun_s.json')); print('SUN', d['value'], d['ms_per_step_median'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sa_prof_s -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sa_prof_s.json 2> $O/sa_prof_s.err || { tail -5 $O/sa_prof_s.err; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$O/sa_prof_s/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sa_dy' in r['Name'] or 'sa_layer' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
