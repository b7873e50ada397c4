# round-5: sa_dy9 with the dz epilogue in the dW3 chain's MFMA shadow: SA tests, parity, probe,
# kernel time, SUN bench
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_parity_full.py > $O/r5r_tests.log 2>&1 || { tail -30 $O/r5r_tests.log; exit 1; }
tail -2 $O/r5r_tests.log
timeout -k 10 200 python tools/sa_probe.py run > $O/saprobe9r.json 2> $O/saprobe9r.err || { tail -5 $O/saprobe9r.err; exit 1; }
python -c "import json; d=json.load(open('$O/saprobe9r.json')); print('dy9', d['total_cycles_per_tile'], d['cycles_per_tile_by_phase'])"
timeout -k 10 200 python tools/sa_bwd_check.py 2>&1 | grep -E "S=64" | head -6
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_r.json 2> $O/sun_r.err || { tail -5 $O/sun_r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sun_r.json')); print('SUN', d['value'], d['ms_per_step_median'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sa_prof_r -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sa_prof_r.json 2> $O/sa_prof_r.err || { tail -5 $O/sa_prof_r.err; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$O/sa_prof_r/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sa_dy' in r['Name'] or 'sa_layer' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
