# round-5: SA layer-3 forward with one extreme per channel (MODE_POOL1): tests, forward phase
# probe, SUN A/B against OV3D_SA_POOL_BOTH=1, kernel times
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_parity_full.py > $O/r5m_tests.log 2>&1 || { tail -30 $O/r5l_tests.log; exit 1; }
tail -2 $O/r5m_tests.log
timeout -k 10 200 python tools/sa_probe.py run fwd > $O/saprobe_fwd3.json 2> $O/saprobe_fwd3.err || { tail -5 $O/saprobe_fwd3.err; exit 1; }
python -c "import json; d=json.load(open('$O/saprobe_fwd3.json')); print('pool1', d['total_cycles_per_tile'], d['cycles_per_tile_by_phase'])"
for rep in 1 2; do
  for v in "X=0" "OV3D_SA_POOL_BOTH=1"; do
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_m.json 2> $O/sun_m.err || { tail -5 $O/sun_m.err; exit 1; }
    python -c "import json; d=json.load(open('$O/sun_m.json')); print('SUN $v', d['value'], d['ms_per_step_median'])"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sa_prof_m -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sa_prof_m.json 2> $O/sa_prof_m.err || { tail -5 $O/sa_prof_m.err; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$O/sa_prof_m/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sa_dy' in r['Name'] or 'sa_layer' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
