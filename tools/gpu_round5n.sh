# round-5: SA layer-2 backward restructured (sa_dy2b): SA tests, full-step parity, SUN / C4 A/B
# against OV3D_SA_DY2_OLD=1 (with the old kernel's 256 workgroups), kernel times
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_parity_full.py > $O/r5n_tests.log 2>&1 || { tail -30 $O/r5n_tests.log; exit 1; }
tail -2 $O/r5n_tests.log
for rep in 1 2; do
  for v in "X=0" "OV3D_SA_DY2_OLD=1 OV3D_SA_DY2_NWG=256"; do
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_n.json 2> $O/sun_n.err || { tail -5 $O/sun_n.err; exit 1; }
    python -c "import json; d=json.load(open('$O/sun_n.json')); print('SUN $v', d['value'], d['ms_per_step_median'])"
  done
done
for v in "X=0" "OV3D_SA_DY2_OLD=1 OV3D_SA_DY2_NWG=256"; do
  env $v timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_n.json 2> $O/c4_n.err || { tail -5 $O/c4_n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_n.json')); print('C4 $v', d['value'], d['ms_per_step_median'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sa_prof_n -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sa_prof_n.json 2> $O/sa_prof_n.err || { tail -5 $O/sa_prof_n.err; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$O/sa_prof_n/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sa_dy' in r['Name'] or 'sa_layer' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
