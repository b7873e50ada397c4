# round-5: SA layer-3 backward with its MFMA chains fed ahead (sa_dy9): tests, SUN A/B against
# sa_dy8 (OV3D_SA_DY8=1), kernel times from a trace of each
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_sa_fused_gpu.py tests/test_parity_full.py > $O/r5i_tests.log 2>&1 || { tail -30 $O/r5i_tests.log; exit 1; }
tail -2 $O/r5i_tests.log
for rep in 1 2; do
  for v in "X=0" "OV3D_SA_DY8=1"; do
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_i.json 2> $O/sun_i.err || { tail -5 $O/sun_i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/sun_i.json')); print('SUN $v', d['value'], d['ms_per_step_median'])"
  done
done
for v in "X=0" "OV3D_SA_DY8=1"; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sa_prof_$tag -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sa_prof_$tag.json 2> $O/sa_prof_$tag.err || { tail -5 $O/sa_prof_$tag.err; exit 1; }
  python - <<PY
import csv,glob
f=glob.glob('$O/sa_prof_$tag/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sa_dy' in r['Name'] or 'sa_layer' in r['Name']:
        print('$v', r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
