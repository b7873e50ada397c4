# round-5: sa_dy2b (one workgroup per CU: co-resident pairs corrupt its results, under
# investigation) vs sa_dy2_fused: kernel times and SUN A/B
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for v in "OV3D_SA_DY2_NWG=256" "OV3D_SA_DY2_LDSPAD=65536" "OV3D_SA_DY2_OLD=1 OV3D_SA_DY2_NWG=256"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dy2_$tag -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/dy2_$tag.json 2> $O/dy2_$tag.err || { tail -5 $O/dy2_$tag.err; exit 1; }
  python - <<PY
import csv,glob
f=glob.glob('$O/dy2_$tag/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sa_dy2' in r['Name']:
        print('$v', r['Name'][:50], r['Calls'], r['AverageNs'])
PY
done
