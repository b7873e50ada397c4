# round-5: the encoder's 16384-row GEMMs on gemm256 (OV3D_GEMM256_MIN_M=16384) vs tile_gemm: SUN A/B
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "X=0" "OV3D_GEMM256_MIN_M=16384"; do
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_p.json 2> $O/sun_p.err || { tail -5 $O/sun_p.err; exit 1; }
    python -c "import json; d=json.load(open('$O/sun_p.json')); print('SUN $v', d['value'], d['ms_per_step_median'])"
  done
done
env OV3D_GEMM256_MIN_M=16384 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/g256_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/g256_prof.json 2> $O/g256_prof.err || { tail -5 $O/g256_prof.err; exit 1; }
python - <<PY
import csv,glob
f=glob.glob('$O/g256_prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gemm' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
PY
