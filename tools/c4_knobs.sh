set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() {
  timeout -k 10 300 env "$@" python bench.py --workload ${WL:-scannet} --steps 20 --warmup 5 --no-cpu-baseline > $OUT/k.json 2> $OUT/k.err || { tail $OUT/k.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/k.json')); print('$*', d['value'], d['ms_per_step'])"
}
run A=1
run OV3D_SA_DY_NWG=248
run OV3D_SA_DY_NWG=248 OV3D_WGRAD_WGS=248
run A=2
