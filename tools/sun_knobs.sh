set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() {
  timeout -k 10 300 env "$@" python bench.py --workload ${WL:-sun} --steps 30 --warmup 5 --no-cpu-baseline > $OUT/k.json 2> $OUT/k.err || { tail $OUT/k.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/k.json')); print('$*', d['value'], d['ms_per_step'])"
}
for kv in ${KNOBS}; do run $(echo $kv | tr ',' ' '); done
