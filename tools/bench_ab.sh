set -u
# A/B of an environment switch on the default-workload bench: alternating runs (AB_VAR=value
# vs unset), BENCH_REPS pairs; BENCH_C4=1 adds one C4 pair
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O
run() {  # name workload envassign
  env $3 timeout -k 10 300 python bench.py --workload $2 --steps 30 --warmup 5 --no-cpu-baseline > $O/ab_$1.json 2> $O/ab_$1.err || { tail -5 $O/ab_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab_$1.json')); print('$1', '$3', d['value'], d['ms_per_step_median'])"
}
for i in $(seq 1 ${BENCH_REPS:-2}); do
  run sun_a$i sun X=0 || exit 1
  run sun_b$i sun "$AB_VAR" || exit 1
done
if [ "${BENCH_C4:-0}" = 1 ]; then
  run c4_a scannet X=0 || exit 1
  run c4_b scannet "$AB_VAR" || exit 1
fi
