set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O
run() {
  env $2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/ab_$1.json 2> $O/ab_$1.err || { tail -5 $O/ab_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ab_$1.json')); print('$1', '$2', d['value'], d['ms_per_step_median'])"
}
for i in 1 2; do
  run a$i X=0 || exit 1
  run b$i OV3D_PLAN_MID_START=0 || exit 1
  run c$i OV3D_PLAN_SPLIT_AT=pre_encoder || exit 1
done
