# round-5: C4 with the next batch's sampling plan started mid-step (after the encoder) vs with
# the step (its FPS now 3.9 ms with the pair kernel, the C4 step 7.3 ms)
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "X=0" "OV3D_PLAN_MID_START=1" "OV3D_PLAN_MID_START=1 OV3D_PLAN_SPLIT_AT=memory_kv"; do
    env $v timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_q.json 2> $O/c4_q.err || { tail -5 $O/c4_q.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c4_q.json')); print('C4 $v', d['value'], d['ms_per_step_median'])"
  done
done
