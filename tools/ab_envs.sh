#!/bin/bash
# A/B of several env settings on the default SUN bench, two rounds, base first each round:
#   bash tools/ab_envs.sh "OV3D_A=1" "OV3D_B=2 OV3D_C=3" ...
#   BENCH_ARGS="--workload scannet": another workload
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out; mkdir -p $O
for i in 1 2; do
  for e in "X=0" "$@"; do
    env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $O/abe.json 2> $O/abe.err || { tail -5 $O/abe.err; exit 1; }
    python -c "import json; d=json.load(open('$O/abe.json')); print('$i', '$e', d['value'], d['ms_per_step_median'])"
  done
done
