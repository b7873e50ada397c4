#!/bin/bash
# SUN bench under each env setting in turn (usage: bench_envs.sh "A=1 B=0" "A=0" ...), stops at
# the first failing run (a fault ends the call there); one summary line per setting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
n=0
for e in "$@"; do
  n=$((n + 1))
  env $e timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
      > gpurun_out/be_$n.json 2> gpurun_out/be_$n.err || { echo "FAILED: $e"; tail -25 gpurun_out/be_$n.err; exit 1; }
  echo "$e -> $(python -c 'import json,sys;d=json.load(open(sys.argv[1]));print(d["value"], d["ms_per_step_median"])' gpurun_out/be_$n.json)"
done
