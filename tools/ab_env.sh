#!/bin/bash
# A/B of env overrides in one tree (usage: ab_env.sh VAR=value ...): the bench value and the
# in-step attention times of each, default first, twice round
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for i in 1 2; do
for e in "OV3D_AB=0" "$@"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "$e $(python -c 'import json;d=json.load(open("gpurun_out/ab.json"));r=d["roofline"];b=d["attn_bwd"];print(d["value"], d["ms_per_step_median"], "fwd", r["avg_launch_ms"], "dq", b["dq_ms"], "dkdv", b["dkdv_ms"])')"
done
done
