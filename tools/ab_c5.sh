#!/bin/bash
# A/B of env overrides on the C5 (RegionCLIP) bench, once each (usage: ab_c5.sh "VAR=v VAR2=w" ...)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for e in "OV3D_AB=0" "$@"; do
  env $e timeout -k 10 300 python bench.py --workload sun_image --steps ${STEPS:-8} --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "$e $(python -c 'import json;d=json.load(open("gpurun_out/ab.json"));print(d["value"], d["ms_per_step_median"])')"
done
