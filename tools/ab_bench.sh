# A/B bench: default vs an env override, each in its own process (usage: ab_bench.sh VAR=value ...)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
for e in "OV3D_AB=0" "$@"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "$e $(python -c 'import json;d=json.load(open("gpurun_out/ab.json"));print(d["value"], d["ms_per_step"])')"
done
