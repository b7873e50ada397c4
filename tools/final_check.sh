set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_check.sh || exit $?
OUT=gpurun_out
for wl in scannet sun_image; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > $OUT/final_$wl.json 2> $OUT/final_$wl.err || { tail -3 $OUT/final_$wl.err; exit 1; }
  cat $OUT/final_$wl.json
done
