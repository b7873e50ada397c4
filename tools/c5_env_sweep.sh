set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O
for cfg in "X=0" "OV3D_GEMM256_DELAY=1" "OV3D_GEMM256_DELAY=3" "OV3D_GEMM256_GM=4" "OV3D_GEMM256_GM=16" "OV3D_GEMM256_STAGGER=0"; do
  env $cfg timeout -k 10 200 python bench.py --workload sun_image --steps 8 --warmup 2 --no-cpu-baseline > $O/c5s.json 2> $O/c5s.err || { tail -5 $O/c5s.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5s.json')); r=d['roofline']; print('$cfg', d['ms_per_step_median'], r['ms_per_step'], r['achieved'])"
done
