# env-knob sweep of csrc/gemm256.hip on the shapes of tools/gemm256_time.py (one process per
# setting: the knobs are read once per process)
set -u
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out; mkdir -p $O
for cfg in "GM=0 ST=1 DL=0" "GM=0 ST=0 DL=0" "GM=1 ST=1 DL=0" "GM=8 ST=1 DL=0" "GM=0 ST=1 DL=20" "GM=0 ST=1 DL=60"; do
  eval $cfg
  echo "== $cfg" >> $O/g256_sweep.log
  OV3D_GEMM256_GM=$GM OV3D_GEMM256_STAGGER=$ST OV3D_GEMM256_DELAY=$DL timeout -k 10 200 python -u tools/gemm256_time.py --reps 5 --no-lib --only "${ONLY:-}" >> $O/g256_sweep.log 2>&1 || exit 1
done
