# round-5: the masked encoder's mask packed from the points (no cdist GEMM): attention tests,
# C4 bench with and without, C4 kernel trace
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_attention_gpu.py > $O/r5f_tests.log 2>&1 || { tail -30 $O/r5f_tests.log; exit 1; }
tail -2 $O/r5f_tests.log
for pm in 1 0; do
  OV3D_POINT_MASK=$pm timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_pm$pm.json 2> $O/c4_pm$pm.err || { tail -5 $O/c4_pm$pm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_pm$pm.json')); print('C4 point_mask=$pm', d['value'], d['ms_per_step_median'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4_prof4 -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_prof4.json 2> $O/c4_prof4.err || { tail -5 $O/c4_prof4.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/c4_prof4 -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy8_kernel > $O/c4_trace_steady4.json
