# round-5: ROIAlign LDS window + pipelined attention forward: their tests, C5 bench + trace,
# SUN bench with the pipelined forward on / off, and the in-step attention timings
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attention_gpu.py tests/test_regionclip_gpu.py > $O/r5b_tests.log 2>&1 || { tail -30 $O/r5b_tests.log; exit 1; }
tail -2 $O/r5b_tests.log
for pipe in 1 0; do
  OV3D_ATTN_PIPE=$pipe timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_pipe$pipe.json 2>$O/sun_pipe$pipe.err || { tail -5 $O/sun_pipe$pipe.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sun_pipe$pipe.json')); print('SUN pipe=$pipe', d['value'], d['ms_per_step_median'], 'fwd', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
SKIP_TESTS=1 bash tools/c5_quick.sh
