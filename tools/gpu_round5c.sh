# round-5: attention forward with the dropout hash ahead of the row max: attention + ROIAlign
# tests, SUN bench (in-step attention timings), C4 bench
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attention_gpu.py tests/test_regionclip_gpu.py > $O/r5c_tests.log 2>&1 || { tail -30 $O/r5c_tests.log; exit 1; }
tail -2 $O/r5c_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sun_c.json 2>$O/sun_c.err || { tail -5 $O/sun_c.err; exit 1; }
python -c "import json; d=json.load(open('$O/sun_c.json')); print('SUN', d['value'], d['ms_per_step_median'], 'fwd', d['roofline']['avg_launch_ms'], d['roofline']['frac'], 'bwd', d['attn_bwd'])"
timeout -k 10 300 python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_c.json 2>$O/c4_c.err || { tail -5 $O/c4_c.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_c.json')); print('C4', d['value'], d['ms_per_step_median'], 'fwd', d['roofline']['avg_launch_ms'])"
