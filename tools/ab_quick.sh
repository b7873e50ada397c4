#!/bin/bash
# quick GPU A/B: the SA / model parity tests, bench (20 steps), kernel stats of 10 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_sa_fused_gpu.py tests/test_model_gpu.py} > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || { tail -20 gpurun_out/ab_bench.err; exit 1; }
cut -c1-220 gpurun_out/ab_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> gpurun_out/ab_prof.err || { tail -5 gpurun_out/ab_prof.err; exit 1; }
python tools/prof_summary.py gpurun_out/ab_prof/run_kernel_stats.csv 16 | head -${TOP:-24}
