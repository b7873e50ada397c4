set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sa_fused_gpu.py tests/test_attention_gpu.py tests/test_model_gpu.py > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -2 gpurun_out/q_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { tail -20 gpurun_out/q_bench.err; exit 1; }
cut -c1-200 gpurun_out/q_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> gpurun_out/qprof.err || { tail -5 gpurun_out/qprof.err; exit 1; }
echo done
