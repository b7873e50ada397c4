set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wgrad_gpu.py tests/test_wgrad_defer_gpu.py tests/test_heads_gpu.py > gpurun_out/w_pytest.log 2>&1 || { tail -30 gpurun_out/w_pytest.log; exit 1; }
tail -2 gpurun_out/w_pytest.log
