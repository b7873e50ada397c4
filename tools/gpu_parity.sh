set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_parity_full.py tests/test_sunaug_gpu.py tests/test_model_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/g1.log 2>&1
rc=$?; tail -40 $OUT/g1.log; exit $rc
