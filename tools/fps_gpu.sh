set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fps" > $OUT/fps_tests.log 2>&1
rc=$?; tail -20 $OUT/fps_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/fps_time.py
