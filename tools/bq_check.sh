set -u
# ball query: GPU tests, then the cells-vs-scan timing under a kernel trace (per-kernel split)
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
if [ "${BQ_TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "ball_query or group" > $O/bq_tests.log 2>&1 || { tail -30 $O/bq_tests.log; exit 1; }
  tail -3 $O/bq_tests.log
fi
for v in ${BQ_VARIANTS:-default}; do
  if [ "$v" = loop ]; then export OV3D_BQ_LOOP=1; else unset OV3D_BQ_LOOP; fi
  rm -rf $O/bq_prof
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/bq_prof -o run --output-format csv -- python tools/bq_time.py > $O/bq_time.log 2>&1 || { tail -20 $O/bq_time.log; exit 1; }
  echo "== $v"; grep '^{' $O/bq_time.log
  python tools/bq_kernels.py
done
