# the whole -m gpu suite, one process (round-5 regression check)
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/full_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/full_tests.log | tail -3
grep -E "FAILED|Error" $O/full_tests.log | head -10
exit $rc
