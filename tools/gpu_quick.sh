#!/bin/bash
# quick GPU check: the named test files (default: attention + dp world 2), verbose, one process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
FILES=${FILES:-"tests/test_attention_gpu.py tests/test_dp_world2_gpu.py"}
timeout -k 10 600 python -u -m pytest $FILES -v -s --timeout 300 --timeout-method thread > $OUT/quick.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|largest|checked|hip/torch|q50" $OUT/quick.log | cut -c1-400 | tail -40; exit $rc
