#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg_dp_visual.py > $OUT/dbg.log 2>&1; rc=$?
grep -E "amp|fp32|Error|error" $OUT/dbg.log | tail -30; exit $rc
