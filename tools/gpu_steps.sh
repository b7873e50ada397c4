#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit, output to
# gpurun_out/<name>.log.  Usage: tools/gpu_steps.sh 'name|seconds|command' ...
# A step that ends with a test failure (rc 1) does not stop the chain; a fault, abort,
# segfault or time limit (any other nonzero rc) ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
worst=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc in $(( $(date +%s) - t0 )) s"; tail -4 "$OUT/$name.log"
  case $rc in
    0) ;;
    1) worst=1 ;;
    *) echo "STOP after $name (rc=$rc)"; exit $rc ;;
  esac
done
exit $worst
