#!/bin/bash
# Runs one pytest selection against several library builds on the GPU box; a test failure (rc 1)
# continues with the next build, anything else (timeout, abort, fault) ends the call.
# usage: bash scripts/bisect_tests.sh TAG "PYTEST ARGS" LIB1 LIB2 ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; ARGS=$2; shift 2
for L in "$@"; do
  n=$(echo "$L" | tr '/' '_')
  GENPOSE_HIP_LIB=$L timeout -k 10 600 python -u -m pytest $ARGS --timeout 300 --timeout-method thread > gpurun_out/${TAG}_${n}.log 2>&1
  rc=$?
  echo "$L rc=$rc $(tail -1 gpurun_out/${TAG}_${n}.log)"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
