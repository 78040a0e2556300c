#!/bin/bash
# Selected GPU tests in one pytest process, each run bounded; output to gpurun_out/pytest_sel.log.
# usage: tools/gpu_tests.sh tests/test_a.py tests/test_b.py ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_sel.log
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_sel.log | tail -40
exit $rc
