#!/bin/bash
# The GPU test suite in one process (as the driver runs it), log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${SUITE_TIMEOUT:-1100} python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  ${TESTS:-tests} -m gpu > gpurun_out/${TAG:-r6}_gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/${TAG:-r6}_gpu_tests.log | tail -5
exit $rc
