#!/bin/bash
# xGMI pull protocol + per-kernel self-test + bench ccl key (round 6 item 1/2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_xgmi_gpu.py tests/test_bench_gpu.py -m gpu > gpurun_out/r6_xgmi_tests.log 2>&1
rc=$?
tail -40 gpurun_out/r6_xgmi_tests.log
exit $rc
