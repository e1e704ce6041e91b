#!/bin/bash
# grouped wgrad variants: numerics then the per-class conv budget (retuned)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_conv.py -m gpu -k "wgrad or v2" > gpurun_out/${TAG}_conv_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_conv_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_conv_tests.log
timeout -k 10 500 python -u tools/conv_budget.py > gpurun_out/${TAG}_conv_budget.md 2> gpurun_out/${TAG}_conv_budget.err
rc=$?
head -16 gpurun_out/${TAG}_conv_budget.md
exit $rc
