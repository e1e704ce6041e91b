# round 5: the W = 8 DP step's wrong update, with per-parameter diagnostics
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu \
  tests/test_xgmi_gpu.py -k "dp_resnet_sharded and 8" > gpurun_out/r5_dbg2.log 2>&1
echo "rc=$?"; grep -E "PASSED|FAILED|AssertionError" gpurun_out/r5_dbg2.log | head -20
