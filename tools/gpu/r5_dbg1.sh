# round 5: which part of the W = 8 DP step goes wrong -- W = 2 with the same large mixed buckets
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu \
  tests/test_xgmi_gpu.py -k "dp_resnet_sharded" > gpurun_out/r5_dbg1.log 2>&1
echo "rc=$?"; grep -E "PASSED|FAILED|assert " gpurun_out/r5_dbg1.log | head -20
