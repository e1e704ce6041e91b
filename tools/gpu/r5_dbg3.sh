# round 5: is the W = 8 weight divergence in the build's broadcast? model-sized broadcasts at
# W = 2 and 8, then the existing broadcast/all-gather tests at W = 8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_xgmi_gpu.py -k "model_sized_broadcast or broadcast_allgather_bit_exact" \
  > gpurun_out/r5_dbg3.log 2>&1
echo "rc=$?"; grep -E "PASSED|FAILED|AssertionError" gpurun_out/r5_dbg3.log | head -20
