# round 5: collectives of ranks sharing one GPU capped at 128 / W blocks per launch -- the
# model-sized broadcast and the DP step at W = 8, then the rest of the multi-process suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_xgmi_gpu.py -k "model_sized_broadcast or dp_resnet_sharded" > gpurun_out/r5_dbg4.log 2>&1
echo "rc=$?"; grep -E "PASSED|FAILED|AssertionError" gpurun_out/r5_dbg4.log | head -20
