# round 5: down_bn's backward sums added by bn3's dx pass (no down_bn reduction pass) -- BN / conv
# / ResNet GPU tests, then a step A/B against down_bn reducing itself
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_bn_gpu.py tests/test_conv.py tests/test_bn_fold.py tests/test_trainer_gpu.py \
  > gpurun_out/r5_t26a.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r5_t26a.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/cnn_ab.py --modes auto,auto:noressums,auto,auto:noressums \
  --rounds 8 --chunk 10 > gpurun_out/r5_ressums_ab.jsonl 2> gpurun_out/r5_ressums_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_ressums_ab.jsonl
