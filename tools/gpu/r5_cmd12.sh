# round 5: 16 accumulator replicas -- BN suites, then the epilogue-sum thresholds A/B again
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_gpu.py tests/test_bn_fold.py > gpurun_out/r5_t12a.log 2>&1
rc=$?; echo "bn tests rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/cnn_ab.py \
  --modes auto,auto:accP1048576+laccP1048576,auto:accP4194304+laccP4194304 --rounds 6 \
  > gpurun_out/r5_accrep16_ab.jsonl 2> gpurun_out/r5_accrep16_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_accrep16_ab.jsonl
