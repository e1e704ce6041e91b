# round 5: replicated BatchNorm accumulators (abi.h ARENA_ACC_REP) -- BN / fold / conv suites,
# then the epilogue-sum thresholds A/B (the replicas cut same-address atomic chains 4x)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_gpu.py tests/test_bn_fold.py tests/test_conv.py > gpurun_out/r5_t11a.log 2>&1
rc=$?; echo "bn/conv tests rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/cnn_ab.py \
  --modes auto,auto:accP524288+laccP524288,auto:accP1048576+laccP1048576 --rounds 6 \
  > gpurun_out/r5_accrep_ab.jsonl 2> gpurun_out/r5_accrep_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_accrep_ab.jsonl
