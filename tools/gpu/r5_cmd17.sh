# round 5: BN dx pass unrolled by two (loads of both vectors before the first store) -- BN suites,
# then a cross-build A/B against abtree/base (the same tree without the unroll), alternating runs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_gpu.py tests/test_bn_fold.py tests/test_pool_gpu.py > gpurun_out/r5_t17a.log 2>&1
rc=$?; echo "bn tests rc=$rc"; tail -n 2 gpurun_out/r5_t17a.log; if [ $rc -ne 0 ]; then exit $rc; fi
R=$PWD
for arm in u2 base u2 base u2 base; do
  if [ $arm = base ]; then cd "$R/abtree/base"; else cd "$R"; fi
  timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
    --num_batches 60 --num_warmup_batches 8 > "$R/gpurun_out/r5_dx_$arm.out" \
    2> "$R/gpurun_out/r5_dx_$arm.err" || exit 1
  grep "total images/sec" "$R/gpurun_out/r5_dx_$arm.out" | sed "s/^/$arm /"
done
