# round 5: replicated BatchNorm accumulators, cross-build A/B on one box: the tree (1 replica,
# epilogue sums up to 128 k tile-channel pairs, the rest per-tile partials + finalize launches)
# against abtree/r4 (4 replicas, every layer's statistics summed in the conv epilogue)
set -o pipefail
mkdir -p gpurun_out
R=$PWD
for arm in r1 r4 r1 r4 r1 r4; do
  if [ $arm = r4 ]; then
    cd "$R/abtree/r4"; export ARENA_BN_ACC_MAX_PAIRS=4194304 ARENA_BN_LINK_ACC_MAX_PAIRS=4194304
  else
    cd "$R"; unset ARENA_BN_ACC_MAX_PAIRS ARENA_BN_LINK_ACC_MAX_PAIRS
  fi
  timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
    --num_batches 60 --num_warmup_batches 8 > "$R/gpurun_out/r5_acc_$arm.out" \
    2> "$R/gpurun_out/r5_acc_$arm.err" || exit 1
  grep "total images/sec" "$R/gpurun_out/r5_acc_$arm.out" | sed "s/^/$arm /"
done
