# round 5: 4 vs 8 accumulator replicas (every layer summed in the conv epilogue), cross-build
# A/B on one box: the tree (ARENA_ACC_REP 4) against abtree/r8
set -o pipefail
mkdir -p gpurun_out
R=$PWD
for arm in r4 r8 r4 r8 r4 r8; do
  if [ $arm = r8 ]; then
    cd "$R/abtree/r8"
  else
    cd "$R"
  fi
  timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
    --num_batches 60 --num_warmup_batches 8 > "$R/gpurun_out/r5_acc2_$arm.out" \
    2> "$R/gpurun_out/r5_acc2_$arm.err" || exit 1
  grep "total images/sec" "$R/gpurun_out/r5_acc2_$arm.out" | sed "s/^/$arm /"
done
