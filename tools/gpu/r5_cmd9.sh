# round 5: LDS fragment prefetch in the v2 pipelined / halo MFMA loops, A/B on one box: the tree
# build (ARENA_CONV_PF=1) against a copy of the package linked with conv_kernels built with
# -DARENA_CONV_PF=0 (abtree/pf0); per-layer plan timings and cnn_bench throughput, alternated
set -o pipefail
mkdir -p gpurun_out
R=$PWD
for arm in pf1 pf0 pf1 pf0; do
  if [ $arm = pf0 ]; then cd "$R/abtree/pf0"; else cd "$R"; fi
  ARENA_CONV_LOG=1 timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 \
    --batch_size 128 --num_batches 40 --num_warmup_batches 5 > "$R/gpurun_out/r5_$arm.out" \
    2> "$R/gpurun_out/r5_${arm}_plan.log" || exit 1
  grep "total images/sec" "$R/gpurun_out/r5_$arm.out" | sed "s/^/$arm /"
done
