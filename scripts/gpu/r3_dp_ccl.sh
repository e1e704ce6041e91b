# Round 3: data-parallel rehearsals with 2 ranks sharing GPU 0 (xGMI kernels over same-device
# hipIpc mappings: protocol and launch cost, not link bandwidth): the collective sweep
# (allreduce, fused Adam, broadcast, all-gather, sharded bf16 SGD) and the ResNet-50 DP step with
# the sharded bf16 master SGD, eager and as a hipGraph, with its replica check.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ccl_bench.py --same-gpu 2 > gpurun_out/r3_ccl_same_gpu.jsonl \
  2> gpurun_out/r3_ccl_same_gpu.err || { tail -n 30 gpurun_out/r3_ccl_same_gpu.err; exit 1; }
cat gpurun_out/r3_ccl_same_gpu.jsonl | cut -c1-220
for g in 0 1; do
  timeout -k 10 400 python scripts/dp_cnn_same_gpu.py --world 2 --model resnet50 --batch_size 32 \
    --steps 20 --graph $g >> gpurun_out/r3_dp_cnn_same_gpu.jsonl 2>> gpurun_out/r3_dp_cnn_same_gpu.err \
    || { tail -n 30 gpurun_out/r3_dp_cnn_same_gpu.err; exit 1; }
done
cat gpurun_out/r3_dp_cnn_same_gpu.jsonl | cut -c1-400
