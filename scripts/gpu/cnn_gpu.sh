#!/bin/bash
# ResNet-50 synthetic-ImageNet training on one MI355X (tf_cnn_benchmarks shape), then a
# rocprofv3 kernel-stats pass. Outputs under gpurun_out/cnn/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cnn
mkdir -p "$OUT"
export TMPDIR=/tmp
BS=${BS:-128}
timeout -k 10 900 python -m arena_amd.examples.cnn_bench --model resnet50 --batch_size "$BS" \
    --num_batches 60 --num_warmup_batches 8 --json > "$OUT/r50_bs$BS.log" 2>&1 || exit $?
tail -3 "$OUT/r50_bs$BS.log"
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o r50 -- \
      python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size "$BS" \
      --num_batches 20 --num_warmup_batches 5 > "$OUT/prof.log" 2>&1 || exit $?
  find "$OUT/prof" -name '*kernel_stats.csv' -exec head -25 {} \; | cut -c1-150
fi
