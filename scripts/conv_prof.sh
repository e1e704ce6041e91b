#!/bin/bash
# GPU: kernel stats of ResNet-50 bs128 with the autotuned conv kernels (+ the per-shape choices).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/conv_prof
mkdir -p "$OUT"
export TMPDIR=/tmp
ARENA_CONV_LOG=1 ARENA_CONV=${MODE:-auto} timeout -k 10 600 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$OUT/prof" -o r50 -- python3 -m arena_amd.examples.cnn_bench \
    --model resnet50 --batch_size 128 --num_batches 30 --num_warmup_batches 8 --json \
    > "$OUT/r50.log" 2> "$OUT/r50.err" || { tail -20 "$OUT/r50.err"; exit 1; }
tail -1 "$OUT/r50.log"
TRACE=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 scripts/steady_kernels.py "$TRACE" --last-ms 400 --top 40 --csv "$OUT/steady_top.csv" \
    > "$OUT/steady.txt" 2>&1 || true
cat "$OUT/steady.txt"
head -41 "$OUT/steady_top.csv" | cut -c1-170
