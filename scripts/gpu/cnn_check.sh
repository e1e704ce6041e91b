#!/bin/bash
# GPU: BN + conv kernel tests, an in-process A/B of ResNet-50 bs128 steps, the glue-op
# attribution (torch.profiler) and a rocprofv3 steady-state kernel breakdown.
# Outputs under gpurun_out/cnn_check/. STEPS (comma list) picks a subset: tests,ab,glue,prof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cnn_check
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,ab,glue,prof}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 420 python -u -m pytest tests/test_bn_gpu.py tests/test_conv.py -m gpu -x -v \
      --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
      || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
if has ab; then
  timeout -k 10 600 python scripts/cnn_ab.py --modes ${MODES:-auto,miopen} --batch 128 \
      --rounds ${ROUNDS:-4} > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err"; exit 1; }
  cat "$OUT/ab.jsonl"
fi
if has glue; then
  timeout -k 10 300 python scripts/cnn_glue_prof.py > "$OUT/glue.txt" 2> "$OUT/glue.err" \
      || { tail -20 "$OUT/glue.err"; exit 1; }
  grep -A30 -- "--- per op ---" "$OUT/glue.txt" | head -20
fi
if has prof; then
  ARENA_CONV_LOG=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof" -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 \
      --batch_size 128 --num_batches 30 --num_warmup_batches 8 --json \
      > "$OUT/r50.log" 2> "$OUT/r50.err" || { tail -20 "$OUT/r50.err"; exit 1; }
  tail -1 "$OUT/r50.log"
  TRACE=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
  python3 scripts/steady_kernels.py "$TRACE" --last-ms 400 --top 45 --csv "$OUT/steady_top.csv" \
      > "$OUT/steady.txt" 2>&1 || true
  head -12 "$OUT/steady.txt"
  rm -f "$TRACE"   # ~100 MB: keep the summaries only (gpurun copies back at most 64 MiB)
fi
