#!/bin/bash
# GPU: conv/BN tests, then the captured ResNet-50 step replayed after eager GPU/host churn
# (scripts/graph_mem_check.py) REPS times -- every run must reproduce the same losses -- then an
# A/B timing. Outputs gpurun_out/safety/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/safety
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_conv.py tests/test_bn_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in $(seq 1 ${REPS:-5}); do
  timeout -k 10 240 python scripts/graph_mem_check.py --mode ${MODE:-auto} --eager_kernel torch_small \
      --eager_n 400 > "$OUT/mem_$rep.txt" 2>&1 || { tail -5 "$OUT/mem_$rep.txt"; exit 1; }
  echo "run $rep: $(grep -E 'replay (0|3)' "$OUT/mem_$rep.txt" | tr '\n' ' ')"
done
if [ "${AB:-1}" = 1 ]; then
  timeout -k 10 600 python scripts/cnn_ab.py --modes auto,auto --batch 128 --rounds 4 \
      > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err"; exit 1; }
  cat "$OUT/ab.jsonl"
fi
