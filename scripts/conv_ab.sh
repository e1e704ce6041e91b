#!/bin/bash
# GPU: conv kernel tests, then an in-process interleaved A/B of ResNet-50 bs128 training steps
# with MIOpen convolutions vs the autotuned MFMA kernels. Outputs under gpurun_out/conv_ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/conv_ab
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 900 python scripts/cnn_ab.py --modes ${MODES:-miopen,auto} --batch 128 \
    > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err"; exit 1; }
cat "$OUT/ab.jsonl"
