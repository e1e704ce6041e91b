#!/bin/bash
# 8-wave halo variants (V2+16..18): numerics, per-layer timings, the tuned conv budget, step time
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r6w8}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py -m gpu > gpurun_out/${T}_conv_tests.log 2>&1 || { tail -30 gpurun_out/${T}_conv_tests.log; exit 1; }
tail -1 gpurun_out/${T}_conv_tests.log
FLAGS=0 timeout -k 10 300 python -u tools/halo_ablation.py > gpurun_out/${T}_halo_variants.jsonl 2> gpurun_out/${T}_halo.err || { tail -20 gpurun_out/${T}_halo.err; exit 1; }
cat gpurun_out/${T}_halo_variants.jsonl
timeout -k 10 300 python -u tools/conv_budget.py > gpurun_out/${T}_conv_budget.md 2> gpurun_out/${T}_budget.err || { tail -5 gpurun_out/${T}_budget.err; exit 1; }
head -16 gpurun_out/${T}_conv_budget.md
timeout -k 10 400 python -u tools/cnn_ab.py --modes auto --rounds 6 2> gpurun_out/${T}_ab.err | tail -1
