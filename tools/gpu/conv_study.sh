#!/bin/bash
# 3x3 halo ablation + per-class conv budget (round 6 conv study), outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/halo_ablation.py > gpurun_out/${TAG:-r6}_halo_ablation.jsonl 2> gpurun_out/${TAG:-r6}_halo_ablation.err && \
timeout -k 10 500 python -u tools/conv_budget.py > gpurun_out/${TAG:-r6}_conv_budget.md 2> gpurun_out/${TAG:-r6}_conv_budget.err
rc=$?
tail -3 gpurun_out/${TAG:-r6}_halo_ablation.err
head -20 gpurun_out/${TAG:-r6}_conv_budget.md
exit $rc
