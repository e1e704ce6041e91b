#!/bin/bash
# 8-wave halo variants (V2+16..): numerics, per-layer timings, whole-step A/B against the 4-wave set
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r6w8}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py -m gpu > gpurun_out/${T}_conv_tests.log 2>&1 || { tail -30 gpurun_out/${T}_conv_tests.log; exit 1; }
tail -1 gpurun_out/${T}_conv_tests.log
FLAGS=0 timeout -k 10 300 python -u tools/halo_ablation.py > gpurun_out/${T}_halo_variants.jsonl 2> gpurun_out/${T}_halo.err || { tail -20 gpurun_out/${T}_halo.err; exit 1; }
python3 - <<PY
import json
for l in open("gpurun_out/${T}_halo_variants.jsonl"):
    d = json.loads(l); print(d["layer"], d["variant"], d["stats"], d["us"])
PY
timeout -k 10 700 python -u tools/cnn_ab.py --modes auto,auto:nohalowide,auto,auto:nohalowide --rounds 8 \
  > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err || { tail -20 gpurun_out/${T}_ab.err; exit 1; }
cut -c1-150 gpurun_out/${T}_ab.jsonl
