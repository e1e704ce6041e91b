#!/bin/bash
# new halo variants: numerics (test_conv v2 tests) then the ablation timing of every halo form
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_conv.py -m gpu -k "v2" > gpurun_out/${TAG:-r6h}_conv_tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-r6h}_conv_tests.log; exit 1; }
tail -2 gpurun_out/${TAG:-r6h}_conv_tests.log
timeout -k 10 400 python -u tools/halo_ablation.py > gpurun_out/${TAG:-r6h}_halo_ablation.jsonl 2> gpurun_out/${TAG:-r6h}_halo_ablation.err
