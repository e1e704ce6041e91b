#!/bin/bash
# whole-step A/B of the 8-wave halo forms (interleaved graph replays, one process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r6hw}
timeout -k 10 700 python -u tools/cnn_ab.py --modes auto,auto:nohalowide,auto,auto:nohalowide --rounds 8 \
  > gpurun_out/${T}_ab.jsonl 2> gpurun_out/${T}_ab.err || { tail -20 gpurun_out/${T}_ab.err; exit 1; }
cat gpurun_out/${T}_ab.jsonl
