#!/bin/bash
# GPU: graph_mem_check in "ours" mode with one direction forced to MIOpen (ARENA_CONV_DIRS),
# two runs each, eager kernels between replays.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for d in "bwd,wgrad" "fwd,wgrad" "fwd,bwd"; do
    label="miopen_$(echo fwd,bwd,wgrad | tr ',' '\n' | grep -vxF -f <(echo $d | tr ',' '\n'))"
    ARENA_CONV_DIRS=$d timeout -k 10 240 python scripts/graph_mem_check.py --mode ours \
        --eager_kernel torch_small --eager_n 400 > "gpurun_out/md_${label}_$rep.txt" 2>&1 \
        || { echo "$label $rep: rc=$?"; exit 1; }
    echo "$label $rep: $(grep 'replay 3' gpurun_out/md_${label}_$rep.txt)"
  done
done
