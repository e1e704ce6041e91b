#!/bin/bash
# GPU: repeat graph_mem_check over configs (flaky failure -> several runs each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for cfg in ${CFGS:-"auto_tgraph|0|--mode auto" "auto_teager|1|--mode auto" "ours|0|--mode ours" "miopen|0|--mode miopen"}; do
    IFS='|' read -r label teager opts <<< "$cfg"
    ARENA_CONV_TIME_EAGER=$teager timeout -k 10 240 python scripts/graph_mem_check.py $opts \
        --eager_kernel torch_small --eager_n 400 > "gpurun_out/mm_${label}_$rep.txt" 2>&1 \
        || { echo "$label $rep: rc=$?"; exit 1; }
    echo "$label $rep: $(grep 'replay 3' gpurun_out/mm_${label}_$rep.txt)"
  done
done
