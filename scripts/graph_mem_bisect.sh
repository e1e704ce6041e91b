#!/bin/bash
# GPU: graph_mem_check.py over feature switches (see that script). Outputs gpurun_out/memchk_*.txt
# CFG_LIST: newline-separated "label options..." lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG_LIST=${CFG_LIST:-"auto --mode auto"}
while read -r label opts; do
  [ -z "$label" ] && continue
  timeout -k 10 240 python scripts/graph_mem_check.py $opts > "gpurun_out/memchk_$label.txt" 2>&1 \
    || { echo "$label: rc=$?"; tail -3 "gpurun_out/memchk_$label.txt"; exit 1; }
  echo "$label: $(grep 'replay 3' gpurun_out/memchk_$label.txt)"
done <<< "$CFG_LIST"
