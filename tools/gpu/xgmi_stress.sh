#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/xgmi_stress.py --world 8 --rounds 3 --elems 400000 --timeout-s 10 > gpurun_out/${TAG}_stress8.jsonl 2> gpurun_out/${TAG}_stress8.err
rc=$?
cat gpurun_out/${TAG}_stress8.jsonl | cut -c1-400
exit $rc
