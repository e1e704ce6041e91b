#!/bin/bash
# BN apply / dx passes with the first data loads issued ahead of the coefficient prologue (tree)
# vs without (ab_old/, the previous commit's build): BN GPU tests, then alternating processes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r6p}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_gpu.py tests/test_cnn.py -m gpu > gpurun_out/${T}_bn_tests.log 2>&1 || { tail -30 gpurun_out/${T}_bn_tests.log; exit 1; }
tail -1 gpurun_out/${T}_bn_tests.log
: > gpurun_out/${T}_ab.jsonl
for rep in 1 2; do
  for arm in new old; do
    dir=.; [ $arm = old ] && dir=ab_old
    timeout -k 10 200 python -u $dir/tools/bn_pass_bw.py --configs slice:1024 2>> gpurun_out/${T}_ab.err | tail -1 | sed "s/^/{\"arm\": \"$arm\", \"rep\": $rep, \"bn\": /; s/\$/}/" >> gpurun_out/${T}_ab.jsonl || exit 1
    timeout -k 10 300 python -u $dir/tools/cnn_ab.py --modes auto --rounds 6 2>> gpurun_out/${T}_ab.err | sed "s/^/{\"arm\": \"$arm\", \"rep\": $rep, \"step\": /; s/\$/}/" >> gpurun_out/${T}_ab.jsonl || exit 1
  done
done
cut -c1-300 gpurun_out/${T}_ab.jsonl
