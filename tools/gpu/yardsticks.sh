#!/bin/bash
# fair 1x1 BLAS yardstick (split-K wgrad) + BN pass byte-floor table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/conv_vs_blas.py --batch 128 > gpurun_out/${TAG}_conv_vs_blas.jsonl 2> gpurun_out/${TAG}_conv_vs_blas.err && \
timeout -k 10 200 python -u tools/bn_pass_bw.py --configs slice:1024 > gpurun_out/${TAG}_bn_pass_bw.jsonl 2> gpurun_out/${TAG}_bn_pass_bw.err
rc=$?
tail -2 gpurun_out/${TAG}_conv_vs_blas.jsonl; tail -1 gpurun_out/${TAG}_bn_pass_bw.jsonl
exit $rc
