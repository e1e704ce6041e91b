#!/bin/bash
# Fused-BN numerics tests, then ResNet-50 throughput with the fused kernels (no profiler pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cnn
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bn_gpu.py > gpurun_out/bn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
PROF=${PROF:-0} bash scripts/cnn_gpu.sh
