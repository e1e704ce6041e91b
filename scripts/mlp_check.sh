#!/bin/bash
# MNIST kernel iteration on the GPU box: kernel/trainer/xGMI numerics tests, then the flagship bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_trainer_gpu.py tests/test_xgmi_gpu.py > gpurun_out/mlp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mlp_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err || exit $?
  cut -c1-160 gpurun_out/bench_$i.json
done
