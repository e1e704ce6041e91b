#!/bin/bash
# ResNet head kernels: pool / xent GPU tests, the CNN tests, then the step's framework kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pool_gpu.py tests/test_cnn.py tests/test_trainer_gpu.py -m gpu > gpurun_out/r6hp_tests.log 2>&1 || { tail -30 gpurun_out/r6hp_tests.log; exit 1; }
tail -1 gpurun_out/r6hp_tests.log
bash tools/gpu/kernel_neighbors.sh > /dev/null 2>&1 || { tail -5 gpurun_out/nb.log; exit 1; }
grep "^----" gpurun_out/nb.txt | cut -c1-150
grep "images/sec" gpurun_out/nb.log | tail -1
