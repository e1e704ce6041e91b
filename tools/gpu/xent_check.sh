# Fused cross-entropy after the one-wave-per-row forward: numerics, the DP ResNet test that uses it,
# then the steady ResNet-50 kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py tests/test_xgmi_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "cross_entropy or global_avg or dp_resnet" > gpurun_out/xent_tests.log 2>&1 \
  || { tail -n 60 gpurun_out/xent_tests.log; exit 1; }
tail -n 2 gpurun_out/xent_tests.log
TOPN=50 bash tools/gpu/prof.sh
