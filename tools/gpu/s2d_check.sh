# Space-to-depth stem kernel after the vector-load / 32-bit-index rewrite: layout and conv tests,
# then the steady ResNet-50 kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py tests/test_pool_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "s2d or stem" > gpurun_out/s2d_tests.log 2>&1 \
  || { tail -n 60 gpurun_out/s2d_tests.log; exit 1; }
tail -n 2 gpurun_out/s2d_tests.log
TOPN=60 bash tools/gpu/prof.sh
