# round 5: data-parallel checks on one GPU -- sharded SGD / DP ResNet at W = 2, 4, 8 (xGMI and
# RCCL backends), plan sharing, bench self-launch; the bottleneck fold test; the DP overlap trace
# with mixed-dtype buckets (rank 0, HIP events per bucket)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  tests/test_optim.py tests/test_planstore.py tests/test_xgmi_gpu.py tests/test_bench_gpu.py \
  > gpurun_out/r5_t6a.log 2>&1
rc=$?; echo "dp tests rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_bn_fold.py -k bottleneck > gpurun_out/r5_t6b.log 2>&1
rc=$?; echo "fold block rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/dp_cnn_same_gpu.py --world 2 --batch_size 32 --steps 10 \
  --trace gpurun_out/r5_dp_overlap_same_gpu.jsonl > gpurun_out/r5_dp_cnn_same_gpu.json \
  2> gpurun_out/r5_dp_cnn_same_gpu.err
echo "overlap rc=$?"
