# round 5: the data-parallel GPU tests after the W = 8 DP step went quiet for 180 s (one 0.05 MB
# bucket per tensor = ~53 eight-process rendezvous per step): progress lines (-s), 4 MB buckets at
# W = 8; then the bottleneck fold test and the DP overlap trace with mixed-dtype buckets
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_xgmi_gpu.py tests/test_bench_gpu.py > gpurun_out/r5_t8a.log 2>&1
rc=$?; echo "dp tests rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_bn_fold.py -k bottleneck > gpurun_out/r5_t8b.log 2>&1
rc=$?; echo "fold block rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/dp_cnn_same_gpu.py --world 2 --batch_size 32 --steps 10 \
  --trace gpurun_out/r5_dp_overlap_same_gpu.jsonl > gpurun_out/r5_dp_cnn_same_gpu.json \
  2> gpurun_out/r5_dp_cnn_same_gpu.err
echo "overlap rc=$?"
