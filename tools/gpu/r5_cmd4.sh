# round 5: block-level fold test (same variants), data-parallel W = 8 tests, bench self-launch
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bn_fold.py -k bottleneck > gpurun_out/r5_t4a.log 2>&1
rc=$?; echo "fold block rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_optim.py tests/test_planstore.py tests/test_xgmi_gpu.py tests/test_bench_gpu.py > gpurun_out/r5_t4b.log 2>&1
echo "dp tests rc=$?"
