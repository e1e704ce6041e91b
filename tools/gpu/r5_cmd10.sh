# round 5: conv suite (v1/v2 split hand-off now write-through), the DP / bench suites after the
# collective XgmiComm.close, and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_conv.py > gpurun_out/r5_t10a.log 2>&1
rc=$?; echo "conv tests rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_xgmi_gpu.py tests/test_bench_gpu.py > gpurun_out/r5_t10b.log 2>&1
rc=$?; echo "dp tests rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench_default.json 2> gpurun_out/r5_bench_default.err
echo "bench rc=$?"; cat gpurun_out/r5_bench_default.json
