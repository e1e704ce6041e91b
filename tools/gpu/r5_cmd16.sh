# round 5: BN pass grid cap 1024 by default -- BN / fold / pool suites and the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_gpu.py tests/test_bn_fold.py tests/test_pool_gpu.py > gpurun_out/r5_t16a.log 2>&1
rc=$?; echo "bn tests rc=$rc"; tail -n 2 gpurun_out/r5_t16a.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench_n1b.json 2> gpurun_out/r5_bench_n1b.err
echo "bench rc=$?"; cat gpurun_out/r5_bench_n1b.json
