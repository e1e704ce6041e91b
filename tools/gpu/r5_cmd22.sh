# round 5: single-process GPU suites + smoke on the sliced-BN build, grid-size A/B around the new
# defaults (apply / dx block caps), and the driver-form bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_fold.py tests/test_bn_gpu.py tests/test_conv.py tests/test_ops_gpu.py \
  tests/test_optim.py tests/test_pool_gpu.py tests/test_trainer_gpu.py \
  > gpurun_out/r5_t22a.log 2>&1
rc=$?; echo "gpu tests A rc=$rc"; tail -n 3 gpurun_out/r5_t22a.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
rc=$?; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/cnn_ab.py \
  --modes auto,auto:ebk512,auto:ebk2048,auto:dxb512,auto:dxb2048 --rounds 8 --chunk 10 \
  > gpurun_out/r5_grid_ab.jsonl 2> gpurun_out/r5_grid_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_grid_ab.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench_n1c.json 2> gpurun_out/r5_bench_n1c.err
echo "bench rc=$?"; cat gpurun_out/r5_bench_n1c.json
