# round 5 final check, part A: every GPU test outside the multi-process suites, then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_fold.py tests/test_bn_gpu.py tests/test_conv.py tests/test_ops_gpu.py \
  tests/test_optim.py tests/test_pool_gpu.py tests/test_trainer_gpu.py \
  > gpurun_out/r5_final_a.log 2>&1
rc=$?; echo "gpu tests A rc=$rc"; tail -n 3 gpurun_out/r5_final_a.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
