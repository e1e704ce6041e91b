timeout -k 10 800 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_optim.py tests/test_planstore.py tests/test_xgmi_gpu.py tests/test_bench_gpu.py > gpurun_out/r5_t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 330 python -u tools/conv_vs_blas.py --batch 128 > gpurun_out/r5_conv_vs_blas.jsonl 2> gpurun_out/r5_conv_vs_blas.err
  echo "blas rc=$?"
fi
