# End-to-end GPU check at HEAD: full GPU suite, smoke(), the driver's bench invocation
# (--steps 20 --warmup 5, MNIST headline + ResNet-50 keys) and the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 80 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { tail -n 40 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json \
  2> gpurun_out/bench_driver.err || { tail -n 40 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 python bench.py --resnet 0 > gpurun_out/bench_default.json \
  2> gpurun_out/bench_default.err || { tail -n 40 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
