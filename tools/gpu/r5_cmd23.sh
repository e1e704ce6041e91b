# round 5 final check, part B on the sliced-BN build: the multi-process suites (xGMI / DP / plan
# sharing / bench self-launch), the N=2 same-GPU bench line, then the steady-state kernel profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_planstore.py tests/test_xgmi_gpu.py tests/test_bench_gpu.py \
  > gpurun_out/r5_final_b.log 2>&1
rc=$?; echo "gpu tests B rc=$rc"; tail -n 3 gpurun_out/r5_final_b.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --gpus 2 --same-gpu > gpurun_out/r5_bench_n2_same.json \
  2> gpurun_out/r5_bench_n2_same.err
rc=$?; echo "bench n2 same-gpu rc=$rc"; cat gpurun_out/r5_bench_n2_same.json; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/r5_prof_final.sh
