# Round 3: BN GPU tests + ResNet-50 A/B of the finished BN statistics (ARENA_BN_FINAL=1 vs 0),
# alternating processes so clock/thermal drift hits both arms; then a rocprofv3 steady-state
# kernel breakdown of the default arm. FULL=1 runs the whole GPU suite first.
set -o pipefail
mkdir -p gpurun_out
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -n 80 gpurun_out/r3_pytest_gpu.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 \
    || { tail -n 80 gpurun_out/r3_pytest_gpu.log; exit 1; }
fi
tail -n 3 gpurun_out/r3_pytest_gpu.log
: > gpurun_out/r3_bn_final_ab.jsonl
for rep in 1 2 3; do
  for fin in 1 0; do
    ARENA_BN_FINAL=$fin timeout -k 10 240 python -m arena_amd.examples.cnn_bench --model resnet50 \
      --batch_size 128 --num_batches 40 --num_warmup_batches 8 --json 2>/dev/null \
      | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['bn_final']=$fin; print(json.dumps(d))" \
      >> gpurun_out/r3_bn_final_ab.jsonl || exit 1
  done
done
cat gpurun_out/r3_bn_final_ab.jsonl
if [ "${PROF:-1}" = 1 ]; then
  rm -rf gpurun_out/r3_prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_prof \
    -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
    --num_batches 30 --num_warmup_batches 8 > gpurun_out/r3_prof.log 2>&1 || exit 1
  TRACE=$(find gpurun_out/r3_prof -name '*kernel_trace.csv' | head -1)
  python scripts/steady_kernels.py "$TRACE" --top 30 --last-ms 150 \
    --csv gpurun_out/r3_steady_kernels.csv > gpurun_out/r3_steady_summary.txt
  cat gpurun_out/r3_steady_summary.txt | head -40
  rm -rf gpurun_out/r3_prof
fi
