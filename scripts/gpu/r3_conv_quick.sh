# Conv kernel check + per-layer autotuned plan (no PMC): GPU conv tests, conv_plan_dump.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv.py \
  -k "${TESTK:-conv}" > gpurun_out/r3_conv_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/r3_conv_tests.log; exit 1; }
tail -n 2 gpurun_out/r3_conv_tests.log
timeout -k 10 400 python scripts/conv_plan_dump.py > gpurun_out/r3_conv_plan.jsonl \
  2> gpurun_out/r3_conv_plan.err || { tail -n 30 gpurun_out/r3_conv_plan.err; exit 1; }
tail -n 1 gpurun_out/r3_conv_plan.jsonl
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
    --num_batches 40 --num_warmup_batches 8 --json 2>/dev/null | tail -n 1
fi
