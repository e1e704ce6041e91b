# round 5: v2 split-K -- kernel numerics, the per-layer plan with split candidates, and an
# in-process A/B against the plan without them
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_conv.py -k "split or v2_matches" > gpurun_out/r5_t5a.log 2>&1
rc=$?; echo "conv split tests rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
ARENA_CONV_LOG=1 timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 \
  --batch_size 128 --num_batches 20 --num_warmup_batches 3 > gpurun_out/r5_split_plan.out 2> gpurun_out/r5_split_plan.log
rc=$?; echo "plan log rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 480 python -u tools/cnn_ab.py --modes auto,auto:v2split --rounds 6 \
  > gpurun_out/r5_split_ab.jsonl 2> gpurun_out/r5_split_ab.err
echo "ab rc=$?"
