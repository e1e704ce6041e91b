# round 5: per-layer BNGradLink pricing (link only where the linked dgrad epilogue beats the BN's own
# reduction pass) and the stem backward's sums from the forward's saved argmax inputs -- conv / BN /
# pool suites, one cnn_bench with the plan log, then an in-process A/B against always-link and the
# per-pixel stem reduction (interleaved graph replays)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_conv.py tests/test_bn_gpu.py tests/test_pool_gpu.py > gpurun_out/r5_t18a.log 2>&1
rc=$?; echo "conv/bn tests rc=$rc"; tail -n 2 gpurun_out/r5_t18a.log; if [ $rc -ne 0 ]; then exit $rc; fi
ARENA_CONV_LOG=1 timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 \
  --batch_size 128 --num_batches 60 --num_warmup_batches 8 > gpurun_out/r5_link_bench.out \
  2> gpurun_out/r5_link_plan.log
echo "cnn_bench rc=$?"; grep "total images/sec" gpurun_out/r5_link_bench.out
grep -c "link=False" gpurun_out/r5_link_plan.log
timeout -k 10 600 python -u tools/cnn_ab.py --modes auto,auto:linkall,auto:noxsel --rounds 8 \
  --chunk 10 > gpurun_out/r5_link_ab.jsonl 2> gpurun_out/r5_link_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_link_ab.jsonl
