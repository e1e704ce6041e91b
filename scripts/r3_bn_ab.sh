# Round 3: GPU suite + ResNet-50 A/B of the finished BN statistics (ARENA_BN_FINAL=1 vs 0),
# alternating processes so clock/thermal drift hits both arms.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -n 80 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -n 3 gpurun_out/r3_pytest_gpu.log
: > gpurun_out/r3_bn_final_ab.jsonl
for rep in 1 2; do
  for fin in 1 0; do
    ARENA_BN_FINAL=$fin timeout -k 10 240 python -m arena_amd.examples.cnn_bench --model resnet50 \
      --batch_size 128 --num_batches 40 --num_warmup_batches 8 --json 2>/dev/null \
      | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['bn_final']=$fin; print(json.dumps(d))" \
      >> gpurun_out/r3_bn_final_ab.jsonl || exit 1
  done
done
cat gpurun_out/r3_bn_final_ab.jsonl
