#!/bin/bash
# bench.py's multi-rank path rehearsed with W ranks sharing this box's GPU (the driver's SCALE runs
# use one GPU per rank): MNIST DP (xGMI Adam, replica-verified), ResNet-50 DP (sharded SGD), ccl table
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r6r}
for W in 4 8; do
  timeout -k 10 500 python -u bench.py --gpus $W --same-gpu --steps 120 --warmup 20 --verify-every 60 \
    --resnet-batch 32 --resnet-steps 6 > gpurun_out/${T}_bench_sg$W.json 2> gpurun_out/${T}_bench_sg$W.err \
    || { echo "W=$W failed rc=$?"; tail -30 gpurun_out/${T}_bench_sg$W.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${T}_bench_sg$W.json').read().strip().splitlines()[-1])
print('W=$W', d['value'], d['config']['parallelism'], d['config'].get('exec'), 'failed=', d.get('failed'))
print(' resnet', d.get('resnet50_images_per_s'), d.get('resnet50_config',{}).get('comm'))
print(' xgmi', d.get('xgmi') or (d.get('ccl') or {}).get('xgmi'))
"
done
