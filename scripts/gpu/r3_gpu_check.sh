# Round-3 GPU checks: new xGMI kernels (broadcast/allgather/sharded SGD), ADVICE conv fixes,
# the sharded DP ResNet rehearsal on one GPU, then the MNIST graph-length sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_xgmi_gpu.py tests/test_conv.py \
  -k "broadcast or sharded or oversized or async_wgrad or keeps_buffers or rejects or hipgraph_matches" \
  > gpurun_out/r3_new_gpu_tests.log 2>&1 || { tail -n 60 gpurun_out/r3_new_gpu_tests.log; exit 1; }
tail -n 5 gpurun_out/r3_new_gpu_tests.log
timeout -k 10 300 python scripts/dp_cnn_same_gpu.py --world 2 --model resnet50 --batch_size 32 \
  --steps 10 --warmup 3 --graph 1 > gpurun_out/r3_dp_cnn_w2.json 2> gpurun_out/r3_dp_cnn_w2.err \
  || { tail -n 30 gpurun_out/r3_dp_cnn_w2.err; exit 1; }
cat gpurun_out/r3_dp_cnn_w2.json
bash scripts/spg_sweep.sh && cat gpurun_out/spg_sweep.txt
