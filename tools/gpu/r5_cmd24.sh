# round 5: downsample shortcut built after the main path (conv1's stride-1 dgrad completes the join
# and takes the block input's BN-backward sums) -- ResNet GPU tests, step A/B, and a kernel-count
# profile (the unlinked bn_bwd_reduce launches per step should drop)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_conv.py tests/test_trainer_gpu.py tests/test_xgmi_gpu.py -k "resnet or cnn or dp" \
  > gpurun_out/r5_t24a.log 2>&1
rc=$?; echo "resnet tests rc=$rc"; tail -n 3 gpurun_out/r5_t24a.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/cnn_ab.py --modes auto,auto:downfirst,auto,auto:downfirst \
  --rounds 8 --chunk 10 > gpurun_out/r5_down_ab.jsonl 2> gpurun_out/r5_down_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_down_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof24
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof24 \
  -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
  --num_batches 20 --num_warmup_batches 4 > gpurun_out/r5_prof24.log 2>&1
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -n 20 gpurun_out/r5_prof24.log; exit $rc; fi
TRACE=$(find gpurun_out/prof24 -name '*kernel_trace.csv' | head -1)
python tools/steady_kernels.py "$TRACE" --top 60 --last-ms 150 \
  --csv gpurun_out/r5_down_steady_kernels.csv > gpurun_out/r5_down_steady_summary.txt
rm -rf gpurun_out/prof24
cat gpurun_out/r5_down_steady_summary.txt; grep -E "bn_bwd_reduce|bn_bwd_dx" gpurun_out/r5_down_steady_kernels.csv
