# round 5: steady-state kernel profile of the final ResNet-50 step (rocprofv3 kernel trace, last
# 150 ms of a 40-batch run) and the per-layer plan log of the same build
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
  -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
  --num_batches 30 --num_warmup_batches 8 > gpurun_out/r5_prof_final.log 2>&1
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -n 20 gpurun_out/r5_prof_final.log; exit $rc; fi
TRACE=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python tools/steady_kernels.py "$TRACE" --top 60 --last-ms 150 \
  --csv gpurun_out/r5_final_steady_kernels.csv > gpurun_out/r5_final_steady_summary.txt
rm -rf gpurun_out/prof
cat gpurun_out/r5_final_steady_summary.txt
ARENA_CONV_LOG=1 timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 \
  --batch_size 128 --num_batches 40 --num_warmup_batches 5 > gpurun_out/r5_final_plan.out \
  2> gpurun_out/r5_final_plan.log
echo "plan rc=$?"; grep "total images/sec" gpurun_out/r5_final_plan.out
