# Steady-state kernel breakdown of the ResNet-50 bs128 captured training step (rocprofv3 kernel
# trace, last 150 ms) -> gpurun_out/steady_{summary.txt,kernels.csv}
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
  -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
  --num_batches 30 --num_warmup_batches 8 > gpurun_out/prof.log 2>&1 || { tail -n 20 gpurun_out/prof.log; exit 1; }
TRACE=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python tools/steady_kernels.py "$TRACE" --top ${TOPN:-40} --last-ms 150 \
  --csv gpurun_out/steady_kernels.csv > gpurun_out/steady_summary.txt
rm -rf gpurun_out/prof
cat gpurun_out/steady_summary.txt
tail -n 2 gpurun_out/prof.log
