# round 5: where the BN fold costs time -- per-layer plan timings (fold vs plain forms) and the
# steady-state kernel breakdown with the fold on and off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bn_fold.py > gpurun_out/r5_t3.log 2>&1
rc=$?; echo "fold tests rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
ARENA_CONV_LOG=1 timeout -k 10 300 python -u -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 --num_batches 20 --num_warmup_batches 3 > gpurun_out/r5_fold_plan.out 2> gpurun_out/r5_fold_plan.log
echo "plan log rc=$?"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for arm in fold nofold; do
  rm -rf gpurun_out/prof
  if [ $arm = nofold ]; then export ARENA_BN_FOLD=0; else export ARENA_BN_FOLD=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
    -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
    --num_batches 30 --num_warmup_batches 8 > gpurun_out/r5_prof_$arm.log 2>&1 || { tail -n 20 gpurun_out/r5_prof_$arm.log; exit 1; }
  TRACE=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
  python tools/steady_kernels.py "$TRACE" --top 60 --last-ms 150 \
    --csv gpurun_out/r5_steady_kernels_$arm.csv > gpurun_out/r5_steady_summary_$arm.txt
  rm -rf gpurun_out/prof
  echo "prof $arm done"
done
