# Round 3: finalize-free BatchNorm (coefficients derived in the apply / dx passes): BN + conv GPU
# tests, then a same-process ResNet-50 A/B (conv-epilogue acc threshold, backward sums in the
# layer's own set vs pool + finalize), then a steady-state kernel profile of the default.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_bn_gpu.py tests/test_cnn.py ${EXTRA_TESTS:-} > gpurun_out/r3_bnfin_tests.log 2>&1 \
  || { tail -n 60 gpurun_out/r3_bnfin_tests.log; exit 1; }
tail -n 2 gpurun_out/r3_bnfin_tests.log
timeout -k 10 500 python scripts/cnn_ab.py --modes "${MODES:-auto,auto:finbwd0,auto:accP100000000}" \
  --rounds ${ROUNDS:-6} > gpurun_out/r3_bnfin_ab.jsonl 2> gpurun_out/r3_bnfin_ab.err \
  || { tail -n 30 gpurun_out/r3_bnfin_ab.err; exit 1; }
cat gpurun_out/r3_bnfin_ab.jsonl
[ "${PROF:-1}" = 1 ] || exit 0
rm -rf gpurun_out/r3_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_prof \
  -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 \
  --num_batches 30 --num_warmup_batches 8 > gpurun_out/r3_prof.log 2>&1 || { tail -n 20 gpurun_out/r3_prof.log; exit 1; }
TRACE=$(find gpurun_out/r3_prof -name '*kernel_trace.csv' | head -1)
python scripts/steady_kernels.py "$TRACE" --top 40 --last-ms 150 \
  --csv gpurun_out/r3_steady_kernels.csv > gpurun_out/r3_steady_summary.txt
rm -rf gpurun_out/r3_prof
cat gpurun_out/r3_steady_summary.txt
tail -n 2 gpurun_out/r3_prof.log
