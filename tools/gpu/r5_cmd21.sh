# round 5: BN apply / dx passes with 256-channel-sliced grids for C > 256 and a dx block cap --
# BN suites, the per-shape bandwidth probe over the grid configs, then an in-process step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bn_gpu.py tests/test_bn_fold.py tests/test_pool_gpu.py > gpurun_out/r5_t21a.log 2>&1
rc=$?; echo "bn tests rc=$rc"; tail -n 2 gpurun_out/r5_t21a.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bn_pass_bw.py --configs flat:4096,slice:4096,slice:1024,flat:1024 \
  > gpurun_out/r5_bn_pass_bw2.jsonl 2> gpurun_out/r5_bn_pass_bw2.err
echo "probe rc=$?"; grep -E "config|us_per_step" gpurun_out/r5_bn_pass_bw2.jsonl
timeout -k 10 600 python -u tools/cnn_ab.py --modes auto,auto:noslice,auto:dxb1024,auto:noslice+dxb1024 \
  --rounds 8 --chunk 10 > gpurun_out/r5_slice_ab.jsonl 2> gpurun_out/r5_slice_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_slice_ab.jsonl
