# round 5: BN fold numerics, optimizer / plan tests, conv-vs-BLAS yardstick, fold A/B
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_bn_fold.py tests/test_optim.py tests/test_planstore.py > gpurun_out/r5_t2a.log 2>&1
rc=$?; echo "fold/optim/plan pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/conv_vs_blas.py --batch 128 > gpurun_out/r5_conv_vs_blas.jsonl 2> gpurun_out/r5_conv_vs_blas.err
rc=$?; echo "conv_vs_blas rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 420 python -u tools/cnn_ab.py --modes auto,auto:nofold --rounds 6 > gpurun_out/r5_fold_ab.jsonl 2> gpurun_out/r5_fold_ab.err
echo "fold ab rc=$?"
