#!/bin/bash
# round-6 measurements: bench N=1, bench N=2 same-GPU (ccl key), ccl push vs pull, yardsticks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r6m}
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench_n1.json 2> gpurun_out/${T}_bench_n1.err || { tail -5 gpurun_out/${T}_bench_n1.err; exit 1; }
cat gpurun_out/${T}_bench_n1.json | cut -c1-600
timeout -k 10 300 python -u bench.py --gpus 2 --same-gpu --steps 300 --warmup 50 > gpurun_out/${T}_bench_sg2.json 2> gpurun_out/${T}_bench_sg2.err || { tail -5 gpurun_out/${T}_bench_sg2.err; exit 1; }
timeout -k 10 240 python -u tools/ccl_bench.py --same-gpu 2 --forms pull,push > gpurun_out/${T}_ccl_same_gpu2.jsonl 2> gpurun_out/${T}_ccl.err || { tail -5 gpurun_out/${T}_ccl.err; exit 1; }
timeout -k 10 300 python -u tools/conv_vs_blas.py --batch 128 > gpurun_out/${T}_conv_vs_blas.jsonl 2> gpurun_out/${T}_conv_vs_blas.err || { tail -5 gpurun_out/${T}_conv_vs_blas.err; exit 1; }
timeout -k 10 200 python -u tools/bn_pass_bw.py --configs slice:1024 > gpurun_out/${T}_bn_pass_bw.jsonl 2> gpurun_out/${T}_bn_pass_bw.err
rc=$?
tail -1 gpurun_out/${T}_bn_pass_bw.jsonl
exit $rc
