#!/bin/bash
# fence-free end barriers: W = 8 stress, xGMI + bench GPU tests, same-GPU W = 2 collective timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r6e}
timeout -k 10 300 python -u tools/xgmi_stress.py --world 8 --rounds 3 --elems 400000 --timeout-s 10 \
  > gpurun_out/${T}_stress8.jsonl 2> gpurun_out/${T}_stress8.err || { tail -20 gpurun_out/${T}_stress8.err; exit 1; }
grep -c '"ok"' gpurun_out/${T}_stress8.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_xgmi_gpu.py tests/test_bench_gpu.py -m gpu > gpurun_out/${T}_xgmi_tests.log 2>&1 || { tail -30 gpurun_out/${T}_xgmi_tests.log; exit 1; }
tail -2 gpurun_out/${T}_xgmi_tests.log
timeout -k 10 400 python -u tools/ccl_bench.py --same-gpu 2 --forms pull > gpurun_out/${T}_ccl_same_gpu2.jsonl 2> gpurun_out/${T}_ccl.err || { tail -20 gpurun_out/${T}_ccl.err; exit 1; }
grep -v Gloo gpurun_out/${T}_ccl_same_gpu2.jsonl | cut -c1-160
