#!/bin/bash
# One GPU session: numerics tests, smoke, short bench, eager baseline, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/abort/timeout stops the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp

ok_or_stop() {  # rc 0 = pass, 1 = test failures (GPU healthy) -> continue; anything else -> stop
  local rc=$1 what=$2
  echo "[gpu_check] $what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "[gpu_check] stopping after $what (rc=$rc)"; exit "$rc"
  fi
}

STEPS=${STEPS:-all}

if [[ $STEPS == all || $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  ok_or_stop $? "pytest -m gpu"
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1
  ok_or_stop $? "smoke"
  tail -2 gpurun_out/smoke.log
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py --eval > gpurun_out/bench.json 2> gpurun_out/bench.err
  ok_or_stop $? "bench fused"
  cat gpurun_out/bench.json
fi
if [[ $STEPS == all || $STEPS == *eager* ]]; then
  timeout -k 10 600 python bench.py --impl torch --steps 1000 --warmup 100 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err
  ok_or_stop $? "bench torch"
  cat gpurun_out/bench_torch.json
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 600 --warmup 60 > gpurun_out/prof.log 2>&1
  ok_or_stop $? "rocprofv3"
  find gpurun_out/prof -name '*kernel_stats.csv' -exec head -20 {} \;
fi
if [[ $STEPS == all || $STEPS == *e2e* ]]; then
  timeout -k 10 900 bash scripts/e2e_mnist.sh > gpurun_out/e2e_driver.log 2>&1
  ok_or_stop $? "e2e local backend"
  tail -30 gpurun_out/e2e/e2e.log
fi
echo "[gpu_check] done"
