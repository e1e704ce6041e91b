#!/bin/bash
# One perf iteration on the GPU box: GPU tests, kbench, bench, then the instrumented timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_trainer_gpu.py -x -q > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench.txt 2>&1 || exit $?
grep -E "fused|full_step" gpurun_out/kbench.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
rm -rf build/hip_objs && ARENA_TIMELINE=1 timeout 600 python setup.py build_ext --inplace > gpurun_out/tlbuild.log 2>&1 || exit $?
timeout -k 10 300 python scripts/timeline.py > gpurun_out/timeline.json 2> gpurun_out/timeline.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/timeline.json"))
for k in ("fwd", "wgrad"):
    print(k, "span", d[k]["span_us"], {p: v["med_delta_us"] for p, v in d[k]["phases"].items()})
print("boundary", d["fwd_end_to_wgrad_start_us"], "step_span", d["step_span_us"])
PY
