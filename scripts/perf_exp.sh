#!/bin/bash
# Kernel ablations on the GPU box: instrumented builds with ARENA_EXP bits (see mlp_kernels.hip),
# each followed by scripts/timeline.py. Usage: EXPS="0 1 2 4 8" bash scripts/perf_exp.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in ${EXPS:-0 1 2 4 8}; do
  rm -rf build/hip_objs
  ARENA_TIMELINE=1 ARENA_EXP_FLAGS="-DARENA_EXP=$e" timeout 600 python setup.py build_ext --inplace > gpurun_out/exp_build_$e.log 2>&1 || exit $?
  timeout -k 10 300 python scripts/timeline.py > gpurun_out/timeline_exp$e.json 2> gpurun_out/timeline_exp$e.err || exit $?
  E=$e python - <<'PY'
import json, os
e = os.environ["E"]
d = json.load(open(f"gpurun_out/timeline_exp{e}.json"))
for k in ("fwd", "wgrad"):
    print("exp", e, k, "span", d[k]["span_us"], {p: v["med_delta_us"] for p, v in d[k]["phases"].items()})
print("exp", e, "boundary", d["fwd_end_to_wgrad_start_us"], "step_span", d["step_span_us"])
PY
done
