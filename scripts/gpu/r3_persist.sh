# Round 3: persistent conv tiles. Conv + BN GPU tests, the per-layer autotuned plan (which layers
# take persistent forms), and a same-process ResNet-50 A/B against persistence off.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_conv.py tests/test_bn_gpu.py > gpurun_out/r3_persist_tests.log 2>&1 \
  || { tail -n 60 gpurun_out/r3_persist_tests.log; exit 1; }
tail -n 2 gpurun_out/r3_persist_tests.log
timeout -k 10 300 python scripts/conv_plan_dump.py > gpurun_out/r3_persist_plan.jsonl \
  2> gpurun_out/r3_persist_plan.err || { tail -n 30 gpurun_out/r3_persist_plan.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r3_persist_plan.jsonl"):
    d = json.loads(l)
    if "layer" in d:
        print(d["layer"], d["count"], {k: (d[k]["choice"], d[k]["us"]) for k in ("fwd", "bwd", "wgrad") if d.get(k)})
    else:
        print(d)
PY
timeout -k 10 600 python scripts/cnn_ab.py --modes "${MODES:-auto,auto:nopersist}" \
  --rounds ${ROUNDS:-6} > gpurun_out/r3_persist_ab.jsonl 2> gpurun_out/r3_persist_ab.err \
  || { tail -n 30 gpurun_out/r3_persist_ab.err; exit 1; }
cat gpurun_out/r3_persist_ab.jsonl
