# Per-kernel times of chosen conv tile variants on chosen ResNet-50 layers (rocprofv3 kernel
# trace stats; no PMC counters) -> gpurun_out/$1_stats.csv
#   bash tools/gpu/conv_variants_time.sh NAME LAYERS VARIANTS [WGRAD_VARIANTS]
set -o pipefail
NAME=$1; LAYERS=$2; VARIANTS=$3; WG=${4:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/cvt_$NAME
ARGS="--layers $LAYERS --variants $VARIANTS --reps 20 --arms-out gpurun_out/${NAME}_arms.jsonl"
if [ -n "$WG" ]; then ARGS="$ARGS --wgrad $WG"; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cvt_$NAME \
  -o run -- python3 tools/conv_layer_pmc.py $ARGS > gpurun_out/${NAME}.log 2>&1 || { tail -n 20 gpurun_out/${NAME}.log; exit 1; }
STATS=$(find gpurun_out/cvt_$NAME -name '*kernel_stats.csv' | head -1)
TRACE=$(find gpurun_out/cvt_$NAME -name '*kernel_trace.csv' | head -1)
cp "$STATS" gpurun_out/${NAME}_stats.csv
if [ -z "$WG" ]; then python3 tools/arm_times.py "$TRACE" gpurun_out/${NAME}_arms.jsonl > gpurun_out/${NAME}_arms_us.jsonl; fi
rm -rf gpurun_out/cvt_$NAME
python3 - "$NAME" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/{sys.argv[1]}_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us  x{r["Calls"]:>4}  {r["Name"][:110]}')
PY
