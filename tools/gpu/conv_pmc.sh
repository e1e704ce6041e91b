# Per-kernel time and PMC counters of chosen conv variants on chosen layers (tools/conv_layer_pmc.py)
# -> gpurun_out/pmc_<tag>_{trace,p1,p2}.txt. Usage: LAYER=14:256:256:3:1 VARIANTS=0,8,4096 TAG=a \
#    bash tools/gpu/conv_pmc.sh
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LAYER=${LAYER:-14:256:256:3:1}; VARIANTS=${VARIANTS:-0,4096}; WGRAD=${WGRAD:-}; TAG=${TAG:-a}
ARGS="--layers $LAYER --variants $VARIANTS --reps 10"
[ -n "$WGRAD" ] && ARGS="$ARGS --wgrad $WGRAD"
D=gpurun_out/pmc_$TAG
rm -rf $D && mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
  python3 tools/conv_layer_pmc.py $ARGS > $D/trace.log 2>&1 || { tail -n 20 $D/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv \
  -d $D/p1 -o run -- python3 tools/conv_layer_pmc.py $ARGS > $D/p1.log 2>&1 || { tail -n 20 $D/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum \
  GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d $D/p2 -o run -- python3 tools/conv_layer_pmc.py $ARGS > $D/p2.log 2>&1 || { tail -n 20 $D/p2.log; exit 1; }
python3 tools/pmc_summary.py $D/trace --top 20 > gpurun_out/pmc_${TAG}_trace.txt
python3 tools/pmc_summary.py $D/p1 --top 20 > gpurun_out/pmc_${TAG}_p1.txt
python3 tools/pmc_summary.py $D/p2 --top 20 > gpurun_out/pmc_${TAG}_p2.txt
rm -rf $D
cat gpurun_out/pmc_${TAG}_trace.txt gpurun_out/pmc_${TAG}_p1.txt gpurun_out/pmc_${TAG}_p2.txt
