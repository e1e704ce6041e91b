# Round-3 conv diagnosis: per-layer autotuned conv times (conv_plan_dump) and two PMC passes over
# the conv kernels of a short ResNet-50 run (stall/MFMA split, LDS/L2 behaviour).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ "${SKIP_PRE:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py \
  -k "${TESTK:-split or fwd_bwd_wgrad or fused_bn}" > gpurun_out/r3_conv_tests.log 2>&1 \
  || { tail -n 40 gpurun_out/r3_conv_tests.log; exit 1; }
[ "${SKIP_PRE:-0}" = 1 ] || tail -n 2 gpurun_out/r3_conv_tests.log
[ "${SKIP_PRE:-0}" = 1 ] || timeout -k 10 300 python scripts/conv_plan_dump.py > gpurun_out/r3_conv_plan.jsonl \
  2> gpurun_out/r3_conv_plan.err || { tail -n 30 gpurun_out/r3_conv_plan.err; exit 1; }
[ "${SKIP_PRE:-0}" = 1 ] || tail -n 1 gpurun_out/r3_conv_plan.jsonl
P1=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU,GRBM_GUI_ACTIVE
P2=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_LDS,TCC_HIT_sum,TCC_MISS_sum
for p in 1 2; do
  eval "C=\$P$p"
  rm -rf gpurun_out/r3_pmc$p
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/r3_pmc$p \
    -o pmc --kernel-include-regex 'conv_' -- python3 -m arena_amd.examples.cnn_bench \
    --model resnet50 --batch_size 128 --num_batches 30 --num_warmup_batches 3 --graph 0 \
    > gpurun_out/r3_pmc$p.log 2>&1 || { tail -n 30 gpurun_out/r3_pmc$p.log; exit 1; }
  python scripts/pmc_summary.py gpurun_out/r3_pmc$p --top 40 --last-frac ${LASTFRAC:-0.2} > gpurun_out/r3_pmc${p}_summary.tsv
  rm -rf gpurun_out/r3_pmc$p
  head -n 12 gpurun_out/r3_pmc${p}_summary.tsv | cut -c1-300
done
