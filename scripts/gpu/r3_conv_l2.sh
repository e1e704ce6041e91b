# Round 3: L2 -> CU traffic of the conv kernels (substantiates the bytes-per-FLOP limit in
# docs/perf.md): one PMC pass over a short ResNet-50 run, per-kernel summary.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r3_counters.txt 2>&1 || true
grep -o -E "TCP_TCC_READ_REQ_sum|TCC_READ_sum|TCC_HIT_sum|TCC_MISS_sum|TCP_TOTAL_CACHE_ACCESSES_sum|TCC_EA0_RDREQ_sum|SQ_INSTS_VALU_MFMA_MOPS_BF16|SQ_VALU_MFMA_BUSY_CYCLES|GRBM_GUI_ACTIVE" gpurun_out/r3_counters.txt | sort -u
P3=${P3:-TCP_TCC_READ_REQ_sum,TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE,SQ_VALU_MFMA_BUSY_CYCLES}
rm -rf gpurun_out/r3_pmc3
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P3 --output-format csv -d gpurun_out/r3_pmc3 \
  -o pmc --kernel-include-regex 'conv_' -- python3 -m arena_amd.examples.cnn_bench \
  --model resnet50 --batch_size 128 --num_batches 30 --num_warmup_batches 3 --graph 0 \
  > gpurun_out/r3_pmc3.log 2>&1 || { tail -n 30 gpurun_out/r3_pmc3.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/r3_pmc3 --top 25 --last-frac 0.2 > gpurun_out/r3_pmc3_summary.tsv
rm -rf gpurun_out/r3_pmc3
head -n 16 gpurun_out/r3_pmc3_summary.tsv | cut -c1-300
