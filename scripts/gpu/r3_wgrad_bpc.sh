# Round 3: weight-gradient split candidates (blocks per CU the autotuner's split counts aim at),
# one process per arm, arms interleaved, each twice. JSON lines -> gpurun_out/r3_wgrad_bpc.jsonl
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3_wgrad_bpc.jsonl
: > $out
for rep in 1 2; do
  for bpc in ${ARMS:-1,2,4 0.5,1,2,4 1,2,4,8}; do
    line=$(ARENA_WGRAD_BPC=$bpc timeout -k 10 240 python -m arena_amd.examples.cnn_bench \
      --model resnet50 --batch_size 128 --num_batches 60 --num_warmup_batches 8 --json \
      2> gpurun_out/r3_wgrad_bpc.err | tail -n 1) || { tail -n 20 gpurun_out/r3_wgrad_bpc.err; exit 1; }
    echo "{\"bpc\": \"$bpc\", \"rep\": $rep, \"run\": $line}" | tee -a $out
  done
done
