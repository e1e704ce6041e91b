set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -rf gpurun_out/nb
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/nb -o r50 -- python3 -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 --num_batches 4 --num_warmup_batches 4 > gpurun_out/nb.log 2>&1 || { tail -5 gpurun_out/nb.log; exit 1; }
python3 tools/kernel_neighbors.py gpurun_out/nb > gpurun_out/nb.txt; cat gpurun_out/nb.txt
rm -rf gpurun_out/nb
