#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/concurrency_probe.py > gpurun_out/r6c_concurrency.jsonl 2> gpurun_out/r6c_concurrency.err || { tail -20 gpurun_out/r6c_concurrency.err; exit 1; }
cat gpurun_out/r6c_concurrency.jsonl
