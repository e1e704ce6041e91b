set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/conv_budget.py > gpurun_out/r6b_conv_budget.md 2> gpurun_out/r6b_budget.err || { tail -5 gpurun_out/r6b_budget.err; exit 1; }
cat gpurun_out/r6b_conv_budget.md
