# round 5: how much the BN-sum epilogues pay for same-address fp64 atomics (acc form vs per-tile
# partials vs no sums), per ResNet-50 layer
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/acc_contention_probe.py > gpurun_out/r5_acc_probe.jsonl \
  2> gpurun_out/r5_acc_probe.err
echo "probe rc=$?"; cat gpurun_out/r5_acc_probe.jsonl
