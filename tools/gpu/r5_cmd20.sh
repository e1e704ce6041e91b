# round 5: effective bandwidth of the BN apply / dx passes per ResNet-50 shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bn_pass_bw.py > gpurun_out/r5_bn_pass_bw.jsonl \
  2> gpurun_out/r5_bn_pass_bw.err
echo "probe rc=$?"; cat gpurun_out/r5_bn_pass_bw.jsonl; tail -3 gpurun_out/r5_bn_pass_bw.err
