# round 5: BN streaming-pass grid cap (every block derives its coefficients from the replicated
# fp64 sums in its prologue) -- in-process A/B of the cap
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/cnn_ab.py --modes auto,auto:ebk2048,auto:ebk1024,auto:ebk512 \
  --rounds 6 > gpurun_out/r5_ebk_ab.jsonl 2> gpurun_out/r5_ebk_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_ebk_ab.jsonl
