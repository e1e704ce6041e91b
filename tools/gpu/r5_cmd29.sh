# round 5: BN knob A/B on the final tree -- non-temporal loads off, reduction grid sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/cnn_ab.py \
  --modes auto,auto:bnnt0,auto:redG1024x8,auto:redG256x8,auto --rounds 8 --chunk 10 \
  > gpurun_out/r5_knob_ab.jsonl 2> gpurun_out/r5_knob_ab.err
echo "ab rc=$?"; cat gpurun_out/r5_knob_ab.jsonl
