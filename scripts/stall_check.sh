set -u
for i in 1 2; do
  for mode in graph eager; do
    if [ $mode = eager ]; then export ARENA_CONV_TIME_EAGER=1; else unset ARENA_CONV_TIME_EAGER; fi
    timeout -k 10 300 python scripts/cnn_ab.py --modes auto,miopen --rounds 3 > gpurun_out/stall_${mode}_$i.jsonl 2> gpurun_out/stall_${mode}_$i.err || exit 1
    echo "$mode $i: $(grep 'round 2' gpurun_out/stall_${mode}_$i.err)"
  done
done
