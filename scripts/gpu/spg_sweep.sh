set -e
for spg in 1 2 4 5 10 20; do
  for r in 1 2 3; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --resnet 0 --steps-per-graph $spg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($spg, d['value'], d['config']['exec'])" >> gpurun_out/spg_sweep.txt
  done
done
