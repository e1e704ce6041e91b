#!/bin/bash
# SURVEY §7.4 minimum end-to-end slice on a real MI355X: the LocalBackend runs the bundled MNIST
# workloads on the GPU through the CLI, then every read command is exercised.
# Usage: bash tools/e2e_mnist.sh   (outputs under gpurun_out/e2e/)
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/e2e
mkdir -p "$OUT"
export ARENA_HOME=$PWD/$OUT/home PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
A="python -m arena_amd"
cleanup() { $A delete mnist dist hvd prof r50 > /dev/null 2>&1; }
trap cleanup EXIT
trap 'cleanup; exit 143' TERM INT
wait_done() {  # name timeout_s
  local t=0
  while [ $t -lt "$2" ]; do
    s=$($A list | awk -v n="$1" '$1==n {print $2}')
    case "$s" in SUCCEEDED|FAILED) echo "$1 -> $s"; [ "$s" = SUCCEEDED ]; return;; esac
    sleep 2; t=$((t+2))
  done
  echo "$1 timed out"; return 1
}
{
  $A top node -d &&
  $A submit standalonejob --name mnist --gpus 1 \
      "python -m arena_amd.examples.mnist --max_steps 1000 --checkpoint ckpt/mnist.pt" &&
  sleep 5 && $A list && $A top job && $A get mnist && $A top node &&
  wait_done mnist 300 &&
  $A logs mnist --tail 6 && $A get mnist &&
  $A submit tf --name dist --ps 1 --workers 1 --gpus 1 --tensorboard \
      "python -m arena_amd.examples.mnist_ps --max_steps 500" &&
  sleep 3 && $A get dist &&
  wait_done dist 300 &&
  $A logs dist --tail 3 && $A logs dist --tail 2 -i "$($A get dist | awk '/tfjob-ps-0-/ {print $5}')" &&
  $A submit mpi --name hvd --workers 1 --gpus 1 \
      "python -m arena_amd.examples.mnist_hvd --max_steps 500" &&
  wait_done hvd 300 && $A logs hvd --tail 3 &&
  $A submit sj --name prof --gpus 1 --profile-gpu \
      "python -m arena_amd.examples.mnist --max_steps 200" &&
  wait_done prof 300 && $A logs prof --tail 2 &&
  $A submit mpi --name r50 --workers 1 --gpus 1 \
      "python -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128 --num_batches 20 --num_warmup_batches 5" &&
  wait_done r50 300 && $A logs r50 --tail 4 &&
  find "$ARENA_HOME/jobs/prof/traces" -name '*kernel_stats.csv' -exec cp {} "$OUT/prof_job_kernel_stats.csv" \; &&
  head -4 "$OUT/prof_job_kernel_stats.csv" | cut -c1-160 &&
  $A list && $A top job && $A delete mnist dist hvd prof r50 && $A list
} 2>&1 | tee "$OUT/e2e.log"
