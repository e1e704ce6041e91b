# Round 3: the MNIST headline at the driver's short run (20 timed steps): fixed launch/sync latency
# under HIP runtime wait/launch settings, interleaved repeats, one process per arm.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3_mnist_latency.jsonl
: > $out
for rep in 1 2; do
  for arm in default wait2000 devkarg both; do
    case $arm in
      default) envs="" ;;
      wait2000) envs="ROC_ACTIVE_WAIT_TIMEOUT=2000" ;;
      devkarg) envs="HIP_FORCE_DEV_KERNARG=1" ;;
      both) envs="ROC_ACTIVE_WAIT_TIMEOUT=2000 HIP_FORCE_DEV_KERNARG=1" ;;
    esac
    line=$(env $envs timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 5 --resnet 0 \
      2> gpurun_out/r3_mnist_latency.err) || { tail -n 20 gpurun_out/r3_mnist_latency.err; exit 1; }
    echo "{\"arm\": \"$arm\", \"rep\": $rep, \"bench\": $line}" | tee -a $out
  done
done
