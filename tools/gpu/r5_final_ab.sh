# round 5 final check on the final tree: every GPU suite (single- and multi-process), smoke(),
# and the driver-form bench lines (N=1, N=2 same-GPU rehearsal)
set -o pipefail
bash tools/gpu/r5_final_a.sh
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/r5_final_b.sh
