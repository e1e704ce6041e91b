timeout -k 10 600 python -m pytest tests/test_trainer_gpu.py -x -q > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
ARENA_FWD_ROWS=rows timeout -k 10 600 python -m pytest tests/test_trainer_gpu.py -x -q > gpurun_out/pt2.log 2>&1; rc=$?; tail -1 gpurun_out/pt2.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for m in counter rows; do ARENA_FWD_ROWS=$m timeout -k 10 300 python bench.py > gpurun_out/b_$m.json 2>/dev/null || exit $?; echo $m $(python -c "import json;print(json.load(open('gpurun_out/b_$m.json'))['ms_per_step'])"); done; done
