timeout -k 10 600 python -m pytest tests/test_trainer_gpu.py tests/test_xgmi_gpu.py -x -q > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for m in dataset published; do ARENA_WGRAD_X=$m timeout -k 10 300 python bench.py --eval > gpurun_out/bench_$m.json 2>/dev/null || exit $?; echo $m; cat gpurun_out/bench_$m.json | cut -c1-200; done
rm -rf build/hip_objs && ARENA_TIMELINE=1 timeout 600 python setup.py build_ext --inplace > gpurun_out/tlbuild.log 2>&1 || exit $?
for m in dataset published; do ARENA_WGRAD_X=$m timeout -k 10 300 python scripts/timeline.py > gpurun_out/tl_$m.json 2>/dev/null || exit $?; M=$m python -c "
import json,os; m=os.environ['M']; d=json.load(open(f'gpurun_out/tl_{m}.json'))
print(m, 'wgrad', d['wgrad']['span_us'], {p: v['med_delta_us'] for p, v in d['wgrad']['phases'].items()}, 'step', d['step_span_us'])"; done
