timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_trainer_gpu.py tests/test_xgmi_gpu.py -x -q > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --eval > gpurun_out/bench.json 2>/dev/null || exit $?; cut -c1-220 gpurun_out/bench.json
rm -rf build/hip_objs && ARENA_TIMELINE=1 timeout 600 python setup.py build_ext --inplace > gpurun_out/tlbuild.log 2>&1 || exit $?
timeout -k 10 300 python scripts/timeline.py > gpurun_out/tl.json 2>/dev/null || exit $?
python -c "
import json; d=json.load(open('gpurun_out/tl.json'))
for k in ('fwd','wgrad'): print(k, d[k]['span_us'], {p: v['med_delta_us'] for p, v in d[k]['phases'].items()})
print('boundary', d['fwd_end_to_wgrad_start_us'], 'step', d['step_span_us'])"
