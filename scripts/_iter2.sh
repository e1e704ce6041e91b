for e in 0 16; do
rm -rf build/hip_objs && ARENA_TIMELINE=1 ARENA_EXP_FLAGS="-DARENA_EXP=$e" timeout 600 python setup.py build_ext --inplace > gpurun_out/tlbuild.log 2>&1 || exit $?
timeout -k 10 300 python scripts/timeline.py > gpurun_out/tl$e.json 2>/dev/null || exit $?
E=$e python -c "
import json,os; d=json.load(open('gpurun_out/tl'+os.environ['E']+'.json'))
for k in ('fwd','wgrad'): print(os.environ['E'], k, d[k]['span_us'], {p: v['med_delta_us'] for p, v in d[k]['phases'].items()}, {a: b for a, b in d[k].items() if a.startswith('at_')})
print('boundary', d['fwd_end_to_wgrad_start_us'], 'step', d['step_span_us'])"
done
