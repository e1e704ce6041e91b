#!/usr/bin/env python3
"""Where do the framework's (at::native) kernels sit in the step? Reads a rocprofv3 kernel trace
and prints, for each at::native kernel of the LAST step (after the last optimizer kernel but one),
its duration and the kernels around it.

    python tools/kernel_neighbors.py <rocprofv3 output dir> [substring ...]
"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
subs = sys.argv[2:] or ['at::native']
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
opt = [i for i, n in enumerate(names) if 'mt_sgd_master' in n]
lo = opt[-3] if len(opt) >= 3 else 0   # two optimizer launches per step
for i in range(lo + 1, len(names)):
    if any(s in names[i] for s in subs):
        d = (int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3
        print(f'---- {i} {d:.1f} us  {names[i][:120]}')
        for j in range(max(0, i - 2), min(len(names), i + 3)):
            if j != i:
                print('      ', j, names[j][:110])
