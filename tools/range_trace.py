"""Median per-dispatch durations of the gather-backward kernels in a rocprofv3 kernel trace of
tools/range_time.py, in dispatch order, in groups of 53 (one timing loop of the tool each; a kernel absent from a
variant shifts the grouping: read with the tool's order in mind)."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
names = ('gather_bwd_range_kernel', 'gather_bwd_slot_kernel', 'gather_bwd_small_kernel', 'reduce_partials_kernel',
         'gather_bwd_kernel')
per = {n: [] for n in names}
for r in rows:
    m = re.search('|'.join(names), r['Kernel_Name'])
    if m:
        per[m.group(0)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for n, v in per.items():
    for i in range(0, len(v), 53):
        ch = sorted(v[i:i + 53])
        print(f'{n:26s} group {i // 53}: median {ch[len(ch) // 2]:7.1f} us  min {ch[0]:7.1f} us  ({len(ch)})')
