"""Timeline of one timed step from a rocprofv3 kernel trace (tools/gpu_prof.sh with
--prof-markers): every dispatch between the n-th and (n+1)-th step boundary, with its start /
end relative to the step start, its stream (queue) and the gap since the previous kernel ended on
any queue -- the critical path is where no kernel runs. Usage:
  python tools/step_timeline.py gpurun_out/prof [step index, default 3]"""
import csv
import glob
import os
import re
import sys


def short(name):
    name = name.replace('rs::(anonymous namespace)::', '').replace('void ', '')
    name = re.sub(r'\(.*$', '', name)
    return name[:60]


def main():
    root = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    path = glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'prof_marker' in r['Kernel_Name']]
    if len(marks) < 2:
        sys.exit('no timed-region markers')
    lo, hi = marks[0], marks[1]
    seg = rows[lo + 1:hi]
    # step boundaries: the first kernel of each step is the first dispatch after the previous
    # step's last optimizer kernel -- approximated by equal slices of the timed region by count
    ts0 = int(rows[lo]['End_Timestamp'])
    ts1 = int(rows[hi]['Start_Timestamp'])
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    per = (ts1 - ts0) / nsteps
    a, b = ts0 + k * per, ts0 + (k + 1) * per
    cur = [r for r in seg if a <= int(r['Start_Timestamp']) < b]
    last_end = a
    busy = 0.0
    print(f'step {k}: {per / 1e3:.1f} us window')
    print(f'{"start":>8} {"end":>8} {"dur":>7} {"gap":>6} q  kernel')
    ends = []
    for r in cur:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        gap = max(0, s - max(last_end, a))
        print(f'{(s - a) / 1e3:8.1f} {(e - a) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {gap / 1e3:6.1f} {r["Queue_Id"]:>2} '
              f'{short(r["Kernel_Name"])}')
        last_end = max(last_end, e)
        ends.append((s, e))
    # union of busy intervals
    ends.sort()
    cs, ce = None, None
    for s, e in ends:
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        busy += ce - cs
    print(f'busy (any queue) {busy / 1e3:.1f} us of {per / 1e3:.1f}')


if __name__ == '__main__':
    main()
