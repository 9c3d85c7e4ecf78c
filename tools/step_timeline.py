"""One training step's kernel timeline from a rocprofv3 --kernel-trace run: the kernels between
the last two launches of a marker kernel (default: the loss tile kernel), with start offset,
duration, gap to the previous kernel's end, stream and grid. Usage:
python tools/step_timeline.py gpurun_out/<dir>/trace [marker] [must_contain]
(must_contain: pick the last step that launches a kernel with this substring, e.g. attn for the
C2 steps of a bench run that also runs C3)"""
import csv
import os
import sys


def short(n):
    n = n.replace('rs::(anonymous namespace)::', '').replace('rs::', '').replace('void ', '')
    return n.split('(')[0][:60]


def main(path, marker='ce_tile_kernel', must=None):
    rows = list(csv.DictReader(open(os.path.join(path, 'run_kernel_trace.csv'))))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    pairs = list(zip(idx[:-1], idx[1:]))
    if must:
        pairs = [(x, y) for x, y in pairs if any(must in r['Kernel_Name'] for r in rows[x:y])]
        # the shortest such span: the last one may run into the next workload's setup
        pairs.sort(key=lambda p: int(rows[p[1]]['Start_Timestamp']) - int(rows[p[0]]['Start_Timestamp']))
        pairs = pairs[:1]
    a, b = pairs[-1]
    t0 = int(rows[a]['Start_Timestamp'])
    end = t0
    busy = {}
    for r in rows[a:b]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        k = short(r['Kernel_Name'])
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - end) / 1e3:6.1f} q{r['Queue_Id']:>2} "
              f"g{int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):>6}  {k}")
        end = max(end, e)
        busy[k] = busy.get(k, 0) + (e - s)
    print(f'step span {(int(rows[b]["Start_Timestamp"]) - t0) / 1e3:.1f} us')
    for k, v in sorted(busy.items(), key=lambda x: -x[1])[:25]:
        print(f'{v / 1e3:8.1f}  {k}')


if __name__ == '__main__':
    main(*sys.argv[1:])
