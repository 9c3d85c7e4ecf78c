"""Summarise a rocprofv3 run (kernel stats + optional FETCH_SIZE / WRITE_SIZE PMC passes) into a
text table for profiles/. Usage: python tools/prof_summary.py gpurun_out/prof [STEPS LABELS] >
profiles/<name>.txt (STEPS: the bench's --steps under --prof-markers: per-step tables of the timed
regions follow the whole-run table, whose totals include setup and warm-up)

FETCH_SIZE on gfx950 reads exactly half of a wide coalesced stream's bytes (MI355X_MICROARCH.md
§HBM): the table reports the raw counter (KB) and the corrected HBM read bytes = 2 x FETCH_SIZE.
"""
import csv
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace('rs::(anonymous namespace)::', '').replace('rs::', '')
    return name.split('(')[0][:70]


def pmc(path, ctr):
    f = os.path.join(path, f'pmc_{ctr}', 'run_counter_collection.csv')
    if not os.path.exists(f):
        return {}
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] != ctr:
            continue
        a = acc[short(r['Kernel_Name'])]
        a[0] += float(r['Counter_Value'])
        a[1] += 1
    return {k: v[0] / v[1] for k, v in acc.items()}


def bracketed(path, steps, labels):
    """Per timed region (bench.py --prof-markers: an rs_prof_marker dispatch right before and
    after each workload's timed loop, workloads in `labels` order): every kernel dispatched
    between the two markers, with calls per step and the share of the region's kernel time."""
    f = os.path.join(path, 'trace', 'run_kernel_trace.csv')
    if not os.path.exists(f):
        return
    rows = list(csv.DictReader(open(f)))
    marks = sorted(int(r['Start_Timestamp']) for r in rows if 'prof_marker_kernel' in r['Kernel_Name'])
    pairs = list(zip(marks[0::2], marks[1::2]))
    for i, (t0, t1) in enumerate(pairs):
        acc = defaultdict(lambda: [0.0, 0])
        for r in rows:
            s0 = int(r['Start_Timestamp'])
            if t0 < s0 < t1 and 'prof_marker_kernel' not in r['Kernel_Name']:
                a = acc[short(r['Kernel_Name'])]
                a[0] += int(r['End_Timestamp']) - s0
                a[1] += 1
        tot = sum(v[0] for v in acc.values())
        label = labels[i] if i < len(labels) else f'region {i}'
        print(f'\n# timed region {i} ({label}): {steps} steps, {(t1 - t0) / 1e6:.3f} ms between the markers '
              f'({(t1 - t0) / 1e6 / steps:.4f} ms/step wall); kernel time {tot / 1e6 / steps:.4f} ms/step')
        print(f"{'ms/step':>9} {'calls/step':>10} {'avg_us':>9} {'pct':>5}  kernel")
        for k, (ns, n) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
            print(f"{ns / 1e6 / steps:9.4f} {n / steps:10.2f} {ns / n / 1e3:9.2f} {100 * ns / tot:5.1f}  {k}")


def main(path):
    rows = list(csv.DictReader(open(os.path.join(path, 'trace', 'run_kernel_stats.csv'))))
    fetch, write = pmc(path, 'FETCH_SIZE'), pmc(path, 'WRITE_SIZE')
    print(f'# rocprofv3 --kernel-trace --stats  ({path})')
    print(f'# PMC: FETCH_SIZE / WRITE_SIZE in separate --pmc passes; HBM read = 2 x FETCH_SIZE (gfx950)')
    print(f"{'total_ms':>9} {'calls':>6} {'avg_us':>9} {'pct':>5}  {'fetchKB':>10} {'hbm_rdMB':>9} {'writeKB':>10}  kernel")
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
        k = short(r['Name'])
        fk = fetch.get(k)
        wk = write.get(k)
        print(f"{float(r['TotalDurationNs']) / 1e6:9.3f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['Percentage']):5.1f}  {fk if fk is not None else float('nan'):10.1f} "
              f"{2 * fk / 1024 if fk is not None else float('nan'):9.2f} {wk if wk is not None else float('nan'):10.1f}  {k}")


if __name__ == '__main__':
    # prof_summary.py DIR [STEPS LABEL,LABEL,...]: with STEPS, the whole-run table is followed by
    # the bracketed per-step tables of each timed region
    main(sys.argv[1])
    if len(sys.argv) > 2:
        bracketed(sys.argv[1], int(sys.argv[2]), sys.argv[3].split(',') if len(sys.argv) > 3 else [])
