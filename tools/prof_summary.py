"""Summarise a rocprofv3 run (kernel stats + optional FETCH_SIZE / WRITE_SIZE PMC passes) into a
text table for profiles/. Usage: python tools/prof_summary.py gpurun_out/prof > profiles/<name>.txt

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
    main(sys.argv[1])
