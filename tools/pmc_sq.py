"""Per-kernel SQ counter summary of rocprofv3 --pmc passes over a bench run (profiling tool).

    python tools/pmc_sq.py <dir with pmc_*/ subdirectories> [kernel substrings ...]

Sums every counter per kernel name over its dispatches and prints, per kernel: dispatches, the
per-dispatch averages, and the derived shares of the wave cycles (SQ_WAIT_ANY: parked on
s_waitcnt / barrier; SQ_WAIT_INST_ANY: issue stalls; SQ_ACTIVE_INST_ANY: issuing), VALU
instructions per wave and MFMA busy share (MI355X_MICROARCH.md: the three WAIT/ACTIVE buckets sum
to SQ_WAVE_CYCLES; SQ_* cycle counters count quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES)."""
import csv
import glob
import json
import os
import sys


def main(path, subs):
    per = {}
    for f in glob.glob(os.path.join(path, 'pmc_*', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].replace('rs::(anonymous namespace)::', '').replace('rs::', '')
            k = k.split('(')[0].replace('void ', '')[:70]
            d = per.setdefault(k, {'_dispatch': set()})
            d['_dispatch'].add((f, r['Dispatch_Id']))
            d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    rows = []
    for k, d in per.items():
        if subs and not any(s in k for s in subs):
            continue
        n = len({x[1] for x in d.pop('_dispatch')})
        out = {'kernel': k, 'dispatches_per_pass': n}
        wc = d.get('SQ_WAVE_CYCLES')
        if wc:
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU'):
                if c in d:
                    out[c.replace('SQ_', '').lower() + '_share'] = round(d[c] / wc, 3)
        if d.get('SQ_WAVES'):
            for c in ('SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR',
                      'SQ_INSTS_SALU'):
                if c in d:
                    out[c.replace('SQ_INSTS_', '').lower() + '_per_wave'] = round(d[c] / d['SQ_WAVES'], 1)
        if d.get('SQ_BUSY_CYCLES') and d.get('SQ_VALU_MFMA_BUSY_CYCLES'):
            out['mfma_busy_over_busy'] = round(d['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * d['SQ_BUSY_CYCLES']), 4)
        out['avg'] = {c: round(v / max(n, 1)) for c, v in sorted(d.items())}
        rows.append(out)
    rows.sort(key=lambda o: -o['avg'].get('SQ_WAVE_CYCLES', 0))
    for o in rows:
        print(json.dumps(o))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])
