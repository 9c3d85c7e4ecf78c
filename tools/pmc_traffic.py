"""HBM traffic per launch of one entry point from two rocprofv3 --pmc passes of
`bench.py --pmc-bracket auto` (FETCH_SIZE in one pass, WRITE_SIZE in the other: they do not fit
one pass's 4 TCC slots on gfx950).

Attribution: bench.py --pmc-bracket puts an rs_prof_marker dispatch (prof_marker_kernel) before
and after every call of the target entry point; every dispatch between a pair belongs to it.
Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced stream, so HBM read bytes = 2 x FETCH_SIZE (KB x 1024); WRITE_SIZE is exact for
16-B/lane stores and float atomics. Both counters count Infinity-Cache hits as memory traffic.

Usage: python tools/pmc_traffic.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/> <bracket.json>
       > profiles/traffic_<config>_<dtype>.json
"""
import csv
import glob
import json
import os
import sys

MARKER = 'prof_marker_kernel'


def bracketed_sum(path, ctr):
    files = glob.glob(os.path.join(path, f'pmc_{ctr}', '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no counter_collection.csv under {path}/pmc_{ctr}')
    per_dispatch = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            did = int(r['Dispatch_Id'])
            name = r['Kernel_Name']
            d = per_dispatch.setdefault(did, [name, 0.0])
            if r['Counter_Name'] == ctr:
                d[1] += float(r['Counter_Value'])
    inside, total, pairs, kernels = False, 0.0, 0, {}
    for did in sorted(per_dispatch):
        name, val = per_dispatch[did]
        if MARKER in name:
            if inside:
                pairs += 1
            inside = not inside
            continue
        if inside:
            total += val
            k = name.replace('rs::(anonymous namespace)::', '').replace('rs::', '')
            k = k.split('(')[0].replace('void ', '')[:60]
            kernels[k] = kernels.get(k, 0.0) + val
    return total, pairs, kernels


def main(path, bracket_json):
    br = json.loads([ln for ln in open(bracket_json) if ln.startswith('{"pmc_bracket"')][-1])
    fetch_kb, n1, kf = bracketed_sum(path, 'FETCH_SIZE')
    write_kb, n2, kw = bracketed_sum(path, 'WRITE_SIZE')
    if n1 != br['launches'] or n2 != br['launches']:
        raise SystemExit(f'bracket mismatch: {n1}/{n2} marker pairs vs {br["launches"]} launches')
    n = br['launches']
    rd = 2.0 * fetch_kb * 1024 / n
    wr = write_kb * 1024 / n
    out = {
        'entry': br['pmc_bracket'], 'run': br['run'], 'launches': n,
        'hbm_bytes_per_launch': round(rd + wr),
        'hbm_read_bytes_per_launch': round(rd), 'write_bytes_per_launch': round(wr),
        'fetch_size_kb_raw_per_launch': round(fetch_kb / n, 1),
        'alg_bytes_per_launch': round(br['alg_bytes_per_launch']),
        'correction': 'read = 2 x FETCH_SIZE (gfx950 wide-stream halving); write = WRITE_SIZE',
        'kernels_fetch_kb': {k: round(v, 1) for k, v in sorted(kf.items(), key=lambda kv: -kv[1])},
        'kernels_write_kb': {k: round(v, 1) for k, v in sorted(kw.items(), key=lambda kv: -kv[1])},
    }
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
