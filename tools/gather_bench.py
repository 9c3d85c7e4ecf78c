"""Standalone embedding-gather benchmark against the HBM roofline (the >= 70 %
target is reported on a launch of >= 100 MB).

    python tools/gather_bench.py [--vocab 10000000] [--dim 128] [--rows 65536] [--bag 50]

Pooled-mean bags (the C3 history feature) and single-id lookups, forward gather and the
backward table gradient of a large table (rs_lookup_sort + rs_segsum). Algorithmic bytes per
launch:
  fwd: lookups * D * 4 (rows read) + rows * D * 4 (written) + lookups * 8 (int64 ids)
  bwd: lookups * D * 4 (rows scattered) + rows * D * 4 (dout read) + lookups * 4
Prints one JSON line per case.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402
from recommendsystemproject_amd.functions import _seg  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E spec


def timed(fn, it):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--vocab', type=int, default=10_000_000)
    ap.add_argument('--dim', type=int, default=128)
    ap.add_argument('--rows', type=int, default=65536)
    ap.add_argument('--bag', type=int, default=50)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--zipf', type=float, default=None)
    ap.add_argument('--batches', type=int, default=1,
                    help='distinct id sets rotated through the timed loop (8: working set > the 256 MB '
                         'Infinity Cache, as in the training step)')
    ap.add_argument('--fwd-only', action='store_true')
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    V, D, B, L = args.vocab, args.dim, args.rows, args.bag
    g = torch.Generator(device=dev).manual_seed(0)
    table = torch.randn(V, D, device=dev, generator=g)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    copy_gbs = 6290.0  # MI355X_MICROARCH.md: measured float4 copy bandwidth
    for kind, bag in (('pooled_mean', L), ('single_id', 1)):
        ids_all = [torch.randint(1, V, (B, bag), device=dev, generator=g) for _ in range(args.batches)]
        ids = ids_all[0]
        if args.zipf:
            import numpy as np
            z = np.random.default_rng(0).zipf(args.zipf, size=(B, bag)).astype(np.uint64) - np.uint64(1)
            z = ((z * np.uint64(2654435761)) % np.uint64(V - 1)).astype(np.int64) + 1
            ids = torch.from_numpy(z).to(dev)
            ids_all = [ids]
        out = torch.empty(B, D, device=dev)
        segs = []
        for idt in ids_all:
            if bag > 1:
                segs.append(_seg(kind=_hip.RS_SEG_POOL, dim=D, out_col=0, pool_mode=_hip.RS_POOL['mean'], bag=bag,
                                 vocab=V, idx_stride=bag, idx=idt.data_ptr(), table=table.data_ptr(), pad_idx=0))
            else:
                segs.append(_seg(kind=_hip.RS_SEG_SPARSE, dim=D, out_col=0, vocab=V, idx_stride=1,
                                 idx=idt.data_ptr(), table=table.data_ptr(), pad_idx=0))
        it = [0]

        def fwd():
            ops.gather_fwd([segs[it[0] % len(segs)]], B, out, err)
            it[0] += 1
        ms = timed(fwd, args.iters)
        lookups = B * bag
        byts = lookups * D * 4 + B * D * 4 + lookups * 8
        print(json.dumps({'case': f'gather_fwd {kind}', 'vocab': V, 'dim': D, 'rows': B, 'bag': bag,
                          'batches': len(segs),
                          'MB_per_launch': round(byts / 1e6, 1), 'us': round(ms * 1e3, 1),
                          'GBps': round(byts / ms / 1e6, 1), 'frac_of_8TBps': round(byts / ms / 1e6 / PEAK, 3),
                          'frac_of_copy': round(byts / ms / 1e6 / copy_gbs, 3)}))
        if args.fwd_only:
            continue
        # backward: the table gradient of a large (lazy-Adam) table -- the lookups sorted by row
        # (rs_lookup_sort, forward side) and segment-summed (rs_segsum), csrc/lookup.hip
        grad = torch.zeros(V, D, device=dev)
        n = B * bag
        keys = torch.empty(n, dtype=torch.int32, device=dev)
        vals = torch.empty(n, dtype=torch.int32, device=dev)
        wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(n, V))
        wso = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dev)
        sort = lambda: _hip.call('rs_lookup_sort', ids.data_ptr(), 8, B, bag, bag, V, keys.data_ptr(),  # noqa: E731
                                 vals.data_ptr(), wso.data_ptr(), ops.stream())
        ms_sort = timed(sort, args.iters)
        dout = torch.randn(B, D, device=dev)
        wss = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(n, D)) // 4 + 1, dtype=torch.int32, device=dev)
        seg_fn = lambda: _hip.call('rs_segsum', keys.data_ptr(), vals.data_ptr(), n, bag,  # noqa: E731
                                   1 if bag > 1 else 0, 0, dout.data_ptr(), D, D, grad.data_ptr(), 0,
                                   wss.data_ptr(), ops.stream())
        ms = timed(seg_fn, args.iters)
        byts = lookups * D * 4 + B * D * 4 + lookups * 4
        print(json.dumps({'case': f'table_grad {kind} (rs_segsum)', 'MB_per_launch': round(byts / 1e6, 1),
                          'us': round(ms * 1e3, 1), 'GBps': round(byts / ms / 1e6, 1),
                          'frac_of_8TBps': round(byts / ms / 1e6 / PEAK, 3),
                          'frac_of_copy': round(byts / ms / 1e6 / copy_gbs, 3),
                          'sort_us': round(ms_sort * 1e3, 1)}))
        del grad
    assert err.item() == 0


if __name__ == '__main__':
    main()
