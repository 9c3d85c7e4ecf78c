"""Standalone timing of the large-table kernels (csrc/lookup.hip) at the C3 / C5 shapes:
rs_lookup_sort, rs_sorted_catchup (k replayed steps), rs_sorted_adam, rs_sorted_sqnorm, rs_segsum.

    python tools/lazy_bench.py [--V 10000000] [--rows 4096] [--bag 50] [--D 128] [--zipf 1.05]

Prints one JSON line per kernel: avg us per launch over --iters launches (HIP events on the
launch stream) and the algorithmic bytes per launch / GB/s where they are defined.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--V', type=int, default=10_000_000)
    ap.add_argument('--rows', type=int, default=4096)
    ap.add_argument('--bag', type=int, default=50)
    ap.add_argument('--D', type=int, default=128)
    ap.add_argument('--zipf', type=float, default=None)
    ap.add_argument('--pad-frac', type=float, default=0.5)
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    V, D, n = a.V, a.D, a.rows * a.bag
    g = np.random.default_rng(0)
    if a.zipf:
        ids = np.minimum(g.zipf(a.zipf, size=(a.rows, a.bag)) - 1, V - 1)
    else:
        ids = g.integers(1, V, size=(a.rows, a.bag))
    ids[g.random((a.rows, a.bag)) < a.pad_frac] = 0
    ids_t = torch.from_numpy(ids).to(dev)
    S = ops.stream()
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    vals = torch.empty(n, dtype=torch.int32, device=dev)
    wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(n, V))
    ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dev)
    out = []

    def sort():
        _hip.call('rs_lookup_sort', ids_t.data_ptr(), 8, a.rows, a.bag, a.bag, V, keys.data_ptr(),
                  vals.data_ptr(), ws.data_ptr(), S)
    us = timeit(sort, a.iters)
    out.append({'kernel': 'rs_lookup_sort', 'us': round(us, 2), 'n': n})
    uniq = int(torch.unique(ids_t).numel())
    p = torch.randn(V, D, device=dev)
    m = torch.randn(V, D, device=dev) * 1e-3
    v = torch.rand(V, D, device=dev) * 1e-6
    gr = torch.zeros(V, D, device=dev)
    last = torch.zeros(V, 2, dtype=torch.int32, device=dev)  # (moments' step, parameters' step)
    cap = 4096
    consts = torch.zeros(cap, 2, device=dev)
    consts.view(torch.int32)[0, 0] = cap
    step = torch.zeros((), dtype=torch.int64, device=dev)
    for _ in range(100):
        _hip.call('rs_adam_prepare', step.data_ptr(), consts.data_ptr(), cap, 1e-3, 0.9, 0.999, S)
    hyper = (0.9, 0.999, 1e-8, 0.0)
    row_bytes = uniq * D * 4
    for k in (1, 7, 30):
        def catchup():
            last.fill_(100 - k)
            _hip.call('rs_sorted_catchup', keys.data_ptr(), n, D, p.data_ptr(), m.data_ptr(), v.data_ptr(),
                      last.data_ptr(), step.data_ptr(), consts.data_ptr(), *hyper, S)
        fill_us = timeit(lambda: last.fill_(100 - k), a.iters)
        us = timeit(catchup, a.iters) - fill_us
        out.append({'kernel': f'rs_sorted_catchup(k={k})', 'us': round(us, 2), 'rows': uniq,
                    'GB/s': round(6 * row_bytes / (us * 1e-6) / 1e9, 1)})

    def adam():
        last.fill_(99)
        _hip.call('rs_sorted_adam', keys.data_ptr(), n, D, p.data_ptr(), gr.data_ptr(), m.data_ptr(),
                  v.data_ptr(), last.data_ptr(), None, 0, step.data_ptr(), consts.data_ptr(), *hyper, 1.0,
                  None, S)
    fill_us = timeit(lambda: last.fill_(99), a.iters)
    us = timeit(adam, a.iters) - fill_us
    out.append({'kernel': 'rs_sorted_adam', 'us': round(us, 2), 'GB/s': round(8 * row_bytes / (us * 1e-6) / 1e9, 1)})
    ns = int(_hip.lib().rs_sorted_sqnorm_parts())
    wsq = torch.zeros(ns, dtype=torch.float64, device=dev)
    us = timeit(lambda: _hip.call('rs_sorted_sqnorm', keys.data_ptr(), n, D, gr.data_ptr(), None, 0, 1.0,
                                  wsq.data_ptr(), S), a.iters)
    out.append({'kernel': 'rs_sorted_sqnorm', 'us': round(us, 2), 'GB/s': round(row_bytes / (us * 1e-6) / 1e9, 1)})
    dout = torch.randn(a.rows, D, device=dev)
    wss = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(n, D)) // 4 + 1, dtype=torch.int32, device=dev)
    us = timeit(lambda: _hip.call('rs_segsum', keys.data_ptr(), vals.data_ptr(), n, a.bag, 1, 0,
                                  dout.data_ptr(), D, D, gr.data_ptr(), 0, wss.data_ptr(), S), a.iters)
    alg = n * D * 4 + a.rows * D * 4 + n * 4
    out.append({'kernel': 'rs_segsum', 'us': round(us, 2), 'alg_GB/s': round(alg / (us * 1e-6) / 1e9, 1),
                'written_rows_GB/s': round((row_bytes + a.rows * D * 4 + 8 * n) / (us * 1e-6) / 1e9, 1)})
    for o in out:
        o.update({'V': V, 'D': D, 'rows': a.rows, 'bag': a.bag, 'zipf': a.zipf})
        print(json.dumps(o))


if __name__ == '__main__':
    main()
