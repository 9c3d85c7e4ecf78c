"""GEMM micro-benchmark: the encoder's big-M shapes with and without their fused epilogues.

    python tools/gemm_micro.py            # prints one line per (shape, epilogue)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402

DEV = torch.device('cuda:0')
M = 204800


def bench(fn, it=20):
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
    key = torch.tensor([7, 3], dtype=torch.int64, device=DEV)
    rows = []
    for (ta, tb, m, n, k) in [(0, 1, M, 256, 64), (0, 0, M, 256, 64), (0, 1, M, 64, 256), (0, 0, M, 64, 256),
                              (0, 1, M, 192, 64), (0, 0, M, 64, 192), (0, 1, M, 64, 64)]:
        A = torch.randn(m, k, device=DEV)
        B = torch.randn(n, k, device=DEV) if tb else torch.randn(k, n, device=DEV)
        C = torch.empty(m, n, device=DEV)
        aux = torch.randn(m, n, device=DEV)
        bias = torch.randn(n, device=DEV)
        ldb = k if tb else n
        for name, epi, p in [('plain', 0, 0.0), ('bias', 1, 0.0), ('bias+relu', 3, 0.0),
                             ('mask', 8, 0.0), ('bias+relu+dropA', 1 | 2 | 16, 0.1),
                             ('mask+dropA', 8 | 16, 0.1)]:
            def f():
                _hip.call('rs_gemm_f32', ta, tb, m, n, k, 1.0, A.data_ptr(), k, B.data_ptr(), ldb, 0.0,
                          C.data_ptr(), n, epi, bias.data_ptr(), aux.data_ptr(), n, m, p,
                          key.data_ptr(), 0, 1, None, 1, None, ops.stream())
            ms = bench(f)
            fl = 2.0 * m * n * k
            by = 4.0 * (m * k + m * n * (2 if epi & 8 else 1))
            rows.append(f'{ta}{tb} M={m} N={n} K={k} {name:16s} {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s  '
                        f'{by / ms / 1e6:7.1f} GB/s')
            print(rows[-1], flush=True)
    # the MLP towers / loss at B = 4096 (small M or short K: latency and occupancy bound)
    L = _hip.lib()
    for (ta, tb, m, n, k, epi) in [(1, 0, 128, 256, 4096, 0), (1, 0, 128, 128, 4096, 0), (1, 0, 256, 48, 4096, 0),
                                   (1, 0, 256, 172, 4096, 0), (0, 1, 4096, 128, 256, 1), (0, 1, 4096, 256, 172, 1),
                                   (0, 1, 4096, 128, 128, 1), (0, 0, 4096, 256, 128, 0), (0, 0, 4096, 172, 256, 0),
                                   (0, 1, 4096, 4096, 128, 0), (0, 0, 4096, 128, 4096, 0), (1, 0, 4096, 128, 4096, 0)]:
        A = torch.randn(k, m, device=DEV) if ta else torch.randn(m, k, device=DEV)
        B = torch.randn(n, k, device=DEV) if tb else torch.randn(k, n, device=DEV)
        C = torch.empty(m, n, device=DEV)
        bias = torch.randn(n, device=DEV)
        split = int(L.rs_gemm_auto_split(m, n, k))
        wsb = int(L.rs_gemm_ws_bytes(m, n, k, split))
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=DEV)
        lda = m if ta else k
        ldb = k if tb else n

        def f():
            _hip.call('rs_gemm_f32', ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 0.0,
                      C.data_ptr(), n, epi, bias.data_ptr(), None, 0, 0, 0.0, None, 0, 0, None, split,
                      ws.data_ptr(), ops.stream())
        ms = bench(f)
        print(f'{ta}{tb} M={m} N={n} K={k} epi={epi} split={split} {ms * 1e3:8.1f} us  '
              f'{2.0 * m * n * k / ms / 1e9:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
