"""Run ONE GEMM shape/epilogue a few times (for rocprofv3 --pmc on a single kernel).

    python tools/gemm_one.py TA TB M N K EPI [P] [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402


def main():
    ta, tb, m, n, k, epi = (int(x) for x in sys.argv[1:7])
    p = float(sys.argv[7]) if len(sys.argv) > 7 else 0.0
    iters = int(sys.argv[8]) if len(sys.argv) > 8 else 5
    dev = torch.device('cuda:0')
    A = torch.randn(k, m, device=dev) if ta else torch.randn(m, k, device=dev)
    B = torch.randn(n, k, device=dev) if tb else torch.randn(k, n, device=dev)
    C = torch.empty(m, n, device=dev)
    aux = torch.randn(m, n, device=dev)
    bias = torch.randn(n, device=dev)
    key = torch.tensor([7, 3], dtype=torch.int64, device=dev)
    L = _hip.lib()
    split = int(L.rs_gemm_auto_split(m, n, k))
    ws = torch.empty(max(int(L.rs_gemm_ws_bytes(m, n, k, split)), 16), dtype=torch.uint8, device=dev)
    for _ in range(iters):
        _hip.call('rs_gemm_f32', ta, tb, m, n, k, 1.0, A.data_ptr(), m if ta else k, B.data_ptr(),
                  k if tb else n, 0.0, C.data_ptr(), n, epi, bias.data_ptr(), aux.data_ptr(), n, m, p,
                  key.data_ptr(), 0, 1, None, split, ws.data_ptr(), ops.stream())
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
