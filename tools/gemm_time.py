"""Time rs_gemm_f32 on given shapes: python tools/gemm_time.py "TA TB M N K EPI" ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    L = _hip.lib()
    for spec in sys.argv[1:]:
        ta, tb, m, n, k, epi = (int(x) for x in spec.split())
        A = torch.randn(k, m, device=dev) if ta else torch.randn(m, k, device=dev)
        B = torch.randn(n, k, device=dev) if tb else torch.randn(k, n, device=dev)
        C = torch.empty(m, n, device=dev)
        bias = torch.randn(n, device=dev)
        split = int(L.rs_gemm_auto_split(m, n, k))
        ws = torch.empty(max(int(L.rs_gemm_ws_bytes(m, n, k, split)), 16), dtype=torch.uint8, device=dev)

        def f():
            _hip.call('rs_gemm_f32', ta, tb, m, n, k, 1.0, A.data_ptr(), m if ta else k, B.data_ptr(),
                      k if tb else n, 0.0, C.data_ptr(), n, epi, bias.data_ptr(), None, 0, 0, 0.0, None, 0, 0,
                      None, split, ws.data_ptr(), ops.stream())
        for _ in range(2):
            f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(5):
            f()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 5
        ref = (A.t() if ta else A) @ (B.t() if tb else B)
        err = (C - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
        print(f'{spec:28s} split={split:4d} {ms * 1e3:9.1f} us {2.0 * m * n * k / ms / 1e9:7.1f} TF/s relerr {err:.2e}',
              flush=True)


if __name__ == '__main__':
    main()
