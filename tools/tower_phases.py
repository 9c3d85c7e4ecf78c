"""Phase timing of the fused tower kernels (profiling only): runs one C3-shaped user-tower chain
forward + backward with rs_tower_debug_buffer set, one kernel at a time, and prints per-phase
percentiles across workgroups (us since the kernel's first workgroup started).
Phases: 0 start, 1 prologue done, 2 main loop done, 3 C stored, 4 column sums done, 5 hand-off done,
6 C stored, 7 h written (the workgroup's end)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from recommendsystemproject_amd import _hip, precision  # noqa: E402
from test_gpu_tower import _make, _run  # noqa: E402

DEV = torch.device('cuda:0')
precision.set_compute_dtype(os.environ.get('DT', 'bf16'))
C0 = int(os.environ.get('C0', '300'))
m = _make(C0, [256, 128], 128, 0.3)
x = torch.randn(4096, C0, device=DEV)
dout = torch.randn(4096, 128, device=DEV)
for _ in range(3):
    _run(m, x, 1, dout, fused=True)
buf = torch.zeros(4096 * 8, dtype=torch.int64, device=DEV)
L = _hip.lib()
# one launch at a time: hook the ops.call of the tower entry points
from recommendsystemproject_amd import ops  # noqa: E402
orig = ops.call


def call(name, *args):
    if name in ('rs_tower_fwd', 'rs_tower_bwd'):
        buf.zero_()
        L.rs_tower_debug_buffer(buf.data_ptr())
        r = orig(name, *args)
        torch.cuda.synchronize()
        L.rs_tower_debug_buffer(None)
        t = buf.view(-1, 8).cpu().numpy().astype(np.int64)
        t = t[t[:, 0] > 0]
        if not len(t):
            return r
        t0 = t[:, 0].min()
        rel = (t - t0) / 100.0  # 100 MHz -> us
        ph = [f'p{i}:' + '/'.join(f'{np.percentile(rel[:, i][t[:, i] > 0], q):.1f}' for q in (0, 50, 100))
              for i in range(8) if (t[:, i] > 0).any()]
        print(f'{name:14s} wgs={len(t):4d} ' + ' '.join(ph))
        return r
    return orig(name, *args)


ops.call = call
import recommendsystemproject_amd.functions as F  # noqa: E402
F.ops.call = call
_run(m, x, 1, dout, fused=True)
