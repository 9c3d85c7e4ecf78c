"""rs_gather_bwd of C2's per-token genre bags (204,800 rows x 3 ids into a 30 x 8 table) and the towers'
tiny tables at B = 4096, timed with events over 50 calls, per RSYS_OH_RPW (rows per wave of the
one-hot kernel) and against RSYS_NO_ONEHOT_GRAD=1. Run under rocprofv3 --kernel-trace --stats.

    python tools/oh_time.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402
from recommendsystemproject_amd.functions import _seg  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator(device='cpu').manual_seed(0)
keep = []


def seg(V, D, rows, col, bag=None):
    ids = torch.randint(0, V, (rows,) if bag is None else (rows, bag), generator=g).to(dev)
    gr = torch.zeros(V, D, device=dev)
    keep.extend([ids, gr])
    s = dict(kind=_hip.RS_SEG_SPARSE if bag is None else _hip.RS_SEG_POOL, dim=D, out_col=col, vocab=V,
             idx_stride=1 if bag is None else bag, idx=ids.data_ptr(), grad=gr.data_ptr(), pad_idx=0)
    if bag is not None:
        s.update(pool_mode=_hip.RS_POOL['mean'], bag=bag)
    return s


def timeit(segs, rows, ld, n=50):
    dout = torch.randn(rows, (ld + 3) // 4 * 4, device=dev)
    for _ in range(3):
        ops.gather_bwd([_seg(**s) for s in segs], rows, dout)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        ops.gather_bwd([_seg(**s) for s in segs], rows, dout)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


cases = {'genre_tokens': ([seg(30, 8, 204800, 32, 3)], 204800, 40),
         'user_tiny': ([seg(3, 4, 4096, 0), seg(10, 8, 4096, 4), seg(25, 8, 4096, 12)], 4096, 20),
         'item_tiny': ([seg(30, 8, 4096, 0, 3), seg(152, 8, 4096, 8)], 4096, 16)}
for label, (segs, rows, ld) in cases.items():
    for name, env in [('atomic', {'RSYS_NO_ONEHOT_GRAD': '1'}), ('oh', {}), ('oh_rpw32', {'RSYS_OH_RPW': '32'}),
                      ('oh_rpw64', {'RSYS_OH_RPW': '64'}), ('oh_rpw128', {'RSYS_OH_RPW': '128'})]:
        for k in ('RSYS_NO_ONEHOT_GRAD', 'RSYS_OH_RPW'):
            os.environ.pop(k, None)
        os.environ.update(env)
        print(f'{label:15s} {name:10s} {timeit(segs, rows, ld):8.1f} us', flush=True)
