"""rs_gather_bwd on the C2 / C3 towers' ordinary tables at B = 4096 (single ids, the genre bag of 3)
and C2's per-token sequence tables, per plan variant: default (atomic small-table kernel, ranged
for hot 48 KB - 4 MB tables), RSYS_DETERMINISTIC=1 (slot-image / ranged kernels for every table),
RSYS_NO_RANGE_GRAD=1 (atomic scatter for the mid tables too). Event time per call (host launch overhead included); run
under rocprofv3 --kernel-trace --stats for the kernels. RSYS_NO_ONEHOT_GRAD=1 (round 5): the tiny tables back on the atomic / slot kernels.

    python tools/gather_bwd_time.py
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
    t = torch.randn(V, D, device=dev)
    gr = torch.zeros(V, D, device=dev)
    keep.extend([ids, t, gr])
    s = dict(kind=_hip.RS_SEG_SPARSE if bag is None else _hip.RS_SEG_POOL, dim=D, out_col=col, vocab=V,
             idx_stride=1 if bag is None else bag, idx=ids.data_ptr(), table=t.data_ptr(), grad=gr.data_ptr(),
             pad_idx=0)
    if bag is not None:
        s.update(pool_mode=_hip.RS_POOL['mean'], bag=bag)
    return s


B = 4096
cases = {}
small_user = [(3, 4), (10, 8), (25, 8), (700, 16)]
col = 0
segs = []
for V, D in [(6060, 64)] + small_user:
    segs.append(seg(V, D, B, col)); col += D
cases['c2_user'] = (segs, B, col)
segs, col = [], 0
for V, D, bag in [(3500, 32, None), (30, 8, 3), (152, 8, None)]:
    segs.append(seg(V, D, B, col, bag)); col += D
cases['c2_item'] = (segs, B, col)
segs, col = [], 0
for V, D in small_user:
    segs.append(seg(V, D, B, col)); col += D
cases['c3_user_small'] = (segs, B, col)
segs, col = [], 0
for V, D, bag in [(30, 8, 3), (152, 8, None)]:
    segs.append(seg(V, D, B, col, bag)); col += D
cases['c3_item_small'] = (segs, B, col)
rows = B * 50
cases['c2_tokens'] = ([seg(3500, 32, rows, 0), seg(30, 8, rows, 32, 3)], rows, 40)


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


KEYS = ('RSYS_NO_RANGE_GRAD', 'RSYS_DETERMINISTIC', 'RSYS_NO_ONEHOT_GRAD')
for label, (segs, rows, ld) in cases.items():
    for name, env in [('default', {}), ('determ', {'RSYS_DETERMINISTIC': '1'}),
                      ('atomic', {'RSYS_NO_RANGE_GRAD': '1'}), ('no_onehot', {'RSYS_NO_ONEHOT_GRAD': '1'})]:
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        print(f'{label:15s} {name:10s} {timeit(segs, rows, ld):8.1f} us', flush=True)
