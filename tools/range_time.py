"""Timing of rs_gather_bwd on C2's sequence-token tables (hist_movie_ids 3,500 x 32 per token,
hist_genre_ids 30 x 8 mean over 3 tags): the planned path (ranged for the history table) and the
atomic scatter (RSYS_NO_RANGE_GRAD=1). Run under rocprofv3 --kernel-trace for kernel times
(tools/range_trace.py); the event times printed here include the host launch overhead."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402
from recommendsystemproject_amd.functions import _seg  # noqa: E402

dev = torch.device('cuda:0')
B, L, T = 4096, 50, 3
rows = B * L
g = torch.Generator(device='cpu').manual_seed(0)
hist = torch.randint(0, 3500, (rows,), generator=g).to(dev)
genre = torch.randint(0, 19, (rows, T), generator=g).to(dev)
dout = torch.randn(rows, 40, generator=g).to(dev)
gm = torch.zeros(3500, 32, device=dev)
gg = torch.zeros(30, 8, device=dev)
t_m = torch.randn(3500, 32, device=dev)
t_g = torch.randn(30, 8, device=dev)
seg_m = dict(kind=_hip.RS_SEG_SPARSE, dim=32, out_col=0, vocab=3500, idx_stride=1, idx=hist.data_ptr(),
             table=t_m.data_ptr(), grad=gm.data_ptr(), pad_idx=0)
seg_g = dict(kind=_hip.RS_SEG_POOL, dim=8, out_col=32, pool_mode=0, bag=T, vocab=30, idx_stride=T,
             idx=genre.data_ptr(), table=t_g.data_ptr(), grad=gg.data_ptr(), pad_idx=0)


def timeit(segs, n=50):
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


KEYS = ('RSYS_NO_RANGE_GRAD', 'RSYS_DETERMINISTIC')
for segs, label in (([seg_m], 'hist_movie_ids'), ([seg_g], 'hist_genre_ids'), ([seg_m, seg_g], 'both')):
    for name, env in [('default', {}), ('determ', {'RSYS_DETERMINISTIC': '1'}), ('atomic', {'RSYS_NO_RANGE_GRAD': '1'})]:
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        print(f'{label:15s} {name:18s} {timeit(segs):8.1f} us (incl. host launch overhead)', flush=True)
