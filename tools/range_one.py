"""A few rs_gather_bwd calls on C2's hist_movie_ids shape (ranged path) for rocprofv3 --pmc."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip, ops  # noqa: E402
from recommendsystemproject_amd.functions import _seg  # noqa: E402

dev = torch.device('cuda:0')
rows = 4096 * 50
g = torch.Generator(device='cpu').manual_seed(0)
hist = torch.randint(0, 3500, (rows,), generator=g).to(dev)
dout = torch.randn(rows, 40, generator=g).to(dev)
gm = torch.zeros(3500, 32, device=dev)
t_m = torch.randn(3500, 32, device=dev)
seg = dict(kind=_hip.RS_SEG_SPARSE, dim=32, out_col=0, vocab=3500, idx_stride=1, idx=hist.data_ptr(),
           table=t_m.data_ptr(), grad=gm.data_ptr(), pad_idx=0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    ops.gather_bwd([_seg(**seg)], rows, dout)
torch.cuda.synchronize()
print('ok')
