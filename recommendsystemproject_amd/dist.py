"""Data parallelism over RCCL (torch.distributed 'nccl' backend = RCCL on ROCm), one process
per GPU. The batch is sharded: each rank runs the full training step on its own
B samples (own in-batch negatives, own BatchNorm statistics, as DDP applied to the reference),
then ONE all-reduce of the flat gradient buffer (all parameters, ~3.5 MB for the demo schema)
and an identical clip + Adam on every rank. Parameters are broadcast from rank 0 at start.

Large tables trained by lazy-exact Adam (flat.py) stay replicated (a 10M x 128 table with its
Adam state is ~20 GB: it fits 288 GB of HBM many times over) but their gradient is NOT
all-reduced densely (5 GB per table per step): each rank packs only the rows its batch touched,
one all-gather moves [ids | rows] of every rank, and every rank adds the W buffers in rank order
and rebuilds the touched-row list in ascending order, so all ranks hold bitwise-identical
gradients and lists (csrc/sparse.hip rs_sparse_pack / rs_sparse_unpack_add / rs_sparse_compact).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import _hip
from .flat import ensure_flat, flat_of


def is_active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def init_from_env(backend=None):
    """Initialise the default process group from torchrun env vars (no-op for WORLD_SIZE=1)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world <= 1 or (dist.is_available() and dist.is_initialized()):
        return
    if backend is None:
        # RSYS_DIST_BACKEND=gloo: several ranks sharing one GPU (RCCL refuses two ranks on one
        # device) -- rehearses the multi-rank path on a one-GPU box
        backend = os.environ.get('RSYS_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
    if backend == 'nccl':
        torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', '0')))
    dist.init_process_group(backend=backend)


def broadcast_model(model: torch.nn.Module, src: int = 0):
    """Rank-0 parameters and buffers to every rank (flat buffer: one broadcast)."""
    if not is_active():
        return
    f = ensure_flat(model)
    dist.broadcast(f.data, src)
    for b in model.buffers():
        if b.dtype in (torch.float32, torch.int64) and b.numel() > 0:
            dist.broadcast(b, src)


def allreduce_flat_grad(flat_grad: torch.Tensor):
    """Sum the flat gradient over ranks (the mean is folded into the optimizer's grad_scale)."""
    dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)


def allreduce_gradients(model: torch.nn.Module, optimizer=None):
    """After backward: one RCCL all-reduce of the model's flat gradient; the optimizer scales by
    1/world (so clip + Adam see the average gradient, as DDP)."""
    if not is_active():
        return
    params = list(model.parameters())
    f = flat_of(params[0])
    if f is None:
        raise RuntimeError('model is not flattened')
    if f.lazy:
        allreduce_flat_grad(f.grad[:f.dense_numel])
        exchange_lazy_grads(f)
    else:
        allreduce_flat_grad(f.grad)
    from .optim import Adam
    world = dist.get_world_size()
    if isinstance(optimizer, Adam):
        # the flat gradient keeps the SUM; clip (clip_grad_norm_ or the fused clip) and the Adam
        # kernel read it scaled by 1/world, so no extra pass over the gradient is needed
        optimizer.grad_scale = 1.0 / world
        f.grad_scale = 1.0 / world
    else:
        # another optimizer reads p.grad directly: turn the sum into the mean in place
        _hip.call('rs_scale_inplace', f.grad.data_ptr(), f.numel, 1.0 / world, None, _stream())
        f.grad_scale = 1.0


def _stream():
    return torch.cuda.current_stream().cuda_stream


def exchange_lazy_grads(f):
    """Row-sparse gradient exchange of every lazy table of flat buffer f (see module doc)."""
    world = dist.get_world_size()
    dev = f.data.device
    # ids looked up since the last exchange (host count; a replayed hipGraph does not re-run the
    # host side, so the last non-zero count stands in for the replayed forward)
    for t in f.lazy:
        if t.cap > 0:
            t.cap_used, t.cap = t.cap, 0
    caps = torch.tensor([max(1, min(t.cap_used, t.V)) for t in f.lazy], dtype=torch.int64, device=dev)
    dist.all_reduce(caps, op=dist.ReduceOp.MAX)
    caps = caps.tolist()
    nccl = dist.get_backend() == 'nccl'
    for t, cap in zip(f.lazy, caps):
        n = cap * (t.D + 1)
        buf = torch.empty(n, dtype=torch.float32, device=dev)
        _hip.call('rs_sparse_pack', t.ptr(f.grad), t.list.data_ptr(), t.count.data_ptr(), t.D, cap,
                  buf.data_ptr(), None, _stream())
        allbuf = torch.empty(world * n, dtype=torch.float32, device=dev)
        if nccl:
            dist.all_gather_into_tensor(allbuf, buf)
        else:
            dist.all_gather(list(allbuf.split(n)), buf)
        _hip.call('rs_sparse_zero_grad', t.ptr(f.grad), t.list.data_ptr(), t.count.data_ptr(), t.D,
                  _stream())
        for r in range(world):  # fixed summation order: identical rows on every rank
            _hip.call('rs_sparse_unpack_add', t.ptr(f.grad), t.flag.data_ptr(),
                      allbuf.data_ptr() + 4 * r * n, t.D, cap, _stream())
        ws = torch.empty(int(_hip.lib().rs_sparse_compact_ws_bytes(t.V)) // 4 + 1, dtype=torch.int32,
                         device=dev)
        _hip.call('rs_sparse_compact', t.flag.data_ptr(), t.V, t.list.data_ptr(), t.count.data_ptr(),
                  ws.data_ptr(), _stream())
