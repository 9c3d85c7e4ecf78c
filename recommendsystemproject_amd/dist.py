"""Data parallelism over RCCL (torch.distributed 'nccl' backend = RCCL on ROCm), one process
per GPU. The batch is sharded: each rank runs the full training step on its own
B samples (own in-batch negatives, own BatchNorm statistics, as DDP applied to the reference),
then ONE all-reduce of the flat gradient buffer (all parameters, ~3.5 MB for the demo schema)
and an identical clip + Adam on every rank. Parameters are broadcast from rank 0 at start.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .flat import ensure_flat, flat_of


def is_active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def init_from_env(backend=None):
    """Initialise the default process group from torchrun env vars (no-op for WORLD_SIZE=1)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world <= 1 or (dist.is_available() and dist.is_initialized()):
        return
    if backend is None:
        backend = 'nccl' if torch.cuda.is_available() else 'gloo'
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
    allreduce_flat_grad(f.grad)
    if optimizer is not None:
        optimizer.grad_scale = 1.0 / dist.get_world_size()
