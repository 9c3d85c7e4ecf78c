"""Flat parameter / gradient buffers.

Every parameter of a model is re-pointed into ONE contiguous fp32 buffer (64-byte aligned
slots, reference parameters() order) and every .grad into a second one. Consequences:
  * the custom ops accumulate weight gradients straight into their slot of the flat gradient
    (no autograd AccumulateGrad adds),
  * zero_grad is one memset, clip_grad_norm_ one reduction, Adam one streaming kernel,
  * data-parallel gradient exchange is one RCCL all-reduce of one buffer,
  * state_dict() is unchanged (parameters keep their names, shapes and Parameter identity).
"""
from __future__ import annotations

import torch

ALIGN = 16  # floats (64 B)


class FlatParams:
    def __init__(self, params, device):
        self.params = list(params)
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                if p.dtype != torch.float32:
                    raise TypeError(f'only fp32 parameters are supported, got {p.dtype}')
                self.data[o:o + p.numel()].copy_(p.detach().reshape(-1))
        for p, o in zip(self.params, self.offsets):
            p.data = self.data[o:o + p.numel()].view(p.shape)
            p._rs_flat = self
            p._rs_offset = o
        self.attach_grads(zero=False)

    def grad_view(self, i):
        p, o = self.params[i], self.offsets[i]
        return self.grad[o:o + p.numel()].view(p.shape)

    def attach_grads(self, zero=True):
        """(Re)point every p.grad at its flat slot (torch's zero_grad(set_to_none=True) drops
        them). Zeroes the whole flat gradient if any slot had to be re-attached."""
        if zero:
            self.grad.zero_()
        for i, p in enumerate(self.params):
            p.grad = self.grad_view(i)

    def grads_attached(self) -> bool:
        for i, p in enumerate(self.params):
            g = p.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + 4 * self.offsets[i]:
                return False
        return True

    def zero_grad(self):
        self.grad.zero_()

    def __deepcopy__(self, memo):  # copies re-flatten lazily on first use
        return None

    def covers(self, params) -> bool:
        ps = list(params)
        return len(ps) == len(self.params) and all(a is b for a, b in zip(ps, self.params))


def flat_of(p):
    return getattr(p, '_rs_flat', None)


def _valid(f, params) -> bool:
    """All params live in flat buffer f at their recorded slots (module.to()/_apply() or a
    deepcopy re-points .data and breaks this)."""
    base = f.data.data_ptr()
    for p in params:
        if flat_of(p) is not f or p.device != f.data.device or \
                p.data_ptr() != base + 4 * p._rs_offset:
            return False
    return True


def ensure_flat(module: torch.nn.Module) -> FlatParams:
    """Flatten `module`'s parameters on their (HIP) device unless they already share one flat
    buffer (possibly owned by a parent module); re-attach dropped .grad views."""
    params = list(module.parameters())
    if not params:
        raise RuntimeError('module has no parameters')
    f = flat_of(params[0])
    if f is None or not _valid(f, params):
        f = FlatParams(params, params[0].device)
    elif not f.grads_attached():
        f.attach_grads(zero=True)
    return f


def grad_of(p):
    """The flat-gradient slot of parameter p (accumulation target of the custom ops)."""
    f = flat_of(p)
    if f is None:
        raise RuntimeError('parameter is not flattened: call ensure_flat(model) first')
    g = p.grad
    if g is None or g.data_ptr() != f.grad.data_ptr() + 4 * p._rs_offset:
        f.attach_grads(zero=True)
        g = p.grad
    return g
