"""Flat parameter / gradient buffers.

Every parameter of a model is re-pointed into ONE contiguous fp32 buffer (64-byte aligned
slots, reference parameters() order) and every .grad into a second one. Consequences:
  * the custom ops accumulate weight gradients straight into their slot of the flat gradient
    (no autograd AccumulateGrad adds),
  * zero_grad is one memset, clip_grad_norm_ one reduction, Adam one streaming kernel,
  * data-parallel gradient exchange is one RCCL all-reduce of one buffer,
  * state_dict() is unchanged (parameters keep their names, shapes and Parameter identity).

Large embedding tables (>= RSYS_LAZY_ROWS rows, default 65536) are placed after every other
parameter and trained by lazy-exact Adam (csrc/sparse.hip, trap T16): each one gets a LazyTable
(per-row `last` step, touched-row flag/list/count). The dense kernels then only sweep
[0, dense_numel); the tables are touched row-by-row. State (weights, exp_avg, exp_avg_sq) stays
bitwise what dense Adam would produce; rows are brought current before every read (forward
gather, state_dict, load_state_dict).
"""
from __future__ import annotations

import os

import torch

from . import _hip

ALIGN = 16  # floats (64 B)


def lazy_rows_threshold() -> int:
    return int(os.environ.get('RSYS_LAZY_ROWS', 1 << 16))


class LazyTable:
    """Row bookkeeping of one large [V, D] table trained by lazy-exact Adam."""

    def __init__(self, flat, index, param, offset):
        self.flat, self.index, self.param, self.offset = flat, index, param, offset
        self.V, self.D = int(param.shape[0]), int(param.shape[1])
        dev = param.device
        self.flag = torch.zeros(self.V, dtype=torch.int32, device=dev)
        self.list = torch.zeros(self.V, dtype=torch.int32, device=dev)
        self.count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.last = torch.zeros(self.V, dtype=torch.int32, device=dev)
        self.cap = 0       # ids looked up since the last DP exchange (upper bound of count)
        self.cap_used = 0  # the count the last exchange used

    def ptr(self, t):
        return t.data_ptr() + 4 * self.offset

    def touch(self, ids, rows, bag, row_stride, pad):
        """Forward hook: list this step's rows and bring them to the current optimizer step
        before they are gathered."""
        _hip.call('rs_sparse_touch', ids, rows, bag, row_stride, self.V, pad, self.flag.data_ptr(),
                  self.list.data_ptr(), self.count.data_ptr(), _stream())
        self.cap += rows * bag
        opt = self.flat.lazy_opt
        if opt is not None:
            _hip.call('rs_sparse_catchup', self.ptr(self.flat.data), self.ptr(opt['m']),
                      self.ptr(opt['v']), self.last.data_ptr(), self.list.data_ptr(),
                      self.count.data_ptr(), self.D, opt['step_dev'].data_ptr(),
                      opt['consts'].data_ptr(), *opt['hyper'], _stream())

    def flush(self):
        opt = self.flat.lazy_opt
        if opt is None:
            return
        _hip.call('rs_sparse_flush', self.ptr(self.flat.data), self.ptr(opt['m']), self.ptr(opt['v']),
                  self.last.data_ptr(), self.V, self.D, opt['step_dev'].data_ptr(),
                  opt['consts'].data_ptr(), *opt['hyper'], _stream())

    def zero_grad(self):
        _hip.call('rs_sparse_zero_grad', self.ptr(self.flat.grad), self.list.data_ptr(),
                  self.count.data_ptr(), self.D, _stream())


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _is_lazy(p, lazy_ids):
    return id(p) in lazy_ids


class FlatParams:
    def __init__(self, params, device, lazy=()):
        """params: in module.parameters() order; lazy: the subset (large [V, D] embedding
        weights) trained by lazy-exact Adam, laid out after all other parameters."""
        self.params = list(params)
        lazy_ids = {id(p) for p in lazy}
        self.offsets = [0] * len(self.params)
        off = 0
        for second in (False, True):
            for i, p in enumerate(self.params):
                if _is_lazy(p, lazy_ids) == second:
                    self.offsets[i] = off
                    off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
            if not second:
                self.dense_numel = off
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
        self.lazy = [LazyTable(self, i, p, o) for i, (p, o) in enumerate(zip(self.params, self.offsets))
                     if _is_lazy(p, lazy_ids)]
        for t in self.lazy:
            t.param._rs_lazy = t
        self.lazy_opt = None  # set by optim.Adam: m, v, step_dev, consts, hyper
        # the gradient holds grad_scale^-1 x the mean gradient (data parallel: the all-reduced sum,
        # 1/world; dist.allreduce_gradients): clip_grad_norm_ measures the norm of the mean
        self.grad_scale = 1.0
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
        if not self.lazy:
            self.grad.zero_()
            return
        self.grad[:self.dense_numel].zero_()
        for t in self.lazy:  # only listed rows of a large table can hold a gradient
            t.zero_grad()

    def flush(self):
        """Bring every lazily-updated row to the current optimizer step."""
        for t in self.lazy:
            t.flush()

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
        f = FlatParams(params, params[0].device, lazy_tables(module))
    elif not f.grads_attached():
        f.attach_grads(zero=True)
    return f


def lazy_tables(module: torch.nn.Module):
    """Embedding weights of `module` large enough for lazy-exact Adam; registers hooks that flush
    pending row updates before state_dict() / load_state_dict() touch the weights."""
    thr = lazy_rows_threshold()
    out = []
    # only lookup tables read through the gather (GenericTower.embeddings,
    # SequenceFeatureProcessor.embeddings); pos_emb is read whole by a GEMM epilogue
    tables = [m for owner in module.modules() if isinstance(getattr(owner, 'embeddings', None), torch.nn.ModuleDict)
              for m in owner.embeddings.values()]
    for m in tables:
        if isinstance(m, torch.nn.Embedding) and m.num_embeddings >= thr and thr > 0:
            out.append(m.weight)
            if not getattr(m, '_rs_lazy_hooks', False):
                m.register_state_dict_pre_hook(_flush_hook)
                m._register_load_state_dict_pre_hook(_flush_load_hook, with_module=True)
                m._rs_lazy_hooks = True
    return out


def _flush_table(m):
    t = getattr(m.weight, '_rs_lazy', None)
    if t is not None and flat_of(m.weight) is t.flat and t.param is m.weight:
        t.flush()


def _flush_hook(module, prefix, keep_vars):
    _flush_table(module)


def _flush_load_hook(module, state_dict, prefix, *args):
    _flush_table(module)  # rows become current, so the loaded weights start from `last` = step


def touch_table(weight, ids_ptr, rows, bag, row_stride, pad):
    """Forward-side hook of the custom ops for a table lookup (no-op for small tables)."""
    t = getattr(weight, '_rs_lazy', None)
    if t is not None and rows > 0:
        t.touch(ids_ptr, rows, bag, row_stride, -1 if pad is None else pad)


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
