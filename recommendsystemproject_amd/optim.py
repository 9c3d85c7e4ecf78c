"""Adam and clip_grad_norm_ over the flat parameter buffer (HIP kernels, no host sync).

`Adam` takes the same arguments as torch.optim.Adam (train_twotower.py:111) and keeps a
torch-compatible state_dict (state[p] = {step, exp_avg, exp_avg_sq}); when a param group is
exactly one flat buffer (flat.py) the whole update is one streaming kernel over it.
`clip_grad_norm_` mirrors torch.nn.utils.clip_grad_norm_ (training_utils.py:53-54) with the
total norm and the clip coefficient kept on the device.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _hip, ops
from .flat import flat_of

CONSTS_CAP = 1 << 22  # max optimizer steps with lazy tables (32 MB of per-step constants)


def _flat_cover(params):
    """The FlatParams that `params` is exactly (same objects, same order), else None."""
    if not params:
        return None
    f = flat_of(params[0])
    if f is not None and f.covers(params):
        base = f.data.data_ptr()
        if all(p.data_ptr() == base + 4 * p._rs_offset for p in params):
            return f
    return None


def _row_class(D):
    """rs_sorted_*_batch lanes-per-row class of a table width."""
    return 0 if D <= 16 else 1 if D <= 32 else 2 if D <= 64 else 3 if D <= 128 else 4


def _sorted_batches(items):
    """[(rs_sorted_call_t, extra)] -> launches of at most 8 calls of one row class, in order."""
    out, cur, cls = [], [], None
    for sc, extra in items:
        k = _row_class(sc.D)
        if cur and (k != cls or len(cur) == 8):
            out.append(cur)
            cur = []
        cls = k
        cur.append((sc, extra))
    if cur:
        out.append(cur)
    return out


def _sorted_call(t, c, i, p=None, g=None, m=None, v=None, owner=None):
    sc = _hip.SortedCall()
    sc.keys, sc.n, sc.D, sc.call = c.keys.data_ptr(), c.n, t.D, i
    sc.p = None if p is None else t.ptr(p)
    sc.g = None if g is None else t.ptr(g)
    sc.m = None if m is None else t.ptr(m)
    sc.v = None if v is None else t.ptr(v)
    sc.last = t.last.data_ptr() if p is not None else None
    sc.owner = None if owner is None else owner.data_ptr()
    return sc


class _DeviceClip:
    """sqnorm partials -> (total_norm, coef) device scalars."""

    def __init__(self, device):
        self.norm = torch.zeros((), device=device, dtype=torch.float32)
        self.coef = torch.ones((), device=device, dtype=torch.float32)
        self.ticket = torch.zeros((), device=device, dtype=torch.int32)  # rs_grad_sqnorm_clip_step

    def compute(self, g, n, max_norm, scale=1.0, lazy=(), counter=None, prepare=None):
        """2-norm of g[:n] plus the distinct rows of every lazy table's step calls (their other
        rows hold no gradient), one double partial per block, summed in one fixed order.
        `counter` (a device int64 step count): advanced by the same launch (rs_clip_coef_step);
        `prepare` = (step, consts, cap, lr, b1, b2): the lazy tables' next-step Adam constants
        made by the same launch too (rs_clip_coef_prepare). The dense partials ride in the first
        sorted batch's launch (rs_sorted_sqnorm_batch_dense)."""
        L = _hip.lib()
        nd = int(L.rs_sqnorm_parts(n))
        ns = int(L.rs_sorted_sqnorm_parts())
        work = []
        # row-sharded tables last: their partials are per-rank shards of the norm, summed over
        # the ranks before the coefficient (every rank then holds the same total)
        for t in sorted(lazy, key=lambda t: getattr(t, 'shard', None) is not None):
            owner = t.mark_owners()
            for i, c in enumerate(t.step_calls()):
                work.append((t, c, owner, i))
        ws = torch.empty(nd + ns * len(work) + 2, dtype=torch.float64, device=g.device)
        # every call's partials in one launch per row class (call k's at nd + k * ns); the dense
        # region's in the first of those launches
        items = [(_sorted_call(t, c, i, g=g, owner=owner), k) for k, (t, c, owner, i) in enumerate(work)]
        batches = _sorted_batches(items)
        if not work and prepare is None:
            # no lazy tables: the partials and the coefficient in one launch (same bits)
            _hip.call('rs_grad_sqnorm_clip_step', g.data_ptr(), n, float(scale), ws.data_ptr(),
                      self.ticket.data_ptr(), float(max_norm), self.norm.data_ptr(), self.coef.data_ptr(),
                      counter.data_ptr() if counter is not None else None, ops.stream())
            return
        # the dense partials ride in the first sorted launch only when there is a dense region:
        # that launch adds its dense workgroups for n > 0 only, and rs_grad_sqnorm writes the
        # n = 0 partial (0) that rs_clip_coef* then sums
        fuse_dense = n > 0
        if not batches or not fuse_dense:
            _hip.call('rs_grad_sqnorm', g.data_ptr(), n, float(scale), ws.data_ptr(), ops.stream())
        for j, batch in enumerate(batches):
            arr = (_hip.SortedCall * len(batch))(*[sc for sc, _ in batch])
            if j == 0 and fuse_dense:
                _hip.call('rs_sorted_sqnorm_batch_dense', C.addressof(arr), len(batch), float(scale),
                          ws.data_ptr() + 8 * (nd + batch[0][1] * ns), g.data_ptr(), n, ws.data_ptr(), ops.stream())
            else:
                _hip.call('rs_sorted_sqnorm_batch', C.addressof(arr), len(batch), float(scale),
                          ws.data_ptr() + 8 * (nd + batch[0][1] * ns), ops.stream())
        first = next((k for k, w in enumerate(work) if getattr(w[0], 'shard', None) is not None), None)
        if first is not None:
            torch.distributed.all_reduce(ws[nd + first * ns:nd + len(work) * ns])
        if prepare is not None:
            step, consts, cap, lr, b1, b2 = prepare
            _hip.call('rs_clip_coef_prepare', ws.data_ptr(), nd + ns * len(work), float(max_norm),
                      self.norm.data_ptr(), self.coef.data_ptr(), step.data_ptr(), consts.data_ptr(), int(cap),
                      float(lr), float(b1), float(b2), ops.stream())
        elif counter is not None:
            _hip.call('rs_clip_coef_step', ws.data_ptr(), nd + ns * len(work), float(max_norm),
                      self.norm.data_ptr(), self.coef.data_ptr(), counter.data_ptr(), ops.stream())
        else:
            _hip.call('rs_clip_coef', ws.data_ptr(), nd + ns * len(work), float(max_norm),
                      self.norm.data_ptr(), self.coef.data_ptr(), ops.stream())


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False, foreach=None):
    """torch.nn.utils.clip_grad_norm_ semantics (2-norm): grads scaled in place by
    min(1, max_norm / (total + 1e-6)); returns the total norm as a device scalar."""
    if float(norm_type) != 2.0:
        raise NotImplementedError('only the 2-norm (the reference default) is implemented')
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = list(parameters)  # a generator (model.parameters()) is read twice below
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.tensor(0.0)
    _hip.require_device(params[0])
    f = _flat_cover(parameters)
    clip = _DeviceClip(params[0].device)
    if f is not None:
        # lazy tables: their unlisted gradient rows are zero, so scaling the whole region is
        # correct (one sweep of the table gradient: the fused Adam clip avoids it). Under data
        # parallelism the flat gradient holds the SUM over ranks: the norm is the mean's
        # (f.grad_scale = 1/world), as torch DDP's averaged gradients give
        clip.compute(f.grad, f.dense_numel, max_norm, scale=f.grad_scale, lazy=f.lazy)
        _hip.call('rs_scale_inplace', f.grad.data_ptr(), f.numel, 1.0, clip.coef.data_ptr(), ops.stream())
    else:
        # per-tensor partial sums into one workspace would need a multi-tensor kernel; gather
        # the squares through a temporary flat copy instead (rare path: non-flattened params)
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        clip.compute(flat, flat.numel(), max_norm)
        for p in params:
            _hip.call('rs_scale_inplace', p.grad.data_ptr(), p.grad.numel(), 1.0, clip.coef.data_ptr(),
                      ops.stream())
    if error_if_nonfinite and not torch.isfinite(clip.norm):
        raise RuntimeError(f'The total norm of order {norm_type} for gradients is non-finite')
    return clip.norm


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, *, foreach=None, maximize=False, capturable=False,
                 differentiable=False, fused=None):
        if amsgrad or maximize or differentiable:
            raise NotImplementedError('amsgrad / maximize / differentiable are not supported')
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=foreach, capturable=capturable,
                        differentiable=False, fused=fused)
        super().__init__(params, defaults)
        self.grad_scale = 1.0   # 1/world_size under data parallelism (sum all-reduce)
        self._flat_state = {}   # id(FlatParams) -> dict(m, v, step)
        self._clip = None

    # -------------------------------------------------------------- helpers
    def _group_flat(self, group):
        return _flat_cover(group['params'])

    def _state_for_flat(self, f):
        st = self._flat_state.get(id(f))
        if st is None or st['f'] is not f:
            st = dict(f=f, m=torch.zeros_like(f.data), v=torch.zeros_like(f.data), step=0,
                      step_dev=torch.zeros((), dtype=torch.int64, device=f.data.device))
            if f.lazy:
                # consts[s] = {lr/bc1(s), sqrt(bc2(s))} for every step s, replayed by catch-up
                st['consts'] = torch.zeros(CONSTS_CAP, 2, dtype=torch.float32, device=f.data.device)
                # row 0 (step 0 never runs): {capacity, overflow flag} as int bits; the kernels
                # clamp their step index to it (csrc/sparse.hip adam_prepare_kernel)
                st['consts'].view(torch.int32)[0, 0] = CONSTS_CAP
            self._flat_state[id(f)] = st
            for p, o in zip(f.params, f.offsets):
                self.state[p] = {'step': torch.tensor(0.0),
                                 'exp_avg': st['m'][o:o + p.numel()].view(p.shape),
                                 'exp_avg_sq': st['v'][o:o + p.numel()].view(p.shape)}
        return st

    def zero_grad(self, set_to_none: bool = True):
        """Flat gradients are zeroed in place (one memset per flat buffer) and stay attached."""
        done = set()
        for group in self.param_groups:
            for p in group['params']:
                f = flat_of(p)
                if f is not None:
                    if id(f) not in done:
                        done.add(id(f))
                        if not f.grads_attached():
                            f.attach_grads(zero=False)
                        f.zero_grad()
                elif p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()

    # -------------------------------------------------------------- step
    @torch.no_grad()
    def step(self, closure=None, *, clip_max_norm=None):
        """One Adam step. With clip_max_norm the global grad-norm clip (clip_grad_norm_) is fused:
        the coefficient is computed on the device and applied inside the Adam kernel."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group['betas']
            f = self._group_flat(group)
            if f is not None:
                _hip.require_device(f.data)
                st = self._state_for_flat(f)
                st['step'] += 1
                lr, eps, wd = float(group['lr']), float(group['eps']), float(group['weight_decay'])
                coef = None
                counted = prepared = False
                if f.lazy and st['step'] >= CONSTS_CAP - 1:
                    raise RuntimeError(f'lazy Adam: more than {CONSTS_CAP - 2} steps; raise optim.CONSTS_CAP')
                if clip_max_norm is not None and clip_max_norm > 0:
                    if self._clip is None:
                        self._clip = _DeviceClip(f.data.device)
                    # the device step count (and the lazy tables' step constants) advanced by the
                    # clip coefficient's own launch (no rs_counter_add / rs_adam_prepare launch)
                    counted = not f.lazy
                    prepared = bool(f.lazy)
                    self._clip.compute(f.grad, f.dense_numel, clip_max_norm, self.grad_scale, f.lazy,
                                       counter=st['step_dev'] if counted else None,
                                       prepare=(st['step_dev'], st['consts'], CONSTS_CAP, lr, b1, b2)
                                       if prepared else None)
                    coef = self._clip.coef.data_ptr()
                # device-side step count: the same launch replays correctly inside a hipGraph
                if f.lazy and not prepared:
                    _hip.call('rs_adam_prepare', st['step_dev'].data_ptr(), st['consts'].data_ptr(),
                              CONSTS_CAP, lr, float(b1), float(b2), ops.stream())
                elif not f.lazy and not counted:
                    _hip.call('rs_counter_add', st['step_dev'].data_ptr(), 1, ops.stream())
                dense_args = (f.data.data_ptr(), f.grad.data_ptr(), st['m'].data_ptr(), st['v'].data_ptr(),
                              f.dense_numel)
                dense_done = not f.lazy
                if dense_done:
                    _hip.call('rs_adam_step', *dense_args, lr, float(b1), float(b2), eps, wd, 0,
                              st['step_dev'].data_ptr(), float(self.grad_scale), coef, 0, ops.stream())
                if f.lazy:
                    hyper = (float(b1), float(b2), eps, wd)
                    f.lazy_opt = dict(m=st['m'], v=st['v'], step_dev=st['step_dev'],
                                      consts=st['consts'], hyper=hyper)
                    # every table's calls in one launch per row class (a row is stepped by exactly
                    # one call: the lowest holding it, rs_sorted_owner, when a table has several)
                    items = []
                    for t in f.lazy:
                        owner = t.mark_owners() if coef is None else t.owner
                        calls = t.step_calls()
                        for i, c in enumerate(calls):
                            if c.n == 0:
                                continue
                            items.append((_sorted_call(t, c, i, p=f.data, g=f.grad, m=st['m'], v=st['v'],
                                                       owner=None if len(calls) <= 1 else owner), None))
                    for batch in _sorted_batches(items):
                        arr = (_hip.SortedCall * len(batch))(*[sc for sc, _ in batch])
                        if not dense_done:  # the dense region's Adam in the first batch's launch
                            _hip.call('rs_sorted_adam_batch_dense', C.addressof(arr), len(batch),
                                      st['step_dev'].data_ptr(), st['consts'].data_ptr(), *hyper,
                                      float(self.grad_scale), coef, *dense_args, lr, ops.stream())
                            dense_done = True
                        else:
                            _hip.call('rs_sorted_adam_batch', C.addressof(arr), len(batch), st['step_dev'].data_ptr(),
                                      st['consts'].data_ptr(), *hyper, float(self.grad_scale), coef, ops.stream())
                    if not dense_done:
                        _hip.call('rs_adam_step', *dense_args, lr, float(b1), float(b2), eps, wd, 0,
                                  st['step_dev'].data_ptr(), float(self.grad_scale), coef, 0, ops.stream())
                    for t in f.lazy:
                        t.end_step()
                continue
            if clip_max_norm is not None and clip_max_norm > 0:
                clip_grad_norm_(group['params'], clip_max_norm)
            for p in group['params']:
                if p.grad is None:
                    continue
                _hip.require_device(p)
                state = self.state[p]
                if not state:
                    state['step'] = torch.tensor(0.0)
                    state['exp_avg'] = torch.zeros_like(p)
                    state['exp_avg_sq'] = torch.zeros_like(p)
                state['step'] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                _hip.call('rs_adam_step', p.data_ptr(), g.data_ptr(), state['exp_avg'].data_ptr(),
                          state['exp_avg_sq'].data_ptr(), p.numel(), float(group['lr']), float(b1),
                          float(b2), float(group['eps']), float(group['weight_decay']),
                          int(state['step'].item()), None, float(self.grad_scale), None, 0, ops.stream())
        return loss

    def check_errors(self):
        """Raise if a lazy table ran past its per-step constants (graph replays do not pass through
        the host-side CONSTS_CAP check in step()). One host sync."""
        for st in self._flat_state.values():
            c = st.get('consts')
            if c is not None and int(c.view(torch.int32)[0, 1].item()) != 0:
                raise RuntimeError(f'lazy Adam: more than {CONSTS_CAP - 2} steps; raise optim.CONSTS_CAP')

    def _param_index(self):
        """torch.optim's state_dict numbering: parameters in param-group order."""
        idx, i = {}, 0
        for g in self.param_groups:
            for p in g['params']:
                if id(p) not in idx:
                    idx[id(p)] = i
                    i += 1
        return idx

    def _sharded(self):
        """(param, LazyTable) of every row-sharded lazy table this optimizer steps."""
        out = []
        for st in self._flat_state.values():
            for t in st['f'].lazy:
                if getattr(t, 'shard', None) is not None:
                    out.append((t.param, t))
        return out

    def state_dict(self):
        """torch.optim.Adam's state_dict. Row-sharded tables (flat.py): every rank calls it (a
        collective, as model.state_dict()); exp_avg / exp_avg_sq are the FULL [V, D] moments,
        gathered from the ranks' shards, so the checkpoint has the reference's shapes."""
        for st in self._flat_state.values():
            st['f'].flush()  # lazy tables: exp_avg / exp_avg_sq rows current
            step = float(st['step_dev'].item())  # authoritative (graph replays advance it)
            for p in st['f'].params:
                if p in self.state:
                    self.state[p]['step'] = torch.tensor(step)
        sd = super().state_dict()
        sharded = self._sharded()
        if sharded:
            from .flat import gather_shards
            idx = self._param_index()
            for p, t in sharded:
                s = sd['state'].get(idx[id(p)])
                if s is None:
                    continue
                s = dict(s)
                for k in ('exp_avg', 'exp_avg_sq'):
                    s[k] = gather_shards(s[k], t)
                sd['state'][idx[id(p)]] = s
        return sd

    def load_state_dict(self, state_dict):
        """torch.optim.Adam.load_state_dict, then the loaded exp_avg / exp_avg_sq / step copied
        into the flat buffers the kernels read (the per-parameter state stays views of them).
        Every row of a lazy table is marked current at the loaded step (a checkpoint is written
        flushed), so no earlier step is ever replayed."""
        flats = [self._group_flat(g) for g in self.param_groups]
        for f in flats:  # the flat buffers exist before the loaded per-parameter state lands
            if f is not None:
                self._state_for_flat(f)
        sharded = self._sharded()
        if sharded:  # full [V, D] moments of a row-sharded table: this rank's rows
            idx = self._param_index()
            state_dict = dict(state_dict)
            state_dict['state'] = dict(state_dict['state'])
            for p, t in sharded:
                s = state_dict['state'].get(idx[id(p)])
                if s is None:
                    continue
                s = dict(s)
                W, r = t.shard
                for k in ('exp_avg', 'exp_avg_sq'):
                    if k in s and s[k].shape[0] == t.V_full and t.V_full != t.V:
                        s[k] = s[k][r::W]
                state_dict['state'][idx[id(p)]] = s
        super().load_state_dict(state_dict)
        for f in flats:
            if f is None:
                continue
            st = self._flat_state[id(f)]
            step = 0
            with torch.no_grad():
                for p, o in zip(f.params, f.offsets):
                    s = self.state.get(p)
                    if not s or 'exp_avg' not in s:
                        continue
                    n = p.numel()
                    st['m'][o:o + n].copy_(s['exp_avg'].reshape(-1))
                    st['v'][o:o + n].copy_(s['exp_avg_sq'].reshape(-1))
                    step = max(step, int(float(s['step'])))
                    self.state[p] = {'step': torch.tensor(float(step)),
                                     'exp_avg': st['m'][o:o + n].view(p.shape),
                                     'exp_avg_sq': st['v'][o:o + n].view(p.shape)}
            st['step'] = step
            st['step_dev'].fill_(step)
            for t in f.lazy:
                t.last.fill_(step)
                t.end_step()
