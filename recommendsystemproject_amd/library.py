"""The two-tower step as torch custom ops (namespace `rsys`), registered with torch.library.

The reference's modules reach ATen through nn.Embedding, matmul, BatchNorm1d, the Transformer
encoder and F.cross_entropy (GenericTower.py:45-51,182,234; TwoTowerModel.py:95-140;
SequenceEncoder.py:32-56; Tower.py:37-41). Here each module's forward is ONE custom op whose
implementation is the module's HIP kernel sequence (functions.py, through the C-ABI of
librsys_hip.so), with

* register_fake: the output shapes, so FakeTensorMode / meta tracing / torch.compile see through
  the model without running a kernel;
* register_autograd: the backward is another custom op (`<name>_backward`) that runs the
  module's backward kernels.

The ops are visible to the dispatcher as torch.ops.rsys.* (profiler names, torch.compile graph
nodes). Conventions:

* `handle` (int): the module the op belongs to (a registry of weak references): the kernels
  read its configuration (feature schema, dropout p, BatchNorm momentum) and its parameters,
  which are also passed as `params` so autograd records the dependency.
* `flat_grad`: the flat fp32 gradient buffer (flat.py) the parameters' .grad are views of. The
  backward kernels accumulate the weight gradients into it directly (no AccumulateGrad adds), so
  every backward op declares it mutated; the autograd formula returns None for the parameters.
* `stats` / `flags`: buffers a training-mode forward updates in place (BatchNorm running
  statistics and num_batches_tracked, the dropout RNG state, the id-range error flag). They are
  DECLARED mutated (mutates_args): custom_op's ADInplaceOrView kernel bumps their version
  counters and functionalisation (torch.compile's AOT path) sees the writes. None of them ever
  requires grad. torch.library.register_autograd refuses every op whose schema mutates an
  argument, so the backward formula is installed by `_register_autograd` where register_autograd
  puts it for a functional op: the Autograd kernel custom_op generates (torch/_library/
  autograd.py) runs it. The wrappers below refuse a stats buffer that requires grad.
* Large (lazy-Adam) embedding tables: a forward's catch-up replays the zero-gradient Adam steps a
  row skipped before the row is read (flat.py). The value a row logically holds (what dense Adam
  would hold) does not change, so the tables are not declared mutated -- they are parameters,
  which autograd forbids an op to mutate in place; the optimizer and state_dict() read rows only
  after bringing them current the same way (tests/test_gpu_lazy_adam.py, bitwise equal to dense
  Adam).
* `ticket` (a one-element int64 CPU tensor output): the activations a backward needs stay on
  the device in a per-call record (the kernels' saved tensors: per-layer activations, sorted
  lookups of the large tables, BatchNorm statistics); the ticket names it. The backward op takes
  it and releases the record; a forward whose graph is dropped without a backward releases it
  when the ticket is freed. `need` (torch.is_grad_enabled() at the call) says whether to keep one.

There is no CPU implementation: the ops raise HipError off a HIP device (no fallback).
"""
from __future__ import annotations

import itertools
import weakref
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import functions as fn
from .flat import flat_of

# ------------------------------------------------------------------------------ registries
_MODULES = {}
_NEXT_HANDLE = itertools.count(1)
_SAVED = {}
_NEXT_TICKET = itertools.count(1)


def handle_of(module) -> int:
    """The registry handle of `module` (assigned on first use)."""
    h = getattr(module, '_rs_handle', None)
    if h is None or h not in _MODULES or _MODULES[h]() is not module:
        h = next(_NEXT_HANDLE)
        _MODULES[h] = weakref.ref(module)
        module._rs_handle = h
    return h


def module_of(handle: int):
    ref = _MODULES.get(int(handle))
    m = ref() if ref is not None else None
    if m is None:
        raise RuntimeError(f'rsys op: module handle {handle} is not registered (module freed?)')
    return m


class _Ctx:
    """The autograd.Function context the kernel sequences of functions.py write their saved
    state into, kept between the forward and the backward op."""

    def __init__(self, n_inputs):
        self.needs_input_grad = (False,) * n_inputs
        self.saved_tensors = ()

    def save_for_backward(self, *ts):
        self.saved_tensors = ts


def _alias_outputs(v, ids):
    """v with every tensor in `ids` (the op's outputs) replaced by a detached alias."""
    if isinstance(v, Tensor):
        return v.detach() if id(v) in ids else v
    if isinstance(v, list):
        return [_alias_outputs(x, ids) for x in v]
    if isinstance(v, tuple):
        return tuple(_alias_outputs(x, ids) for x in v)
    return v


def _keep(ctx, *outs) -> Tensor:
    """Park `ctx` until the backward (or until the ticket dies). The op's outputs it holds are
    swapped for detached aliases first: the autograd layer attaches the op's node to those very
    tensors, and ctx -> output -> node -> saved ticket -> ctx would be a cycle through C++ that
    Python's collector cannot break (a forward with no backward would keep its graph, and
    through the parameter edges the model, alive)."""
    ids = {id(o) for o in outs if isinstance(o, Tensor)}
    if ids:
        for k, v in list(vars(ctx).items()):
            setattr(ctx, k, _alias_outputs(v, ids))
    t = next(_NEXT_TICKET)
    _SAVED[t] = ctx
    ticket = torch.tensor([t], dtype=torch.int64)
    weakref.finalize(ticket, _SAVED.pop, t, None)
    return ticket


def _no_ticket() -> Tensor:
    return torch.zeros(1, dtype=torch.int64)


def _take(ticket: Tensor):
    t = int(ticket[0])
    ctx = _SAVED.pop(t, None)
    if ctx is None:
        raise RuntimeError('rsys op backward: no saved state for this forward (a second backward '
                           'through the same graph, or a forward run with grad disabled)')
    return ctx


def _raw(f):
    """The undecorated backward (functions.py wraps them in once_differentiable)."""
    return getattr(f, '__wrapped__', f)


def is_fake(t) -> bool:
    """t is a FakeTensor (FakeTensorMode / torch.compile tracing): no kernel may read it."""
    from torch._subclasses.fake_tensor import is_fake as _is_fake
    return isinstance(t, Tensor) and _is_fake(t)


def fake_mode_active() -> bool:
    from torch._guards import detect_fake_mode
    return detect_fake_mode() is not None


def _fake_ticket() -> Tensor:
    return torch.empty(1, dtype=torch.int64)


def _register_autograd(op, backward, setup_context):
    """op.register_autograd(backward, setup_context=...), also for an op that declares mutated
    buffers (see the module doc): custom_op's generated Autograd kernel calls the formula; the
    mutated arguments never require grad (_check_stats), so no gradient flows through them."""
    if op._opoverload._schema.is_mutable:
        op._backward_fn = backward
        op._setup_context_fn = setup_context
    else:
        op.register_autograd(backward, setup_context=setup_context)


def _check_stats(ts):
    for t in ts:
        if t.requires_grad:
            raise RuntimeError('rsys op: a buffer the op updates in place requires grad')
    return ts


# ------------------------------------------------------------------------------ sequence encoder
@torch.library.custom_op('rsys::seq_encoder', mutates_args=('stats',))
def _seq_encoder(seq: List[Tensor], params: List[Tensor], stats: List[Tensor], flat_grad: Tensor, handle: int,
                 keys: str, need: bool) -> Tuple[Tensor, Tensor]:
    """SequenceEncoder.forward (SequenceEncoder.py:32-56) -> ([B, d_model], ticket)."""
    enc = module_of(handle)
    ctx = _Ctx(3 + len(params))
    out = fn.SeqEncoderFn.forward(ctx, need, enc, dict(zip(keys.split(','), seq)), *params)
    return out, (_keep(ctx, out) if need else _no_ticket())


@_seq_encoder.register_fake
def _(seq, params, stats, flat_grad, handle, keys, need):
    enc = module_of(handle)
    return seq[0].new_empty((seq[0].shape[0], enc.feature_embedder.target_dim), dtype=torch.float32), \
        _fake_ticket()


@torch.library.custom_op('rsys::seq_encoder_backward', mutates_args=('flat_grad',))
def _seq_encoder_backward(grad: Tensor, ticket: Tensor, flat_grad: Tensor) -> None:
    ctx = _take(ticket)
    _raw(fn.SeqEncoderFn.backward)(ctx, grad)


@_seq_encoder_backward.register_fake
def _(grad, ticket, flat_grad):
    return None


def _seq_encoder_setup(ctx, inputs, output):
    seq, params, stats, flat_grad = inputs[:4]
    ctx.shape = (len(seq), len(params), len(stats))
    ctx.save_for_backward(output[1])
    ctx.flat_grad = flat_grad  # not a saved tensor: every backward op bumps its version


def _seq_encoder_bwd(ctx, gout, gticket):
    (ticket,) = ctx.saved_tensors
    flat_grad = ctx.flat_grad
    torch.ops.rsys.seq_encoder_backward(gout.contiguous(), ticket, flat_grad)
    ns, npar, nst = ctx.shape
    return [None] * ns, [None] * npar, [None] * nst, None, None, None, None


_register_autograd(_seq_encoder, _seq_encoder_bwd, _seq_encoder_setup)


def seq_encoder(enc, input_dict) -> Tensor:
    """SequenceEncoder.forward through rsys::seq_encoder."""
    params = list(enc.parameters())
    keys = [k for k in input_dict]
    out, _ = _seq_encoder([input_dict[k] for k in keys], params, _check_stats([enc.rng_state, enc.err_flag]),
                          flat_of(params[0]).grad,
                          handle_of(enc), ','.join(keys), torch.is_grad_enabled())
    return out


# ------------------------------------------------------------------------------ sequence features
@torch.library.custom_op('rsys::seq_features', mutates_args=('stats',))
def _seq_features(seq: List[Tensor], params: List[Tensor], stats: List[Tensor], flat_grad: Tensor, handle: int,
                  keys: str, need: bool) -> Tuple[Tensor, Tensor]:
    """SequenceFeatureProcessor.forward (SequenceFeatureProcessor.py:38-85) on its own: per-token
    gather + tag pooling + projection + positional embedding + the two dropouts -> [B, L, d]."""
    proc = module_of(handle)
    ctx = _Ctx(3 + len(params))
    out = fn.SeqFeaturesFn.forward(ctx, need, proc, dict(zip(keys.split(','), seq)), *params)
    return out, (_keep(ctx, out) if need else _no_ticket())


@_seq_features.register_fake
def _(seq, params, stats, flat_grad, handle, keys, need):
    proc = module_of(handle)
    first = seq[0]
    return first.new_empty((first.shape[0], first.shape[1], proc.target_dim), dtype=torch.float32), _fake_ticket()


@torch.library.custom_op('rsys::seq_features_backward', mutates_args=('flat_grad',))
def _seq_features_backward(grad: Tensor, ticket: Tensor, flat_grad: Tensor) -> None:
    ctx = _take(ticket)
    _raw(fn.SeqFeaturesFn.backward)(ctx, grad)


@_seq_features_backward.register_fake
def _(grad, ticket, flat_grad):
    return None


def _seq_features_bwd(ctx, gout, gticket):
    (ticket,) = ctx.saved_tensors
    torch.ops.rsys.seq_features_backward(gout.contiguous(), ticket, ctx.flat_grad)
    ns, npar, nst = ctx.shape
    return [None] * ns, [None] * npar, [None] * nst, None, None, None, None


_register_autograd(_seq_features, _seq_features_bwd, _seq_encoder_setup)


def seq_features(proc, input_dict) -> Tensor:
    """SequenceFeatureProcessor.forward through rsys::seq_features."""
    params = list(proc.parameters())
    keys = [k for k in input_dict]
    out, _ = _seq_features([input_dict[k] for k in keys], params, _check_stats([proc.rng_state, proc.err_flag]),
                           flat_of(params[0]).grad, handle_of(proc), ','.join(keys), torch.is_grad_enabled())
    return out


# ------------------------------------------------------------------------------ tower features
@torch.library.custom_op('rsys::tower_features', mutates_args=('flags',))
def _tower_features(sparse: Optional[Tensor], dense: Optional[Tensor], seq: List[Tensor], seq_vec: Optional[Tensor],
                    params: List[Tensor], flags: List[Tensor], flat_grad: Tensor, handle: int, keys: str,
                    need: bool) -> Tuple[Tensor, Tensor]:
    """GenericTower.forward's feature loop + concat (GenericTower.py:133-233): every sparse /
    pooled / dense feature gathered into [B, total_embed_dim], the sequence vector in the last
    slot; `flags`: the tower's id-range error flag. Large tables: their rows are brought to the
    current optimizer step first (lazy-exact Adam's catch-up: the value a row logically holds
    does not change, so the tables are not declared mutated)."""
    tower = module_of(handle)
    d = {}
    if sparse is not None:
        d['sparse'] = sparse
    if dense is not None:
        d['dense'] = dense
    if keys:
        d['sequence'] = dict(zip(keys.split(','), seq))
    ctx = _Ctx(5 + len(params))
    out = fn.TowerFeatureFn.forward(ctx, need, tower, d, getattr(tower, '_rs_call_mapping', None), seq_vec,
                                    *params)
    return out, (_keep(ctx, out) if need else _no_ticket())


@_tower_features.register_fake
def _(sparse, dense, seq, seq_vec, params, flags, flat_grad, handle, keys, need):
    tower = module_of(handle)
    first = next(t for t in (sparse, dense, *seq, seq_vec) if t is not None)
    return first.new_empty((first.shape[0], tower.total_embed_dim), dtype=torch.float32), _fake_ticket()


@torch.library.custom_op('rsys::tower_features_backward', mutates_args=('flat_grad',))
def _tower_features_backward(grad: Tensor, ticket: Tensor, flat_grad: Tensor, seq_shape: List[int]) -> Tensor:
    """-> the sequence vector's gradient (shape seq_shape; [0] if the tower has none)."""
    ctx = _take(ticket)
    res = _raw(fn.TowerFeatureFn.backward)(ctx, grad)
    return res[4] if res[4] is not None else grad.new_empty(0)


@_tower_features_backward.register_fake
def _(grad, ticket, flat_grad, seq_shape):
    return grad.new_empty(seq_shape)


def _tower_features_setup(ctx, inputs, output):
    sparse, dense, seq, seq_vec, params, flags, flat_grad = inputs[:7]
    ctx.n = (len(seq), len(params), len(flags))
    ctx.seq_shape = None if seq_vec is None else list(seq_vec.shape)
    ctx.save_for_backward(output[1])
    ctx.flat_grad = flat_grad  # not a saved tensor: every backward op bumps its version


def _tower_features_bwd(ctx, gout, gticket):
    (ticket,) = ctx.saved_tensors
    flat_grad = ctx.flat_grad
    dseq = torch.ops.rsys.tower_features_backward(gout.contiguous(), ticket, flat_grad, ctx.seq_shape or [0])
    ns, npar, nfl = ctx.n
    return None, None, [None] * ns, (dseq if ctx.seq_shape is not None else None), [None] * npar, \
        [None] * nfl, None, None, None, None


_register_autograd(_tower_features, _tower_features_bwd, _tower_features_setup)


def tower_features(tower, input_dict, mapping, seq_vec) -> Tensor:
    """TowerFeatureFn through rsys::tower_features."""
    params = list(tower.embeddings.parameters())
    seqd = input_dict.get('sequence') or {}
    keys = [k for k in seqd]
    tower._rs_call_mapping = mapping
    out, _ = _tower_features(input_dict.get('sparse'), input_dict.get('dense'), [seqd[k] for k in keys], seq_vec,
                             params, _check_stats([tower.err_flag]), flat_of(tower.feature_bn.weight).grad,
                             handle_of(tower),
                             ','.join(keys), torch.is_grad_enabled())
    return out


# ------------------------------------------------------------------------------ fused tower chain
def _bn_stats(bns):
    out = []
    for b in bns:
        if b.track_running_stats and b.running_mean is not None:
            out += [b.running_mean, b.running_var, b.num_batches_tracked]
    return out


def _mlp_bns(mlp):
    seq = mlp.mlp
    return [seq[4 * j + 1] for j in range((len(seq) - 1) // 4)]


@torch.library.custom_op('rsys::tower_chain', mutates_args=('stats',))
def _tower_chain(x: Tensor, params: List[Tensor], stats: List[Tensor], flat_grad: Tensor, handle: int, groups: int,
                 need: bool) -> Tuple[Tensor, Tensor]:
    """feature_bn + MLP_Tower in training mode (GenericTower.py:229-236; Tower.py:16-41) as one
    kernel per Linear (csrc/tower.hip); updates the BatchNorm running statistics."""
    tower = module_of(handle)
    ctx = _Ctx(5 + len(params))
    out = fn.TowerChainFn.forward(ctx, need, tower.feature_bn, tower.mlp, x, groups, *params)
    return out, (_keep(ctx, out) if need else _no_ticket())


@_tower_chain.register_fake
def _(x, params, stats, flat_grad, handle, groups, need):
    tower = module_of(handle)
    return x.new_empty((x.shape[0], tower.mlp.mlp[-1].out_features)), _fake_ticket()


@torch.library.custom_op('rsys::tower_chain_backward', mutates_args=('flat_grad',))
def _tower_chain_backward(grad: Tensor, ticket: Tensor, flat_grad: Tensor, x_shape: List[int]) -> Tensor:
    ctx = _take(ticket)
    return _raw(fn.TowerChainFn.backward)(ctx, grad)[3]


@_tower_chain_backward.register_fake
def _(grad, ticket, flat_grad, x_shape):
    return grad.new_empty(x_shape)


def _x_setup(ctx, inputs, output):
    x, params, stats, flat_grad = inputs[:4]
    ctx.n = (len(params), len(stats))
    ctx.x_shape = list(x.shape)
    ctx.save_for_backward(output[1])
    ctx.flat_grad = flat_grad  # not a saved tensor: every backward op bumps its version


def _make_x_bwd(opname):
    def bwd(ctx, gout, gticket):
        (ticket,) = ctx.saved_tensors
        flat_grad = ctx.flat_grad
        dx = getattr(torch.ops.rsys, opname)(gout.contiguous(), ticket, flat_grad, ctx.x_shape)
        npar, nst = ctx.n
        return dx, [None] * npar, [None] * nst, None, None, None, None
    return bwd


_register_autograd(_tower_chain, _make_x_bwd('tower_chain_backward'), _x_setup)


def tower_chain(tower, x, groups) -> Tensor:
    params = list(tower.feature_bn.parameters()) + list(tower.mlp.parameters())
    stats = _check_stats(_bn_stats([tower.feature_bn] + _mlp_bns(tower.mlp)) + [tower.mlp.rng_state])
    out, _ = _tower_chain(x, params, stats, flat_of(params[0]).grad, handle_of(tower), int(groups),
                          torch.is_grad_enabled())
    return out


# ------------------------------------------------------------------------------ BatchNorm1d, MLP_Tower
@torch.library.custom_op('rsys::batch_norm', mutates_args=('stats',))
def _batch_norm(x: Tensor, params: List[Tensor], stats: List[Tensor], flat_grad: Tensor, handle: int, groups: int,
                need: bool) -> Tuple[Tensor, Tensor]:
    """nn.BatchNorm1d (GenericTower.py:234): batch statistics and running-stat update in
    training, running statistics in eval; `groups` independent row blocks."""
    bn = module_of(handle)
    ctx = _Ctx(4 + len(params))
    y = fn.BatchNormFn.forward(ctx, need, bn, x, groups, *params)
    return y, (_keep(ctx, y) if need else _no_ticket())


@_batch_norm.register_fake
def _(x, params, stats, flat_grad, handle, groups, need):
    return x.new_empty(x.shape), _fake_ticket()


@torch.library.custom_op('rsys::batch_norm_backward', mutates_args=('flat_grad',))
def _batch_norm_backward(grad: Tensor, ticket: Tensor, flat_grad: Tensor, x_shape: List[int]) -> Tensor:
    ctx = _take(ticket)
    return _raw(fn.BatchNormFn.backward)(ctx, grad)[2]


@_batch_norm_backward.register_fake
def _(grad, ticket, flat_grad, x_shape):
    return grad.new_empty(x_shape)


_register_autograd(_batch_norm, _make_x_bwd('batch_norm_backward'), _x_setup)


def batch_norm(bn, x, groups) -> Tensor:
    params = [bn.weight, bn.bias]
    y, _ = _batch_norm(x, params, _check_stats(_bn_stats([bn])), flat_of(bn.weight).grad, handle_of(bn), int(groups),
                       torch.is_grad_enabled())
    return y


@torch.library.custom_op('rsys::mlp_tower', mutates_args=('stats',))
def _mlp_tower(x: Tensor, params: List[Tensor], stats: List[Tensor], flat_grad: Tensor, handle: int, groups: int,
               need: bool) -> Tuple[Tensor, Tensor]:
    """MLP_Tower.forward (Tower.py:16-41): [Linear -> BatchNorm1d -> ReLU -> Dropout] x n, Linear,
    F.normalize."""
    mlp = module_of(handle)
    ctx = _Ctx(4 + len(params))
    out = fn.MLPFn.forward(ctx, need, mlp, x, groups, *params)
    return out, (_keep(ctx, out) if need else _no_ticket())


@_mlp_tower.register_fake
def _(x, params, stats, flat_grad, handle, groups, need):
    mlp = module_of(handle)
    return x.new_empty((x.shape[0], mlp.mlp[-1].out_features)), _fake_ticket()


@torch.library.custom_op('rsys::mlp_tower_backward', mutates_args=('flat_grad',))
def _mlp_tower_backward(grad: Tensor, ticket: Tensor, flat_grad: Tensor, x_shape: List[int]) -> Tensor:
    ctx = _take(ticket)
    return _raw(fn.MLPFn.backward)(ctx, grad)[2]


@_mlp_tower_backward.register_fake
def _(grad, ticket, flat_grad, x_shape):
    return grad.new_empty(x_shape)


_register_autograd(_mlp_tower, _make_x_bwd('mlp_tower_backward'), _x_setup)


def mlp_tower(mlp, x, groups) -> Tensor:
    params = list(mlp.parameters())
    out, _ = _mlp_tower(x, params, _check_stats(_bn_stats(_mlp_bns(mlp)) + [mlp.rng_state]), flat_of(params[0]).grad,
                        handle_of(mlp), int(groups), torch.is_grad_enabled())
    return out


# ------------------------------------------------------------------------------ in-batch loss
@torch.library.custom_op('rsys::inbatch_softmax_loss', mutates_args=())
def _inbatch_loss(U: Tensor, I: Tensor, item_ids: Optional[Tensor], H: Optional[Tensor],
                  temperature: float, need: bool) -> Tuple[Tensor, Tensor]:
    """TwoTowerModel.compute_loss (TwoTowerModel.py:81-140): logits U I^T / T, off-diagonal
    equal-id collisions at -1e9, hard-negative logits appended, cross_entropy(arange(B)) mean.
    `need`: a backward follows (the fp32 form then keeps S = U I^T for it)."""
    ctx = _Ctx(5)
    loss = fn.InBatchLossFn.forward(ctx, U, I, item_ids, H, temperature, need)
    return loss, (_keep(ctx, loss) if need else _no_ticket())


@_inbatch_loss.register_fake
def _(U, I, item_ids, H, temperature, need):
    return U.new_empty(()), _fake_ticket()


@torch.library.custom_op('rsys::inbatch_softmax_loss_backward', mutates_args=())
def _inbatch_loss_backward(grad: Tensor, ticket: Tensor, u_shape: List[int], h_shape: List[int],
                           h_stride: List[int]) -> Tuple[Tensor, Tensor, Tensor]:
    """-> dU, dI (U's shape), dH (H's shape and strides; [0] without hard negatives)."""
    ctx = _take(ticket)
    dU, dI, _, dH = _raw(fn.InBatchLossFn.backward)(ctx, grad)[:4]
    return dU, dI, (dH if dH is not None else dU.new_empty(0))


@_inbatch_loss_backward.register_fake
def _(grad, ticket, u_shape, h_shape, h_stride):
    dH = grad.new_empty_strided(h_shape, h_stride) if h_shape != [0] else grad.new_empty(0)
    return grad.new_empty(u_shape), grad.new_empty(u_shape), dH


def _inbatch_setup(ctx, inputs, output):
    U, I, item_ids, H = inputs[:4]
    ctx.u_shape = list(U.shape)
    if H is None:
        ctx.h = ([0], [1])
    else:  # the forward keeps a unit-column-stride H as it is (InBatchLossFn), else a contiguous copy
        Hs = H if H.stride(2) == 1 else H.contiguous()
        ctx.h = (list(H.shape), list(Hs.stride()))
    ctx.has_h = H is not None
    ctx.save_for_backward(output[1])


def _inbatch_bwd(ctx, gloss, gticket):
    (ticket,) = ctx.saved_tensors
    dU, dI, dH = torch.ops.rsys.inbatch_softmax_loss_backward(gloss.contiguous(), ticket, ctx.u_shape, *ctx.h)
    return dU, dI, None, (dH if ctx.has_h else None), None, None


_register_autograd(_inbatch_loss, _inbatch_bwd, _inbatch_setup)


def inbatch_softmax_loss(U, I, item_ids=None, H=None, temperature=0.1) -> Tensor:
    need = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (U, I, H))
    loss, _ = _inbatch_loss(U, I, item_ids, H, float(temperature), need)
    return loss
