"""Autograd functions of the two-tower training step, one per reference module.

Each function runs its whole module (forward and backward) as a sequence of librsys_hip kernels;
autograd only connects the modules (SequenceEncoder -> tower features -> feature_bn -> MLP ->
loss), so the graph has a handful of nodes per tower instead of hundreds of ATen ops. Weight
gradients are accumulated by the kernels directly into the flat gradient buffer (flat.py); the
functions return None for parameters (they are inputs only so autograd records the dependency).

Dropout uses counter-based masks (csrc/rng.h): each forward draws a fresh (seed, counter) key
on the device (graph-replay safe) and the backward re-derives the same masks from it. Sites:
  sequence input: 0 projection dropout, 1 dropout after + pos_emb      (T5)
  encoder layer i: 16+8i attention probs, +1 dropout1, +2 FFN inner, +3 dropout2
  MLP hidden layer j: 256+j
With p = 0 (the parity setting) nothing is hashed.

`need` (first argument of every forward) is torch.is_grad_enabled() at the call site: inside
Function.forward grad mode is always off, so the modules decide whether to keep activations.
"""
from __future__ import annotations

import ctypes as C
import os

import torch
from torch.autograd.function import once_differentiable

from . import _hip, ops, precision
from . import dist as _dp
from .flat import SEG_MEAN, SEG_ONE, SEG_SUM, _dp_active, catchup_batch, flat_of, grad_of, lookup_table


def _seg(**kw):
    s = _hip.FeatureSeg()
    s.pad_idx = -1
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def _pad(v):
    return -1 if v is None else int(v)


def _agreed(x, tokens=False):
    """Data parallel: (rows, bag, ragged) over the ranks of the lookup call reading batch tensor x,
    from this forward's one shape agreement (dist.agree_batch), or None. tokens: a [B, L] / [B, L, T]
    sequence feature read as one call of B * L rows."""
    h = _dp.agreed_dims(x)
    if h is None:
        return None
    dims, ragged = h
    if tokens:
        return dims[0] * dims[1], (dims[2] if len(dims) == 3 else 1), ragged
    return dims[0], (dims[1] if len(dims) >= 2 else 1), ragged


def _read_through():
    """RSYS_READ_THROUGH=1: recorded lookups of lazy tables read their rows through the catch-up
    inside the gather (rs_gather_fwd_lazy) instead of a catch-up pass that writes them back first.
    Off by default: the replay is VALU work (~14 operations per element and skipped step), and
    read-through does it twice (gather, then the optimizer step) where the pass does it once --
    measured at C3 (rows 7 steps stale): gather 0.194 ms + Adam 0.160 against catch-up 0.154 +
    gather 0.036 + Adam 0.095. It pays off only when the rows are mostly current."""
    return os.environ.get('RSYS_READ_THROUGH', '0') == '1'


def _lookup_lazy(segs, tables, rows, keep=None, record=True, err=None):
    """Large (lazy-Adam) tables, flat.py: bring this call's rows to the current optimizer step
    before the gather reads them -- or, recorded lookups, have the gather read them through the
    catch-up (segment lazy_last) -- and (`record`: a backward follows) sort its ids by row
    (csrc/lookup.hip). Returns ({segment index: LookupCall}, the gather's lazy launch arguments or
    None); ordinary tables are not listed.
    `keep` (the id tensors the segments point into) stays referenced by the calls until the
    optimizer step (the data-parallel exchange re-reads the ids after the backward).
    A row-sharded table (flat.py module doc) is looked up here: its segment is replaced by one
    reading this rank's rows as the exchange returned them (the all-to-all's row buckets, or
    the reduce-scatter's pooled bags), kept alive through `keep`.
    Every table's sort runs first, then one batched catch-up of all the calls (round 6; before,
    the second and later tables' sort + catch-up chains were forked onto side streams, which inside
    the replayed hipGraph still ran on the forking stream's queue)."""
    calls = {}
    lazy = None
    groups = {}  # table -> segment indices, first-seen order
    for i, (s, t) in enumerate(zip(segs, tables)):
        if s.kind in (_hip.RS_SEG_SPARSE, _hip.RS_SEG_POOL) and hasattr(t, '_rs_lazy'):
            lt = t._rs_lazy
            if getattr(lt, 'shard', None) is not None and flat_of(t) is lt.flat:
                c, newseg, held = lt.shard_lookup(s, rows, record, None if err is None else err.data_ptr())
                keep.extend(held)
                segs[i] = newseg
                if c is not None:
                    calls[i] = c
                continue
            groups.setdefault(id(t), []).append(i)

    def one(i):
        nonlocal lazy
        s, t = segs[i], tables[i]
        lt = t._rs_lazy
        pool = s.kind == _hip.RS_SEG_POOL
        bag = s.bag if pool else 1
        mode = SEG_ONE
        if pool:
            mode = {_hip.RS_POOL['mean']: SEG_MEAN, _hip.RS_POOL['sum']: SEG_SUM}.get(s.pool_mode)
        args = lt.read_through_args() if record and mode is not None and _read_through() else None
        c = lookup_table(t, s.idx, rows, bag, s.idx_stride, None if s.pad_idx < 0 else s.pad_idx,
                         -1 if mode is None else mode, keep=keep, record=record, read_through=args is not None,
                         agreed=getattr(s, 'agreed', None), defer_catchup=True)
        if c is not None:
            calls[i] = c
            if pool and mode is not None and args is None and getattr(c, 'a2a', None) is None and not _dp_active():
                # the gather stages this call's hot rows (runs of equal sorted keys) into LDS; only
                # for a single-process call, whose sorted keys are the table's global row ids (a
                # data-parallel exchange's keys can be slot indices)
                s.hot_keys, s.hot_n = c.keys.data_ptr(), c.n
        if args is not None and flat_of(t) is lt.flat:
            if lazy is not None and lazy != args:
                raise RuntimeError('lazy tables of one gather must share one flat buffer and optimizer')
            lazy = args
            s.lazy_last = lt.last.data_ptr()
        return c

    # every table's sort on the current stream, then the catch-ups of all of them in one launch
    # (rs_sorted_catchup_batch; a table's later calls in later launches). Round 6: C3 fp32
    # 0.722 -> 0.711 ms per step against a sort + catch-up chain per table (the second and later
    # tables forked onto side streams, which inside the replayed graph ran on the same queue)
    order = sorted(groups.values(), key=lambda idxs: -sum(int(segs[i].vocab) for i in idxs))
    done = []
    for idxs in order:
        for i in idxs:
            c = one(i)
            if c is not None and c.catchup_due:
                done.append((tables[i]._rs_lazy, c))
    catchup_batch(done)
    return calls, lazy


def _grad_tables(segs, calls, dout, tables, rows, params=()):
    """Backward of a gather: the ordinary segments (ordinary tables, dense, copies, and max-pooled
    large tables, whose arg-max gradient keeps the atomic scatter) through rs_gather_bwd first;
    then -- the op's dense gradients all queued, its data-parallel bucket may start its
    all-reduce (dist.GradBuckets) -- the large-table segments: rs_segsum per call (deterministic,
    no atomics)."""
    from .flat import _dp_active
    rest, big = [], []
    dp = _dp_active()
    for i, s in enumerate(segs):
        c = calls.get(i) if calls else None
        ptr = dout.data_ptr() + 4 * s.out_col
        sharded = c is not None and getattr(tables[i]._rs_lazy, 'shard', None) is not None
        if c is not None and dp and c.mode < 0:
            # max pooling under data parallelism: the arg-max scatter's contributions as per-lookup
            # gradient rows (rs_pool_max_grad), exchanged like rows x bag single-id lookups
            # (GenericTower.py:159-160; max-pooled tables are never row-sharded, flat.lazy_tables)
            big.append((tables[i]._rs_lazy, _max_as_single(c, s, dout), None))
            continue
        # under data parallelism a call only keeps its output gradient rows here (rs_pack_rows,
        # any alignment / row stride); the exchange segment-sums every rank's
        if sharded or (c is not None and c.mode >= 0 and (dp or (ptr % 16 == 0 and dout.stride(0) % 4 == 0))):
            big.append((tables[i]._rs_lazy, c, ptr))
        else:
            rest.append(s)
    if rest:
        rest = _sorted_ordinary(rest, rows, dout)
    if rest:
        ops.gather_bwd(rest, rows, dout)
    _dp.note_writer(params, written=True)
    # calls of different tables of one row width share one launch pair (rs_segsum_batch, up to 4
    # a launch); a table's calls keep their order (each its own launch after the first)
    pending = []

    def flush():
        if pending:
            arr = (_hip.SegsumCall * len(pending))(*[sc for _, sc, _ in pending])
            _hip.call('rs_segsum_batch', C.addressof(arr), len(pending), pending[0][0].D, ops.stream())
            pending.clear()

    for t, c, ptr in big:
        if ptr is None:  # max-pooled: its per-lookup gradient rows are already the call's dseg
            continue
        args = t.segsum_call(c, ptr, dout.stride(0))
        if args is None:
            flush()
            t.segsum(c, ptr, dout.stride(0))
            continue
        if len(pending) == 4 or any(pt is t for pt, _, _ in pending) or (pending and pending[0][0].D != t.D):
            flush()
        pending.append((t, args[0], args[1]))
    flush()


_SORTED_ORDINARY_BYTES = 4 << 20


def _sorted_ordinary(segs, rows, dout):
    """Deterministic mode (torch.use_deterministic_algorithms / RSYS_DETERMINISTIC): the gradient
    of an ORDINARY (dense-Adam) table above 4 MB -- too large for the LDS-image kernels, so the
    default is the float-atomic scatter -- through the large tables' sorted path instead: sort the
    call's ids by row (rs_lookup_sort), then the segment sum (rs_segsum, accumulate), each row's
    contributions added in lookup order with plain stores. The same two kernels and inputs as a
    lazy table's call, so a model trained with RSYS_LAZY_ROWS=0 (dense Adam over every row) gets
    bitwise the lazy path's table gradients. Returns the segments left to rs_gather_bwd."""
    ops.sync_deterministic()
    if not ops.deterministic_enabled() or not dout.is_cuda:
        return segs
    rest = []
    for sg in segs:
        pooled = sg.kind == _hip.RS_SEG_POOL
        mode = SEG_ONE if sg.kind == _hip.RS_SEG_SPARSE else \
            {_hip.RS_POOL['mean']: SEG_MEAN, _hip.RS_POOL['sum']: SEG_SUM}.get(sg.pool_mode) if pooled else None
        ptr = dout.data_ptr() + 4 * sg.out_col
        if (mode is None or not sg.grad or int(sg.vocab) * sg.dim * 4 <= _SORTED_ORDINARY_BYTES or
                sg.dim % 4 or sg.dim > 256 or ptr % 16 or dout.stride(0) % 4):
            rest.append(sg)
            continue
        bag = sg.bag if pooled else 1
        n = rows * bag
        if n == 0:
            continue
        L = _hip.lib()
        keys = torch.empty(n, dtype=torch.int32, device=dout.device)
        vals = torch.empty(n, dtype=torch.int32, device=dout.device)
        wsb = int(L.rs_lookup_sort_ws_bytes(n, int(sg.vocab)))
        sws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dout.device) if wsb else None
        _hip.call('rs_lookup_sort', sg.idx, 8, rows, bag, sg.idx_stride, int(sg.vocab), keys.data_ptr(),
                  vals.data_ptr(), None if sws is None else sws.data_ptr(), ops.stream())
        ws = torch.empty(int(L.rs_segsum_ws_bytes(n, sg.dim)) // 4 + 1, dtype=torch.int32, device=dout.device)
        _hip.call('rs_segsum', keys.data_ptr(), vals.data_ptr(), n, bag, mode, sg.pad_idx, ptr,
                  dout.stride(0), sg.dim, sg.grad, 1, ws.data_ptr(), ops.stream())
    return rest


def _max_as_single(c, s, dout):
    """A max-pooled large-table call under data parallelism, turned into rows x bag single-id
    lookups whose gradient rows (kept for the exchange, c.dseg) are the arg-max scatter's
    contributions: dout[r] at each column's first arg-max position of bag r, zeros elsewhere. The
    call's sorted values (r * bag + l) already index those rows."""
    if s.idx_stride != s.bag:
        raise RuntimeError('max-pooled large table: the id matrix must be contiguous')
    n = c.rows * c.bag
    g = torch.empty(n, s.dim, device=dout.device, dtype=torch.float32)
    _hip.call('rs_pool_max_grad', s.table, s.idx, 8, c.rows, c.bag, s.idx_stride, s.vocab, s.dim, s.pad_idx,
              dout.data_ptr() + 4 * s.out_col, dout.stride(0), g.data_ptr(), ops.stream())
    if c.agreed is not None:
        rmax, bmax, ragged = c.agreed
        c.agreed = (rmax * bmax, 1, ragged)
    c.rows, c.bag, c.row_stride, c.mode = n, 1, 1, SEG_ONE
    c.local_rows = n
    c.dseg = g
    return c


# ================================================================================ sequence input
def seq_feature_segments(proc, seqd, B, L):
    """Per-token gather plan of SequenceFeatureProcessor.forward (SequenceFeatureProcessor.py:57-76):
    2-D [B, L] features give one id per token, 3-D [B, L, T] tag lists are pooled by mean/sum (T4),
    widths concatenated in config order. Returns (segments, tables, width, kept id tensors)."""
    segs, tables, keep, col = [], [], [], 0
    for f in proc.feature_config_list:
        name = f['name']
        if name not in seqd:
            print(f'Configuration Error: Unable to find {name} in the input dictionary, {name} has skipped')
            continue
        x = seqd[name]
        agreed = _agreed(x, tokens=True)
        x = (x if x.dtype == torch.int64 else x.long()).contiguous()
        keep.append(x)
        emb = proc.embeddings[name]
        D = emb.embedding_dim
        pad = _pad(emb.padding_idx)
        if x.dim() == 2:
            if tuple(x.shape) != (B, L):
                raise RuntimeError(f'sequence feature {name}: shape {tuple(x.shape)}, expected {(B, L)}')
            segs.append(_seg(kind=_hip.RS_SEG_SPARSE, dim=D, out_col=col, vocab=emb.num_embeddings,
                             idx_stride=1, idx=x.data_ptr(), table=emb.weight.data_ptr(), pad_idx=pad))
        elif x.dim() == 3:
            mode = f.get('pooling', None)
            if mode not in ('mean', 'sum'):
                raise RuntimeError(f'Tensors must have same number of dimensions: 3-D sequence feature '
                                   f"{name} needs pooling 'mean' or 'sum' (got {mode!r})")
            T = int(x.shape[2])
            segs.append(_seg(kind=_hip.RS_SEG_POOL, dim=D, out_col=col, pool_mode=_hip.RS_POOL[mode],
                             bag=T, vocab=emb.num_embeddings, idx_stride=T, idx=x.data_ptr(),
                             table=emb.weight.data_ptr(), pad_idx=pad))
        else:
            raise RuntimeError(f'sequence feature {name}: unsupported rank {x.dim()}')
        segs[-1].agreed = agreed
        tables.append(emb.weight)
        col += D
    if not segs:
        raise ValueError('Configuration Error: No valid features were processed!')
    for t in keep:  # the kernels read these through raw pointers
        _hip.require_device(t)
    return segs, tables, col, keep


def seq_input_fwd(proc, seqd, B, L, p, key, err, need=True):
    """gather -> Linear(sum dims -> d) -> Dropout -> + pos_emb -> F.dropout (T5). Returns x [B*L, d]."""
    segs, tables, dcat, keep = seq_feature_segments(proc, seqd, B, L)
    if dcat != proc.feature_projection[0].in_features:
        raise RuntimeError(f'mat1 and mat2 shapes cannot be multiplied ({B * L}x{dcat} and '
                           f'{proc.feature_projection[0].in_features}x{proc.target_dim})')
    M = B * L
    dev = proc.pos_emb.weight.device
    cat = torch.empty(M, dcat, device=dev, dtype=torch.float32)
    calls, lazy = _lookup_lazy(segs, tables, M, keep, record=need, err=err)
    ops.gather_fwd(segs, M, cat, err, lazy=lazy)
    lin = proc.feature_projection[0]
    pos = proc.pos_emb.weight
    # drop_b(drop_a(cat W^T + b) + pos[l]) in the GEMM epilogue (sites 0, 1 = rs_dropout masks)
    x = ops.linear_fwd(cat, lin.weight, lin.bias, aux=pos, aux_mod=L, drop_p=p, drop_key=key,
                       site_a=0, site_b=1)
    return x, (segs, tables, cat, keep, calls)


def seq_input_bwd(proc, saved, dx, B, L, p, key, params=()):
    """Backward of seq_input_fwd; dx [B*L, d] is consumed (modified in place). `params`: the
    calling op's parameters (its data-parallel bucket, dist.GradBuckets)."""
    segs, tables, cat, _, calls = saved
    d = proc.target_dim
    pos_g = grad_of(proc.pos_emb.weight)
    if p > 0 and (L * d) % 4 == 0 and L * d <= 4096:
        # drop_b backward, d pos_emb[l] = sum_b dx[b, l], drop_a backward: one pass
        ops.seq_input_dropout_bwd(dx, pos_g, B, L * d, p, key, 0, 1)
    else:
        if p > 0:
            ops.dropout_bwd(dx, p, key, 1)
        ops.colsum(dx, pos_g, M=B, N=L * d, ldx=L * d)  # d pos_emb[l] = sum_b dx[b, l]
        if p > 0:
            ops.dropout_bwd(dx, p, key, 0)
    lin = proc.feature_projection[0]
    # dx is final here (the dropout backward above ran in place before this point)
    ops.linear_bwd_weight(dx, cat, grad_of(lin.weight), db=grad_of(lin.bias))
    dcat = ops.linear_bwd_input(dx, lin.weight)
    for s, t in zip(segs, tables):
        s.grad = grad_of(t).data_ptr()
    _grad_tables(segs, calls, dcat, tables, B * L, params)


class SeqFeaturesFn(torch.autograd.Function):
    """SequenceFeatureProcessor.forward on its own (SequenceFeatureProcessor.py:38-85): the
    per-token gather, tag pooling, projection, positional embedding and dropouts of
    seq_input_fwd -> [B, L, d]."""

    @staticmethod
    def forward(ctx, need, proc, seqd, *params):
        first = next(v for v in seqd.values())
        B, L = int(first.shape[0]), int(first.shape[1])
        if L > proc.pos_emb.num_embeddings:
            raise IndexError('index out of range in self')
        p = proc.dropout if proc.training else 0.0
        key = ops.rng_next(proc.rng_state) if p > 0 else None
        x, saved = seq_input_fwd(proc, seqd, B, L, p, key, proc.err_flag, need)
        if need:
            ctx.proc, ctx.saved, ctx.B, ctx.L, ctx.p, ctx.key = proc, saved, B, L, p, key
            ctx.params = params
            _dp.note_writer(params)
        return x.view(B, L, proc.target_dim)

    @staticmethod
    @once_differentiable
    def backward(ctx, dx):
        dx = dx.contiguous().view(ctx.B * ctx.L, -1).clone()  # consumed in place below
        seq_input_bwd(ctx.proc, ctx.saved, dx, ctx.B, ctx.L, ctx.p, ctx.key, ctx.params)
        ctx.saved = ctx.params = None
        return (None, None, None) + (None,) * (len(ctx.needs_input_grad) - 3)


# ================================================================================ encoder layer
def _is_fake(t):
    from torch._subclasses.fake_tensor import FakeTensor
    return isinstance(t, FakeTensor)


def _ffn_fwd(lyr, x1, p, key, site):
    """x2 = norm2(x1 + dropout2(linear2(dropout(relu(linear1(x1)))))) on any row count."""
    if ops.ffn_supported(x1, lyr.linear1.weight):
        # bf16 mode: the whole feed-forward block in one kernel; f1 stays on chip (csrc/ffn.hip)
        h2, x2, m2, r2, fmask = ops.ffn_fwd_bf16(x1, lyr.linear1.weight, lyr.linear1.bias,
                                                 lyr.linear2.weight, lyr.linear2.bias, lyr.norm2.weight,
                                                 lyr.norm2.bias, lyr.norm2.eps, p, key, site + 2, site + 3)
        return x2, (('ffn', fmask), h2, m2, r2)
    f1 = ops.linear_fwd(x1, lyr.linear1.weight, lyr.linear1.bias, relu=True, drop_p=p, drop_key=key,
                        site_a=site + 2)  # dropout(relu(.)) fused
    h2, x2, m2, r2 = ops.linear_add_layernorm(f1, lyr.linear2.weight, lyr.linear2.bias, x1,
                                              lyr.norm2.weight, lyr.norm2.bias, lyr.norm2.eps, p, key,
                                              site + 3)  # h2 = x1 + dropout2(ff), x2 = norm2(h2)
    return x2, (f1, h2, m2, r2)


def layer_fwd(lyr, x, key_pad, B, L, d, H, p, key, site):
    """nn.TransformerEncoderLayer (norm_first=False, relu) forward on x [B*L, d]."""
    sa_mod = lyr.self_attn
    # bf16 mode: qkv stored as bf16 (only ever an MFMA operand: same products, half the bytes)
    qkv = ops.linear_fwd(x, sa_mod.in_proj_weight, sa_mod.in_proj_bias,
                         out_dtype=torch.bfloat16 if ops.qkv_bf16_ok(L, d, H, B * L) else torch.float32)
    att, lse = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, site)
    # h1 = x + dropout1(out_proj(att)), x1 = norm1(h1): GEMM + residual + LayerNorm in one kernel
    h1, x1, m1, r1 = ops.linear_add_layernorm(att, sa_mod.out_proj.weight, sa_mod.out_proj.bias, x,
                                              lyr.norm1.weight, lyr.norm1.bias, lyr.norm1.eps, p, key,
                                              site + 1)
    x2, ff = _ffn_fwd(lyr, x1, p, key, site)
    return x2, (x, qkv, att, lse, h1, x1, m1, r1) + ff


def prune_last_layer() -> bool:
    """The final encoder layer runs its post-attention half on the B selected rows only (T7):
    SequenceEncoder returns context[b, last[b]] (SequenceEncoder.py:58-74), so every other row of
    that layer is dead: same loss, same gradients. RSYS_FULL_LAST_LAYER=1 computes all rows."""
    return not os.environ.get('RSYS_FULL_LAST_LAYER')


def layer_fwd_last(lyr, x, key_pad, last, B, L, d, H, p, key, site):
    """The final encoder layer for the selected rows last[b] only -> x2 [B, d] (= the encoder
    output): qkv for all rows (every key / value is live), attention of the B selected queries,
    then out-proj + LN1 + FFN + LN2 on B rows."""
    sa_mod = lyr.self_attn
    qkv = ops.linear_fwd(x, sa_mod.in_proj_weight, sa_mod.in_proj_bias,
                         out_dtype=torch.bfloat16 if ops.qkv_bf16_ok(L, d, H, B * L) else torch.float32)
    att, lse = ops.attn_rows_fwd(qkv, key_pad, last, B, L, d, H, p, key, site)
    # the residual rows x[b, last[b]] read in place by the fused kernel (bf16 mode), else gathered
    post = ops.linear_add_layernorm_rows(att, sa_mod.out_proj.weight, sa_mod.out_proj.bias, x, last, L,
                                         lyr.norm1.weight, lyr.norm1.bias, lyr.norm1.eps, p, key, site + 1)
    if post is None:
        xs = torch.empty(B, d, device=x.device, dtype=torch.float32)
        ops.gather_fwd([_seg(kind=_hip.RS_SEG_LASTVALID, dim=d, out_col=0, bag=L, idx=last.data_ptr(),
                             table=x.data_ptr())], B, xs)
        post = ops.linear_add_layernorm(att, sa_mod.out_proj.weight, sa_mod.out_proj.bias, xs,
                                        lyr.norm1.weight, lyr.norm1.bias, lyr.norm1.eps, p, key, site + 1)
    h1, x1, m1, r1 = post
    x2, ff = _ffn_fwd(lyr, x1, p, key, site)
    return x2, (x, qkv, att, lse, h1, x1, m1, r1) + ff


def _post_attn_bwd(lyr, saved, dx2, p, key, site):
    """Backward of out-proj + LN1 + FFN + LN2 (any row count). Returns (dh1, datt): dh1 the
    gradient of the layer input through the residual, datt the gradient of the attention output."""
    x, qkv, att, lse, h1, x1, m1, r1, f1, h2, m2, r2 = saved
    g = grad_of
    sa_mod = lyr.self_attn
    # x2 = LN2(x1 + drop2(ff))
    ln1_done = False
    if isinstance(f1, tuple):
        # bf16 mode, fused feed-forward block: norm2 backward + FFN backward + norm1 backward in one
        # pass (csrc/ffn.hip): dh2 and dx1 stay on chip; dff = drop2(dh2) is written for the fused
        # weight gradients, which recompute f1 / dPre1 on chip
        dh1, dsa, dff = ops.ffn_bwd_ln2_bf16(
            x1, lyr.linear1.weight, lyr.linear1.bias, lyr.linear2.weight, f1[1], dx2, h2, lyr.norm2.weight,
            m2, r2, g(lyr.norm2.weight), g(lyr.norm2.bias), h1, lyr.norm1.weight, m1, r1,
            g(lyr.norm1.weight), g(lyr.norm1.bias), p, key, site + 1, site + 3)
        ln1_done = True
        ops.ffn_wgrad_bf16(x1, lyr.linear1.weight, lyr.linear1.bias, lyr.linear2.weight, f1[1], dff, p,
                           g(lyr.linear1.weight), g(lyr.linear1.bias), g(lyr.linear2.weight),
                           g(lyr.linear2.bias))
    else:
        dff = torch.empty_like(dx2) if p > 0 else None
        dh2 = ops.layernorm_bwd(h2, dx2, lyr.norm2.weight, m2, r2, g(lyr.norm2.weight), g(lyr.norm2.bias),
                                da=dff, p=p, key=key, site=site + 3)
        dff = dh2 if dff is None else dff
        ops.linear_bwd_weight(dff, f1, g(lyr.linear2.weight), db=g(lyr.linear2.bias))
        # f1 holds relu(.) after dropout: (f1 > 0) == kept & positive, kept scale 1/(1-p)
        df1 = ops.linear_bwd_input(dff, lyr.linear2.weight, relu_mask_of=f1,
                                   alpha=(1.0 / (1.0 - p)) if p > 0 else 1.0)
        ops.linear_bwd_weight(df1, x1, g(lyr.linear1.weight), db=g(lyr.linear1.bias))
        ops.linear_bwd_input(df1, lyr.linear1.weight, out=dh2, beta=1.0)  # dx1 = dh2 + df1 W1
    # x1 = LN1(x + drop1(sa))
    if not ln1_done:
        dsa = torch.empty_like(dh2) if p > 0 else None
        dh1 = ops.layernorm_bwd(h1, dh2, lyr.norm1.weight, m1, r1, g(lyr.norm1.weight), g(lyr.norm1.bias),
                                da=dsa, p=p, key=key, site=site + 1)
    if dsa is None:  # p == 0: dsa IS dh1 (read here before the in-proj backward accumulates into it)
        dsa = dh1
    ops.linear_bwd_weight(dsa, att, g(sa_mod.out_proj.weight), db=g(sa_mod.out_proj.bias))
    datt = ops.linear_bwd_input(dsa, sa_mod.out_proj.weight)
    return dh1, datt


def _in_proj_bwd(lyr, x, dqkv, dx=None):
    """in_proj weight gradient and dx (+)= dqkv W_in."""
    g = grad_of
    sa_mod = lyr.self_attn
    if dqkv.dtype == torch.bfloat16:  # bf16 dqkv (RS_ATTN_QKV_BF16): bf16-MFMA weight gradient
        ops.wgrad_bf16(dqkv, x, g(sa_mod.in_proj_weight), db=g(sa_mod.in_proj_bias))
    else:
        ops.linear_bwd_weight(dqkv, x, g(sa_mod.in_proj_weight), db=g(sa_mod.in_proj_bias))
    if dx is None:
        return ops.linear_bwd_input(dqkv, sa_mod.in_proj_weight)
    return ops.linear_bwd_input(dqkv, sa_mod.in_proj_weight, out=dx, beta=1.0)  # dx = dh1 + dqkv Win


def layer_bwd(lyr, saved, dx2, key_pad, B, L, d, H, p, key, site):
    """Backward of layer_fwd. dx2 is consumed; returns dx [B*L, d]."""
    x, qkv, lse = saved[0], saved[1], saved[3]
    dh1, datt = _post_attn_bwd(lyr, saved, dx2, p, key, site)
    dqkv = ops.attn_bwd(qkv, key_pad, saved[2], datt, lse, B, L, d, H, p, key, site)
    return _in_proj_bwd(lyr, x, dqkv, dx=dh1)


def layer_bwd_last(lyr, saved, dx2, key_pad, last, B, L, d, H, p, key, site):
    """Backward of layer_fwd_last: dx2 [B, d] (the encoder output's gradient) -> dx [B*L, d]."""
    x, qkv, lse = saved[0], saved[1], saved[3]
    dh1, datt = _post_attn_bwd(lyr, saved, dx2, p, key, site)
    dqkv = ops.attn_rows_bwd(qkv, key_pad, last, datt, lse, B, L, d, H, p, key, site)
    dx = _in_proj_bwd(lyr, x, dqkv)
    # the residual rows x[b, last[b]] got dh1: add it back at those rows
    ops.gather_bwd([_seg(kind=_hip.RS_SEG_LASTVALID, dim=d, out_col=0, bag=L, idx=last.data_ptr(),
                         grad=dx.data_ptr())], B, dh1)
    return dx


def _layer_site(i):
    return 16 + 8 * i


class SeqEncoderFn(torch.autograd.Function):
    """SequenceEncoder.forward (SequenceEncoder.py:32-56): padding mask from the first feature
    with the all-padding fix (T6), feature embedding + projection + positional embedding (T5),
    n post-LN encoder layers (T8), last-valid gather (T7). Returns [B, d]."""

    @staticmethod
    def forward(ctx, need, enc, seqd, *params):
        proc = enc.feature_embedder
        first = proc.feature_config_list[0]
        main = seqd[first['name']]
        if main.dim() < 2:
            raise RuntimeError('the first sequence feature must be [B, L]')
        main = main if main.dtype == torch.int64 else main.long()
        B, L = int(main.shape[0]), int(main.shape[1])
        d, H = proc.target_dim, enc.n_head
        if L > proc.pos_emb.num_embeddings:
            raise IndexError(f'index out of range in self (sequence length {L} > max_seq_len '
                             f'{proc.pos_emb.num_embeddings})')
        key_pad, last = ops.seq_mask(main, first.get('padding_index', 0))
        p = enc.dropout_p if enc.training else 0.0
        key = ops.rng_next(enc.rng_state) if p > 0 else None
        err = enc.err_flag
        x, in_saved = seq_input_fwd(proc, seqd, B, L, p, key, err, need)
        layers = list(enc.transformer_backbone.layers)
        if enc.transformer_backbone.norm is not None:
            raise NotImplementedError('TransformerEncoder(norm=...) is not used by the reference')
        prune = prune_last_layer() and len(layers) > 0 and L <= 256
        saved = []
        for i, lyr in enumerate(layers):
            if prune and i == len(layers) - 1:
                x, s = layer_fwd_last(lyr, x, key_pad, last, B, L, d, H, p, key, _layer_site(i))
            else:
                x, s = layer_fwd(lyr, x, key_pad, B, L, d, H, p, key, _layer_site(i))
            saved.append(s)
        if prune:
            out = x  # [B, d]: the final layer produced the selected rows only
        else:
            out = torch.empty(B, d, device=x.device, dtype=torch.float32)
            seg = _seg(kind=_hip.RS_SEG_LASTVALID, dim=d, out_col=0, bag=L, idx=last.data_ptr(),
                       table=x.data_ptr())
            ops.gather_fwd([seg], B, out)
        if need:
            ctx.prune = prune
            ctx.enc, ctx.B, ctx.L, ctx.p = enc, B, L, p
            ctx.key, ctx.key_pad, ctx.last = key, key_pad, last
            ctx.in_saved, ctx.layer_saved, ctx.layers = in_saved, saved, layers
            ctx.params = params
            _dp.note_writer(params)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        enc, B, L, p, key = ctx.enc, ctx.B, ctx.L, ctx.p, ctx.key
        proc = enc.feature_embedder
        d, H = proc.target_dim, enc.n_head
        dout = dout.contiguous()
        n = len(ctx.layers)
        # the encoder's weight / LayerNorm / positional gradient reductions queued and run as one
        # launch at the end (ops.deferred_reduce): not under data parallelism (the bucket's
        # all-reduce starts inside seq_input_bwd)
        from .flat import _dp_active
        with ops.deferred_reduce(not _dp_active()):
            if ctx.prune:
                # the fused bf16 FFN backward only reads the output gradient; the fp32 path's
                # norm2 backward runs in place over it (autograd's buffer: give it a copy)
                ls = ctx.layer_saved[n - 1]
                d_last = dout if isinstance(ls[8], tuple) else dout.clone()
                dx = layer_bwd_last(ctx.layers[n - 1], ls, d_last, ctx.key_pad,
                                    ctx.last, B, L, d, H, p, key, _layer_site(n - 1))
                n -= 1
            else:
                dx = torch.zeros(B * L, d, device=dout.device, dtype=torch.float32)
                seg = _seg(kind=_hip.RS_SEG_LASTVALID, dim=d, out_col=0, bag=L, idx=ctx.last.data_ptr(),
                           grad=dx.data_ptr())
                ops.gather_bwd([seg], B, dout)
            for i in reversed(range(n)):
                dx = layer_bwd(ctx.layers[i], ctx.layer_saved[i], dx, ctx.key_pad, B, L, d, H, p, key,
                               _layer_site(i))
            seq_input_bwd(proc, ctx.in_saved, dx, B, L, p, key, ctx.params)
        ctx.layer_saved = ctx.in_saved = ctx.params = None
        return (None, None, None) + (None,) * (len(ctx.needs_input_grad) - 3)


# ================================================================================ tower features
def tower_segments(tower, input_dict, mapping):
    """GenericTower.forward feature loop (GenericTower.py:133-222): config order, pooled sparse
    features in place (T9), dense Linear(1, D) on one column (T11). Returns (segs, params, keep,
    width, seq_col)."""
    segs, params, keep, col = [], [], [], 0
    sparse_cfg = tower.sparse_features or []
    dense_cfg = tower.dense_features or []
    if sparse_cfg and 'sparse' in input_dict:
        sparse = input_dict['sparse']
        seqd = input_dict.get('sequence', {}) or {}
        non_pooled = [f['name'] for f in sparse_cfg if 'pooling' not in f]
        for f in sparse_cfg:
            name = f['name']
            emb = tower.embeddings[name]
            if 'pooling' in f:
                if name not in seqd:
                    print(f'Warning: Pooled feature {name} missing from sequence dict')
                    continue
                x = seqd[name]
                agreed = _agreed(x)
                x = (x if x.dtype == torch.int64 else x.long())
                if x.dim() == 1:
                    x = x.unsqueeze(1)
                x = x.contiguous()
                keep.append(x)
                mode = tower.pooling_config[name]
                if mode not in _hip.RS_POOL:
                    raise ValueError(f'unsupported pooling {mode!r} for {name}')
                segs.append(_seg(kind=_hip.RS_SEG_POOL, dim=emb.embedding_dim, out_col=col,
                                 pool_mode=_hip.RS_POOL[mode], bag=int(x.shape[1]),
                                 vocab=emb.num_embeddings, idx_stride=int(x.stride(0)),
                                 idx=x.data_ptr(), table=emb.weight.data_ptr(), pad_idx=_pad(emb.padding_idx)))
                segs[-1].agreed = agreed
            else:
                if sparse is None:
                    continue
                if mapping and 'sparse' in mapping:
                    c = mapping['sparse'].get(name)
                    if c is None:
                        raise ValueError(f"Feature '{name}' not found in column mapping")
                else:
                    c = non_pooled.index(name)
                sp = sparse if sparse.dtype == torch.int64 else sparse.long()
                keep.append(sp)
                segs.append(_seg(kind=_hip.RS_SEG_SPARSE, dim=emb.embedding_dim, out_col=col,
                                 vocab=emb.num_embeddings, idx_stride=int(sp.stride(0)),
                                 idx=sp.data_ptr() + 8 * c * int(sp.stride(1)),
                                 table=emb.weight.data_ptr(), pad_idx=_pad(emb.padding_idx)))
                ag = _agreed(sparse)
                segs[-1].agreed = None if ag is None else (ag[0], 1, ag[2])
            params.append((emb.weight, None))
            col += emb.embedding_dim
    if dense_cfg and 'dense' in input_dict:
        dense = input_dict['dense']
        names = [f['name'] for f in dense_cfg]
        dn = dense if dense.dtype == torch.float32 else dense.float()
        keep.append(dn)
        for f in dense_cfg:
            name = f['name']
            if mapping and 'dense' in mapping:
                c = mapping['dense'].get(name)
                if c is None:
                    raise ValueError(f"Dense feature '{name}' not found in column mapping")
            else:
                c = names.index(name)
            lin = tower.embeddings[name][0]
            if lin.in_features != 1:
                raise RuntimeError(f'mat1 and mat2 shapes cannot be multiplied: dense feature {name} '
                                   f'feeds one column into Linear({lin.in_features}, {lin.out_features})')
            segs.append(_seg(kind=_hip.RS_SEG_DENSE, dim=lin.out_features, out_col=col,
                             idx_stride=int(dn.stride(0)), x=dn.data_ptr() + 4 * c * int(dn.stride(1)),
                             table=lin.weight.data_ptr(), bias=lin.bias.data_ptr()))
            params.append((lin.weight, lin.bias))
            col += lin.out_features
    for t in keep:
        _hip.require_device(t)
    return segs, params, keep, col


class TowerFeatureFn(torch.autograd.Function):
    """Concat of all tower features [B, total_embed_dim] (GenericTower.py:133-233), with the
    sequence-encoder vector copied into the last slot."""

    @staticmethod
    def forward(ctx, need, tower, input_dict, mapping, seq_vec, *params):
        segs, pp, keep, col = tower_segments(tower, input_dict, mapping)
        B = None
        for t in keep:
            B = int(t.shape[0])
            break
        if seq_vec is not None:
            B = int(seq_vec.shape[0]) if B is None else B
            seq_vec = seq_vec.contiguous()
            segs.append(_seg(kind=_hip.RS_SEG_COPY, dim=int(seq_vec.shape[1]), out_col=col,
                             table=seq_vec.data_ptr()))
            col += int(seq_vec.shape[1])
        if not segs:
            raise RuntimeError('Tower received no valid features. Check if input_dict matches config')
        if col != tower.total_embed_dim:
            raise RuntimeError(f'running_mean should contain {col} elements not {tower.total_embed_dim}')
        if len(segs) > _hip.MAX_SEGMENTS:
            raise RuntimeError(f'too many features in one tower ({len(segs)} > {_hip.MAX_SEGMENTS})')
        dev = tower.feature_bn.weight.device
        out = torch.empty(B, col, device=dev, dtype=torch.float32)
        calls, lazy = _lookup_lazy(segs, [w for w, _ in pp], B, keep, record=need, err=tower.err_flag)
        ops.gather_fwd(segs, B, out, tower.err_flag, lazy=lazy)
        if need:
            ctx.segs, ctx.pp, ctx.keep, ctx.B, ctx.calls = segs, pp, keep, B, calls
            ctx.has_seq = seq_vec is not None
            ctx.seq_shape = tuple(seq_vec.shape) if seq_vec is not None else None
            ctx.params = params
            _dp.note_writer(params)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        dout = dout.contiguous()
        segs = ctx.segs
        dseq = None
        n_feat = len(ctx.pp)
        for s, (w, b) in zip(segs[:n_feat], ctx.pp):
            s.grad = grad_of(w).data_ptr()
            if b is not None:
                s.grad_bias = grad_of(b).data_ptr()
        if ctx.has_seq:
            dseq = torch.empty(ctx.seq_shape, device=dout.device, dtype=torch.float32)
            segs[-1].grad = dseq.data_ptr()
        tables = [w for w, _ in ctx.pp] + [None] * (len(segs) - n_feat)
        _grad_tables(segs, ctx.calls, dout, tables, ctx.B, ctx.params)
        ctx.segs = ctx.keep = ctx.calls = ctx.params = None
        return (None, None, None, None, dseq) + (None,) * (len(ctx.needs_input_grad) - 5)


# ================================================================================ batch norm
class BatchNormFn(torch.autograd.Function):
    """nn.BatchNorm1d (training: batch statistics, running-stat update; eval: running stats),
    G independent row groups (hard-negative slots). GenericTower.py:234 (feature_bn)."""

    @staticmethod
    def forward(ctx, need, bn, x, G, *params):
        x = x.contiguous()
        y, mean, rstd = ops.batchnorm_fwd(x, bn, G, relu=False, training=bn.training)
        if need:
            ctx.bn, ctx.G, ctx.x, ctx.mean, ctx.rstd = bn, G, x, mean, rstd
            ctx.training = bn.training
            ctx.params = params
            _dp.note_writer(params)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        if not ctx.training:
            raise NotImplementedError('backward through BatchNorm1d in eval mode')
        bn = ctx.bn
        dx = ops.batchnorm_bwd(ctx.x, None, dy.contiguous(), bn.weight, ctx.mean, ctx.rstd,
                               grad_of(bn.weight), grad_of(bn.bias), ctx.G, relu=False)
        _dp.note_writer(ctx.params, written=True)
        return (None, None, dx, None) + (None,) * (len(ctx.needs_input_grad) - 4)


# ================================================================================ MLP tower
def _tower_wgrad(dz, h, lin):
    """dW += dz^T h, db += colsum(dz) of one tower Linear."""
    ops.linear_bwd_weight(dz, h, grad_of(lin.weight), db=grad_of(lin.bias))


class MLPFn(torch.autograd.Function):
    """MLP_Tower.forward (Tower.py:16-41): [Linear -> BatchNorm1d -> ReLU -> Dropout] x n,
    Linear, F.normalize(p=2, dim=1)."""

    @staticmethod
    def forward(ctx, need, mlp, x, G, *params):
        seq = mlp.mlp
        n_hidden = (len(seq) - 1) // 4
        p = mlp.dropout_p if mlp.training else 0.0
        key = ops.rng_next(mlp.rng_state) if p > 0 else None
        h = x.contiguous()
        saved = []
        for j in range(n_hidden):
            lin, bn = seq[4 * j], seq[4 * j + 1]
            z = ops.linear_fwd(h, lin.weight, lin.bias)
            # Linear -> BatchNorm1d -> ReLU -> Dropout: BN, ReLU and the dropout in one pass
            y, mean, rstd = ops.batchnorm_fwd(z, bn, G, relu=True, training=mlp.training, drop_p=p,
                                              drop_key=key, drop_site=256 + j)
            saved.append((h, z, y, mean, rstd))
            h = y
        last = seq[len(seq) - 1]
        z = ops.linear_fwd(h, last.weight, last.bias)
        out, norm = ops.l2norm_fwd(z)
        if need:
            ctx.mlp, ctx.G, ctx.p, ctx.key = mlp, G, p, key
            ctx.saved, ctx.h_last, ctx.out, ctx.norm = saved, h, out, norm
            ctx.training = mlp.training
            ctx.params = params
            _dp.note_writer(params)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        if not ctx.training:
            raise NotImplementedError('backward through MLP_Tower in eval mode (BatchNorm running stats)')
        seq = ctx.mlp.mlp
        g = grad_of
        last = seq[len(seq) - 1]
        dz = ops.l2norm_bwd(ctx.out, ctx.norm, dout.contiguous())
        _tower_wgrad(dz, ctx.h_last, last)
        dh = ops.linear_bwd_input(dz, last.weight)
        for j in reversed(range(len(ctx.saved))):
            h, z, y, mean, rstd = ctx.saved[j]
            lin, bn = seq[4 * j], seq[4 * j + 1]
            # y is post-ReLU, post-dropout: y > 0 <=> kept and positive, so the dropout's
            # backward is a scale on the same mask (fused into the BN backward)
            dz = ops.batchnorm_bwd(z, y, dh, bn.weight, mean, rstd, g(bn.weight), g(bn.bias), ctx.G,
                                   relu=True, drop_p=ctx.p)
            _tower_wgrad(dz, h, lin)
            dh = ops.linear_bwd_input(dz, lin.weight)
        ctx.saved = None
        _dp.note_writer(ctx.params, written=True)
        return (None, None, dh, None) + (None,) * (len(ctx.needs_input_grad) - 4)


# ================================================================================ fused tower chain
def tower_chain_supported(feature_bn, mlp, x, G) -> bool:
    """The fused chain (csrc/tower.hip) covers training mode with batch statistics: feature_bn and
    every hidden BatchNorm with a momentum, inputs of width <= 512, hidden widths <= 256, an output
    of width <= 128, all multiples of 4. Eval mode (running statistics) and other shapes take the
    per-op path (BatchNormFn + MLPFn)."""
    if not (feature_bn.training and mlp.training) or x.dim() != 2:
        return False
    seq = mlp.mlp
    n_hidden = (len(seq) - 1) // 4
    bns = [feature_bn] + [seq[4 * j + 1] for j in range(n_hidden)]
    if any(b.momentum is None for b in bns):
        return False
    C0 = int(x.shape[1])
    widths = [int(seq[4 * j].out_features) for j in range(n_hidden)]
    out = int(seq[len(seq) - 1].out_features)
    M = int(x.shape[0])
    if C0 % 4 or C0 > 512 or any(w % 4 or w > 256 for w in widths) or out % 4 or out > 128:
        return False
    return M % G == 0 and M * max([C0, out] + widths) < 2 ** 32


def _tower_sync(mlp, dev, n):
    """Zeroed int32 tickets for the chain's statistics hand-offs (csrc/tower.hip): every kernel
    leaves them zero again, so one buffer per tower module serves every call (and graph replay)."""
    t = getattr(mlp, '_rs_tower_sync', None)
    if t is None or t.device != dev or t.numel() < n:
        t = torch.zeros(max(n, 64), dtype=torch.int32, device=dev)
        mlp._rs_tower_sync = t
    return t


def _tower_wgrad_grouped(mlp, jobs, M, bf):
    """dW += dz^T h, db += colsum(dz) of every Linear of the tower in one launch (rs_tower_wgrad;
    bf16 or fp32 MFMA by the compute mode): 64 x 64 dW tiles x row splits, fixed-order reduction
    of the splits."""
    import ctypes as C
    L = _hip.lib()
    dev = jobs[0][0].device
    n = len(jobs)
    Ns = [int(lin.out_features) for _, _, lin in jobs]
    Ks = [int(lin.in_features) for _, _, lin in jobs]
    wsz = [int(L.rs_tower_wgrad_ws_floats(M, a, b)) for a, b in zip(Ns, Ks)]
    ssz = [int(L.rs_tower_wgrad_sync_ints(a, b)) for a, b in zip(Ns, Ks)]
    ws = torch.empty(sum(wsz), device=dev, dtype=torch.float32)
    t = getattr(mlp, '_rs_tower_wsync', None)
    if t is None or t.device != dev or t.numel() < sum(ssz):
        t = mlp._rs_tower_wsync = torch.zeros(max(sum(ssz), 64), dtype=torch.int32, device=dev)
    woff = [sum(wsz[:i]) for i in range(n)]
    soff = [sum(ssz[:i]) for i in range(n)]
    P = C.c_void_p * n
    arrs = [(C.c_int * n)(*Ns), (C.c_int * n)(*Ks),
            P(*[d.data_ptr() for d, _, _ in jobs]), P(*[h.data_ptr() for _, h, _ in jobs]),
            P(*[grad_of(lin.weight).data_ptr() for _, _, lin in jobs]),
            P(*[grad_of(lin.bias).data_ptr() if lin.bias is not None else None for _, _, lin in jobs]),
            P(*[ws[o:].data_ptr() for o in woff]), P(*[t[o:].data_ptr() for o in soff])]
    ops.call('rs_tower_wgrad', n, M, *[C.addressof(a) for a in arrs], bf, ops.stream())


class TowerChainFn(torch.autograd.Function):
    """GenericTower.feature_bn + MLP_Tower in training mode (GenericTower.py:229-236; Tower.py:16-41)
    as one kernel per Linear (csrc/tower.hip): a BatchNorm's statistics are merged by the last
    workgroup of the kernel that produces its input and applied in the next GEMM's operand
    staging; F.normalize is the last GEMM's epilogue. Same dropout draws as MLPFn (key from the
    MLP's rng state, site 256 + j), same running-statistic updates. Parameter gradients are
    accumulated into the flat buffers."""

    @staticmethod
    def forward(ctx, need, feature_bn, mlp, x, G, *params):
        L = _hip.lib()
        seq = mlp.mlp
        n_hidden = (len(seq) - 1) // 4
        p = mlp.dropout_p
        # the dropout key is drawn by rs_tower_stats (rs_rng_next folded into its launch)
        key = torch.empty(2, dtype=torch.int64, device=x.device) if p > 0 else None
        bf = int(precision.compute_dtype() == 'bf16')
        x = x.contiguous()
        dev = x.device
        M = int(x.shape[0])
        Bg = M // G
        f32 = torch.float32
        widths = [int(x.shape[1])] + [int(seq[4 * j].out_features) for j in range(n_hidden)]
        nsync = [L.rs_tower_sync_ints(G, w) for w in widths]
        sync = _tower_sync(mlp, dev, 2 * sum(nsync) + 2 * L.rs_tower_sync_ints(G, int(seq[-1].in_features)))
        ctx_sync_off = sum(nsync)

        def handoff(w, kind, bn, j):
            """part, sync slice, scratch, mean, rstd and running stats of one BatchNorm."""
            part = torch.empty(L.rs_tower_part_floats(G, Bg, w, kind), device=dev, dtype=f32)
            off = sum(nsync[:j])
            scr = torch.empty(G * 2 * w, device=dev, dtype=torch.float64)
            mean = torch.empty(G * w, device=dev, dtype=f32)
            rstd = torch.empty(G * w, device=dev, dtype=f32)
            track = bn.track_running_stats and bn.running_mean is not None
            return (part.data_ptr(), sync[off:].data_ptr(), scr.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                    ops.P(bn.running_mean) if track else None, ops.P(bn.running_var) if track else None,
                    ops.P(bn.num_batches_tracked) if track else None, float(bn.momentum), float(bn.eps)), \
                (part, scr, mean, rstd)

        hf, keep = handoff(widths[0], 0, feature_bn, 0)
        ops.call('rs_tower_stats', x.data_ptr(), G, Bg, widths[0], *hf, ops.P(mlp.rng_state) if p > 0 else None,
                 ops.P(key), ops.stream())
        A, bn, relu, dp, site = x, feature_bn, 0, 0.0, 0
        mean, rstd = keep[2], keep[3]
        layers = []
        out = norm = None
        for j in range(n_hidden + 1):
            lin = seq[4 * j]
            K, N = int(A.shape[1]), int(lin.out_features)
            final = j == n_hidden
            h = torch.empty(M, K, device=dev, dtype=f32) if need else None
            if final:
                z = None
                out = torch.empty(M, N, device=dev, dtype=f32)
                norm = torch.empty(M, device=dev, dtype=f32)
                hf_out, keep_out = (None,) * 8 + (0.0, 0.0), None
            else:
                z = torch.empty(M, N, device=dev, dtype=f32)
                hf_out, keep_out = handoff(N, 1, seq[4 * j + 1], j + 1)
            ops.call('rs_tower_fwd', A.data_ptr(), G, Bg, K, mean.data_ptr(), rstd.data_ptr(),
                     ops.P(bn.weight), ops.P(bn.bias), relu, dp, ops.P(key) if dp > 0 else None, site,
                     ops.P(h), lin.weight.data_ptr(), lin.bias.data_ptr(), N, ops.P(z), *hf_out,
                     ops.P(out), ops.P(norm), 1e-12, bf, ops.stream())
            layers.append((A, h, mean, rstd, bn, relu, dp, site))
            if not final:
                A, mean, rstd = z, keep_out[2], keep_out[3]
                bn, relu, dp, site = seq[4 * j + 1], 1, p, 256 + j
        if need:
            ctx.mlp, ctx.feature_bn, ctx.G, ctx.key, ctx.bf = mlp, feature_bn, G, key, bf
            ctx.layers, ctx.out, ctx.norm = layers, out, norm
            ctx.sync, ctx.sync_off = sync, ctx_sync_off
            ctx.params = params
            _dp.note_writer(params)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        L = _hip.lib()
        seq = ctx.mlp.mlp
        layers = ctx.layers
        n_hidden = len(layers) - 1
        G, bf, key = ctx.G, ctx.bf, ctx.key
        dout = dout.contiguous()
        M = int(dout.shape[0])
        Bg = M // G
        dev = dout.device
        f32 = torch.float32
        off = ctx.sync_off
        gin, mg, mgx = dout, None, None
        wjobs = []  # every layer's weight gradient in one grouped launch at the end
        for j in range(n_hidden, -1, -1):
            lin = seq[4 * j]
            A, h, mean, rstd, bn_in, relu, dp, site = layers[j]
            Kj, N = int(lin.out_features), int(lin.in_features)
            dz = torch.empty(M, Kj, device=dev, dtype=f32)
            g = torch.empty(M, N, device=dev, dtype=f32)
            part = torch.empty(L.rs_tower_part_floats(G, Bg, N, 1), device=dev, dtype=f32)
            scr = torch.empty(G * 2 * N, device=dev, dtype=torch.float64)
            omg = torch.empty(G * N, device=dev, dtype=f32)
            omgx = torch.empty(G * N, device=dev, dtype=f32)
            if j == n_hidden:  # F.normalize backward in the prologue
                pro = (ctx.out.data_ptr(), ctx.norm.data_ptr(), 1e-12, None, None, None, None, None, None)
            else:  # BN_j backward in the prologue: its z / statistics are layer j+1's input
                zj, _, mj, rj, bnj = layers[j + 1][:5]
                pro = (None, None, 0.0, zj.data_ptr(), mj.data_ptr(), rj.data_ptr(), bnj.weight.data_ptr(),
                       mg.data_ptr(), mgx.data_ptr())
            ops.call('rs_tower_bwd', gin.data_ptr(), G, Bg, Kj, *pro, dz.data_ptr(), lin.weight.data_ptr(), N,
                     A.data_ptr(), mean.data_ptr(), rstd.data_ptr(), ops.P(bn_in.weight) if relu else None,
                     ops.P(bn_in.bias) if relu else None, relu, dp, ops.P(key) if dp > 0 else None, site,
                     g.data_ptr(), part.data_ptr(), ctx.sync[off:].data_ptr(), scr.data_ptr(), omg.data_ptr(),
                     omgx.data_ptr(), grad_of(bn_in.weight).data_ptr(), grad_of(bn_in.bias).data_ptr(), bf,
                     ops.stream())
            off += L.rs_tower_sync_ints(G, N)
            wjobs.append((dz, h, lin))
            gin, mg, mgx = g, omg, omgx
        # feature_bn's dx: the BatchNorm backward prologue with no GEMM
        x, _, m0, r0, fbn = layers[0][:5]
        C0 = int(x.shape[1])
        dx = torch.empty(M, C0, device=dev, dtype=f32)
        ops.call('rs_tower_bwd', gin.data_ptr(), G, Bg, C0, None, None, 0.0, x.data_ptr(), m0.data_ptr(),
                 r0.data_ptr(), fbn.weight.data_ptr(), mg.data_ptr(), mgx.data_ptr(), dx.data_ptr(), None, 0,
                 None, None, None, None, None, 0, 0.0, None, 0, None, None, None, None, None, None, None, None,
                 bf, ops.stream())
        for i in range(0, len(wjobs), 4):  # up to 4 Linears per launch (csrc/tower.hip WG_MAXJ)
            _tower_wgrad_grouped(ctx.mlp, wjobs[i:i + 4], M, bf)
        ctx.layers = None
        _dp.note_writer(ctx.params, written=True)
        return (None, None, None, dx, None) + (None,) * (len(ctx.needs_input_grad) - 5)


# ================================================================================ loss
class InBatchLossFn(torch.autograd.Function):
    """TwoTowerModel.compute_loss (TwoTowerModel.py:81-140, T12): logits = U I^T / T with
    off-diagonal equal-id collisions at -1e9, hard-negative logits appended un-masked,
    cross_entropy(labels = arange(B)), mean."""

    @staticmethod
    def forward(ctx, U, I, item_ids, H, temperature, need=True):
        U = U.contiguous()
        I = I.contiguous()
        B, D = int(U.shape[0]), int(U.shape[1])
        dev = U.device
        # bf16: S tiles recomputed on the MFMA, never stored; fp32: the forward stores S (raw
        # U I^T, [B, ldS]) for the backward to read instead of recomputing (csrc/ce_fused.hip)
        fused = D in (64, 128)
        sfx = '' if precision.compute_dtype() == 'bf16' else '_f32'
        S = None
        if fused and sfx and need:  # no backward (evaluation, no_grad): S is not stored
            S = torch.empty(B, int(_hip.lib().rs_inbatch_ce_s_ld(B)), device=dev, dtype=torch.float32)
        if not fused:
            S = torch.empty(B, B, device=dev, dtype=torch.float32)
            ops.gemm(U, I, S, B, B, D, transA=0, transB=1, lda=D, ldb=D, ldc=B)
        N = 0
        Hc = None
        hsr = hss = 0
        if H is not None:
            # [B, N, D] with unit column stride: contiguous, or the permuted [N, B, D] output of
            # one grouped item-tower pass (no copy either way)
            Hc = H if H.stride(2) == 1 else H.contiguous()
            N = int(Hc.shape[1])
            hsr, hss = int(Hc.stride(0)), int(Hc.stride(1))
        ids = None
        st = 0
        if item_ids is not None:
            ids = item_ids.reshape(-1)
            _hip.require_device(ids)
            if ids.dtype != torch.int64:
                ids = ids.long()
            st = int(ids.stride(0))
        lse = torch.empty(B, device=dev, dtype=torch.float32)
        row_loss = torch.empty(B, device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        uib = None
        if fused:
            w = ops.ws(_hip.lib().rs_inbatch_ce_fused_ws_bytes(B, D), dev)
            extra = (S.data_ptr() if S is not None else None,) if sfx else ()
            name = f'rs_inbatch_ce_fused{sfx}_fwd'
            if not sfx and need and os.environ.get('RSYS_CE_UIB', '1') != '0':
                # bf16: the tiles also write U, I as rounded ([2, B, D]) for the backward's streamed
                # operands -- its rounding launch folded into this one
                uib = torch.empty(2, B, D, device=dev, dtype=torch.bfloat16)
                name += '_uib'
            post = (uib.data_ptr(),) if uib is not None else ()
            _hip.call(name, U.data_ptr(), I.data_ptr(), ops.P(Hc), hsr, hss, ops.P(ids), st,
                      B, N, D, float(temperature), lse.data_ptr(), row_loss.data_ptr(), loss.data_ptr(),
                      *extra, w.data_ptr(), *post, ops.stream())
        else:
            _hip.call('rs_inbatch_ce_fwd', S.data_ptr(), B, U.data_ptr(), ops.P(Hc), hsr, hss, ops.P(ids), st,
                      B, N, D, float(temperature), lse.data_ptr(), row_loss.data_ptr(), loss.data_ptr(),
                      ops.stream())
        ctx.save_for_backward(U, I, Hc if Hc is not None else U)
        ctx.S, ctx.ids, ctx.st, ctx.N, ctx.T, ctx.lse = S, ids, st, N, float(temperature), lse
        ctx.fused = fused
        ctx.uib = uib
        ctx.sfx = sfx
        ctx.hs = (hsr, hss)
        return loss

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        U, I, Hc = ctx.saved_tensors
        B, D = int(U.shape[0]), int(U.shape[1])
        N = ctx.N
        S = ctx.S
        gout = gout.contiguous()
        dhl = torch.empty(B, max(N, 1), device=U.device, dtype=torch.float32) if N else None
        if ctx.fused:
            dU = torch.empty_like(U)
            dI = torch.empty_like(I)
            w = ops.ws(_hip.lib().rs_inbatch_ce_fused_ws_bytes(B, D), U.device)
            extra = (S.data_ptr(),) if ctx.sfx else ()
            uib = ctx.uib
            post = (uib.data_ptr(),) if uib is not None else ()
            _hip.call(f'rs_inbatch_ce_fused{ctx.sfx}_bwd' + ('_uib' if uib is not None else ''), U.data_ptr(),
                      I.data_ptr(), ops.P(Hc) if N else None, ctx.hs[0], ctx.hs[1], ops.P(ctx.ids), ctx.st, B, N, D,
                      ctx.T, ctx.lse.data_ptr(), gout.data_ptr(), dU.data_ptr(), dI.data_ptr(), ops.P(dhl), *extra,
                      w.data_ptr(), *post, ops.stream())
            ctx.S = None
            ctx.uib = None
            dH = None
            if N:
                dH = torch.empty_strided(Hc.shape, Hc.stride(), device=Hc.device, dtype=Hc.dtype)
                _hip.call('rs_hardneg_bwd', U.data_ptr(), Hc.data_ptr(), ctx.hs[0], ctx.hs[1], dhl.data_ptr(),
                          dU.data_ptr(), dH.data_ptr(), B, N, D, ops.stream())
            return dU, dI, None, dH, None, None
        _hip.call('rs_inbatch_ce_bwd', S.data_ptr(), B, U.data_ptr(), ops.P(Hc) if N else None,
                  ctx.hs[0], ctx.hs[1], ops.P(ctx.ids), ctx.st, B, N, D, ctx.T, ctx.lse.data_ptr(),
                  gout.data_ptr(), ops.P(dhl), ops.stream())
        dU = torch.empty_like(U)
        ops.gemm(S, I, dU, B, D, B, transA=0, transB=0, lda=B, ldb=D, ldc=D)       # dS @ I
        dI = torch.empty_like(I)
        ops.gemm(S, U, dI, B, D, B, transA=1, transB=0, lda=B, ldb=D, ldc=D)       # dS^T @ U
        dH = None
        if N:
            dH = torch.empty_strided(Hc.shape, Hc.stride(), device=Hc.device, dtype=Hc.dtype)
            _hip.call('rs_hardneg_bwd', U.data_ptr(), Hc.data_ptr(), ctx.hs[0], ctx.hs[1], dhl.data_ptr(),
                      dU.data_ptr(), dH.data_ptr(), B, N, D, ops.stream())
        ctx.S = None
        return dU, dI, None, dH, None, None
