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
(per-row `last` step, this step's sorted lookups: csrc/lookup.hip). The dense kernels then only
sweep [0, dense_numel); the tables are touched row-by-row. State (weights, exp_avg, exp_avg_sq) stays
bitwise what dense Adam would produce; rows are brought current before every read (forward
gather, state_dict, load_state_dict).

Row sharding (data parallel only): a large table is split by rows across the W
ranks, rank r owning rows id % W == r at local row id / W (its weight, exp_avg and exp_avg_sq:
1/W of the memory each; placed last in the flat buffer, never broadcast or all-reduced). By
default every large table is sharded once W >= 4 (then the replicated form's per-rank row work,
which grows with W, would dominate); RSYS_SHARD_ROWS=N shards tables of at least N rows at any
W > 1 (0: never). Two exchange forms (LazyTable.shard_lookup):
  * one id per output row (single-id features, the encoder's per-token history): all-to-all of
    ROWS (csrc/shard.hip). Each rank buckets its distinct ids by owner, the owners gather (after
    the catch-up) and return exactly those rows; the backward segment-sums the call's gradient
    per distinct id and returns it to the owners, which segment-sum what they receive onto their
    rows. Per-rank work and traffic: the call's distinct ids, independent of W;
  * pooled bags (mean / sum): all-gather of the ids, each rank sums the rows it owns into
    per-requester partial bags, a reduce-scatter hands every rank the pooled rows of its own
    batch ([W x rows, D]: one row per bag, not per lookup); the backward all-gathers the bag
    gradients and each rank segment-sums the contributions to its own rows.
state_dict() assembles the full table (a collective: every rank calls it); load_state_dict takes
the owned rows of a full table.
"""
from __future__ import annotations

import os

import torch

from . import _hip

ALIGN = 16  # floats (64 B)


PROFILE_CALLS = None  # profiling only (bench.py): a list receiving (D, keys, n) of every sorted call


def profile_call_rows(calls):
    """[(D, lookups, distinct rows)] of recorded sorted calls (keys ascending; out-of-range ids
    sort last as 0xFFFFFFFF and are not rows). One host sync: profiling passes only."""
    out = []
    for D, keys, n in calls or ():
        if n == 0:
            out.append((D, 0, 0))
            continue
        k = keys[:n]
        valid = k != -1
        heads = torch.ones_like(k, dtype=torch.bool)
        heads[1:] = k[1:] != k[:-1]
        out.append((D, n, int((heads & valid).sum())))
    return out


def lazy_rows_threshold() -> int:
    return int(os.environ.get('RSYS_LAZY_ROWS', 1 << 16))


class LookupCall:
    """One forward lookup of a large table: the call's ids sorted by row (rs_lookup_sort).
    keys[n] = row ids ascending (out-of-range ids last as 0xFFFFFFFF), vals[n] = lookup index
    r * bag + l, ascending within a row. Kept until the optimizer step (gradient segment sums,
    clip norm and Adam all walk the distinct rows of `keys`). Under data parallelism the backward
    keeps the call's output gradient rows (dseg) for the exchange. keys, vals and the sort
    workspace are allocated on the forward's stream and held here until the step ends."""

    __slots__ = ('keys', 'vals', 'ws', 'n', 'rows', 'bag', 'pad', 'mode', 'ids_ptr',
                 'id_bytes', 'row_stride', 'keep', 'dseg', 'local_rows', 'own_rows', 'prescale', 'a2a',
                 'agreed', 'catchup_due')

    def __init__(self, keys, vals, n, rows, bag, pad, mode, ids_ptr, id_bytes, row_stride, keep, ws=None):
        self.keys, self.vals, self.n, self.rows, self.bag = keys, vals, n, rows, bag
        self.pad, self.mode = pad, mode
        self.ids_ptr, self.id_bytes, self.row_stride, self.keep = ids_ptr, id_bytes, row_stride, keep
        self.ws = ws
        self.dseg = None
        self.local_rows = rows  # row-sharded call: the calling rank's rows (rows = world x local)
        self.own_rows = None  # ragged row-sharded bags: this rank's rows of the padded local_rows
        self.prescale = None  # ragged mean bags: 1 / this rank's bag length (union summed as SUM)
        self.a2a = None  # all-to-all row-sharded call: the requester side (A2ARequest)
        self.agreed = None  # data parallel: (rows, bag, ragged) over the ranks (dist.agree_batch)
        self.catchup_due = False  # lookup(defer_catchup=True): its sorted catch-up is the caller's (catchup_batch)


# rs_segsum modes: one id per gradient row, mean bag, sum bag (max pooling: atomic scatter)
SEG_ONE, SEG_MEAN, SEG_SUM = 0, 1, 2


class A2ARequest:
    """The requester side of an all-to-all row-sharded lookup (LazyTable.shard_lookup): its
    sorted ids (keys, vals), the segment-sum keys of the slots (ckey), the bucket capacity and the
    buffers the backward reuses."""

    __slots__ = ('keys', 'vals', 'ckey', 'idx', 'n', 'cap', 'recv_rows', 'send_grad', 'keep')

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)


def shard_capacity(n: int, world: int) -> int:
    """Bucket capacity per (rank, owner) pair of an all-to-all lookup of n ids: the expected n / W
    distinct ids with a margin (RSYS_SHARD_CAPACITY, default 1.5x) plus 64. Ids are deduplicated
    before bucketing, so hot (Zipf) ids do not skew the buckets; ids are spread over owners by
    id % W. An overflow raises at the next check_errors() (the flag's bit 2)."""
    f = float(os.environ.get('RSYS_SHARD_CAPACITY', '1.5'))
    return int(-(-n * f // world)) + 64


class LazyTable:
    """Row bookkeeping of one large [V, D] table trained by lazy-exact Adam.

    Every lookup of the table in a step is a LookupCall (sorted ids). Per step:
      forward  : rs_lookup_sort, then rs_sorted_catchup brings the call's rows to the current
                 optimizer step before the gather reads them (a lookup without a backward:
                 rs_lookup_catchup in id order, no sort);
      backward : rs_segsum writes each distinct row's gradient (plain stores; added to the row
                 when the table has several calls this step), deterministic;
      optimizer: rs_sorted_sqnorm (clip-norm partials) and rs_sorted_adam over each call's
                 distinct rows; a row looked up by several calls is stepped once, by the first
                 (rs_sorted_owner). The calls are then dropped.
    The gradient rows of a large table are zero except the rows of this step's calls."""

    def __init__(self, flat, index, param, offset, shard=None, vocab=None):
        self.flat, self.index, self.param, self.offset = flat, index, param, offset
        self.V, self.D = int(param.shape[0]), int(param.shape[1])  # local rows when sharded
        self.shard = shard  # (world, rank) of a row-sharded table, else None
        self.V_full = int(vocab) if vocab is not None else self.V
        dev = param.device
        # (moments' step, parameters' step) per row: the forward catch-up may bring p alone ahead
        self.last = torch.zeros(self.V, 2, dtype=torch.int32, device=dev)
        self.owner = None   # [V] lowest call index per row; allocated for multi-call steps
        self.calls = []     # this step's LookupCalls, in forward order
        self.exchanged = None  # data parallel: the union calls that replaced the local ones

    def ptr(self, t):
        return t.data_ptr() + 4 * self.offset

    def sort_call(self, ids_ptr, rows, bag, row_stride, pad, mode, id_bytes=8, keep=None):
        """Sort a [rows, bag] id matrix by row (rs_lookup_sort) into a LookupCall."""
        dev = self.param.device
        n = rows * bag
        keys = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        vals = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(n, self.V))
        ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dev) if wsb else None
        _hip.call('rs_lookup_sort', ids_ptr, id_bytes, rows, bag, row_stride, self.V, keys.data_ptr(),
                  vals.data_ptr(), None if ws is None else ws.data_ptr(), _stream())
        if PROFILE_CALLS is not None:
            PROFILE_CALLS.append((self.D, keys, n))
        return LookupCall(keys, vals, n, rows, bag, -1 if pad is None else int(pad), mode, ids_ptr,
                          id_bytes, row_stride, keep, ws)

    def lookup(self, ids_ptr, rows, bag, row_stride, pad, mode, id_bytes=8, keep=None, record=True,
               read_through=False, agreed=None, defer_catchup=False):
        """Forward hook: bring the call's rows to the current optimizer step before they are
        gathered and, when the step will train on this lookup (`record`), list it for the step
        with its ids sorted by row. Default: sort, then rs_sorted_catchup over the distinct rows.
        `read_through`: sort only -- the gather brings the rows current in registers
        (rs_gather_fwd_lazy, read_through_args) and the optimizer step replays the same steps.
        A lookup no backward follows (evaluation) is not sorted at all: rs_lookup_catchup works
        in id order. (Measured and rejected: the sort of recorded lookups on a side stream with
        their catch-up in id order -- 0.833 vs 0.839 ms per C3 step, within noise.)"""
        c = None
        if record:
            c = self.sort_call(ids_ptr, rows, bag, row_stride, pad, mode, id_bytes, keep)
            c.agreed = agreed
            self.calls.append(c)
        opt = self.flat.lazy_opt
        if opt is None or rows * bag == 0 or (c is not None and read_through):
            return c
        hyper = (opt['step_dev'].data_ptr(), opt['consts'].data_ptr(), *opt['hyper'], _stream())
        if c is not None and defer_catchup:
            c.catchup_due = True  # issued with the other tables' by catchup_batch
            return c
        if c is not None:
            _hip.call('rs_sorted_catchup', c.keys.data_ptr(), c.n, self.D, self.ptr(self.flat.data),
                      self.ptr(opt['m']), self.ptr(opt['v']), self.last.data_ptr(), *hyper)
        else:
            _hip.call('rs_lookup_catchup', ids_ptr, id_bytes, rows, bag, row_stride, self.V, self.D,
                      self.ptr(self.flat.data), self.ptr(opt['m']), self.ptr(opt['v']), self.last.data_ptr(),
                      *hyper)
        return c

    def read_through_args(self):
        """rs_gather_fwd_lazy's launch arguments (m_off, v_off, step, consts, b1, b2, eps, wd), or
        None before the first optimizer step (every row is current then)."""
        opt = self.flat.lazy_opt
        if opt is None:
            return None
        base = self.flat.data.data_ptr()
        return ((opt['m'].data_ptr() - base) // 4, (opt['v'].data_ptr() - base) // 4, opt['step_dev'].data_ptr(),
                opt['consts'].data_ptr(), *opt['hyper'])

    def shard_lookup(self, seg, rows, record=True, err_ptr=None):
        """Forward of a lookup of a row-sharded table (module doc) -> (LookupCall or None, the
        segment that now reads this rank's rows, tensors to keep alive until the step ends). seg:
        the rs_feature_seg_t of the lookup (sparse: all-to-all; pooled mean / sum: partial bags)."""
        if seg.kind == _hip.RS_SEG_SPARSE:
            return self._shard_lookup_a2a(seg, rows, record, err_ptr)
        return self._shard_lookup_bags(seg, rows, record, err_ptr)

    def _shard_lookup_a2a(self, seg, rows, record, err_ptr):
        """One id per output row: all-to-all of the distinct ids' rows (csrc/shard.hip)."""
        from .dist import all_to_all
        W, r = self.shard
        dev = self.param.device
        L = _hip.lib()
        n = rows
        keys = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        vals = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        wsb = int(L.rs_lookup_sort_ws_bytes(n, self.V_full))
        ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dev) if wsb else None
        if n:
            _hip.call('rs_lookup_sort', seg.idx, 8, rows, 1, seg.idx_stride, self.V_full, keys.data_ptr(),
                      vals.data_ptr(), None if ws is None else ws.data_ptr(), _stream())
        from .dist import agree_max
        agreed = getattr(seg, 'agreed', None)
        # one bucket shape on every rank (ragged calls): from the forward's batch agreement
        cap = shard_capacity(agreed[0] if agreed is not None else agree_max(n)[0], W)
        send_ids = torch.empty(W * cap, dtype=torch.int32, device=dev)
        counts = torch.empty(W, dtype=torch.int32, device=dev)
        ckey = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        idx = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        bws = torch.empty(int(L.rs_shard_bucket_ws_bytes(n, W)) // 4 + 1, dtype=torch.int32, device=dev)
        _hip.call('rs_shard_bucket', keys.data_ptr(), vals.data_ptr(), n, W, cap, int(seg.pad_idx),
                  send_ids.data_ptr(), counts.data_ptr(), ckey.data_ptr(), idx.data_ptr(), err_ptr, bws.data_ptr(),
                  _stream())
        recv_counts = torch.empty_like(counts)
        all_to_all(recv_counts, counts)
        recv_ids = torch.empty_like(send_ids)
        all_to_all(recv_ids, send_ids)
        # owner: the requested local rows, brought current, gathered into the return buckets
        ids64 = torch.empty(W * cap, dtype=torch.int64, device=dev)
        ids32 = torch.empty(W * cap, dtype=torch.int32, device=dev)
        _hip.call('rs_shard_recv', recv_ids.data_ptr(), recv_counts.data_ptr(), W, cap, self.V, ids64.data_ptr(),
                  ids32.data_ptr(), err_ptr, _stream())
        pad = seg.pad_idx
        pad_local = pad // W if pad >= 0 and pad % W == r else None
        c = self.sort_call(ids32.data_ptr(), W * cap, 1, 1, pad_local, SEG_ONE, id_bytes=4, keep=(ids32,))
        opt = self.flat.lazy_opt
        if opt is not None:
            _hip.call('rs_sorted_catchup', c.keys.data_ptr(), c.n, self.D, self.ptr(self.flat.data),
                      self.ptr(opt['m']), self.ptr(opt['v']), self.last.data_ptr(), opt['step_dev'].data_ptr(),
                      opt['consts'].data_ptr(), *opt['hyper'], _stream())
        from . import ops
        send_rows = torch.empty(W * cap, self.D, device=dev)
        gs = _hip.FeatureSeg()
        gs.kind, gs.dim, gs.out_col, gs.pool_mode, gs.bag, gs.pad_idx = _hip.RS_SEG_SPARSE, self.D, 0, 0, 1, -1
        gs.vocab, gs.idx_stride, gs.idx, gs.table = self.V, 1, ids64.data_ptr(), self.ptr(self.flat.data)
        ops.gather_fwd([gs], W * cap, send_rows, None)
        # the returned buckets, then one zero row: the row an out-of-range or overflowed lookup reads
        recv_rows = torch.empty(W * cap + 1, self.D, device=dev)
        recv_rows[W * cap].zero_()
        all_to_all(recv_rows[:W * cap], send_rows)
        # this rank's lookups read their rows out of the returned buckets
        out = _hip.FeatureSeg()
        out.kind, out.dim, out.out_col, out.pool_mode, out.bag, out.pad_idx = (_hip.RS_SEG_SPARSE, self.D,
                                                                                 seg.out_col, 0, 1, -1)
        out.vocab, out.idx_stride, out.idx, out.table = W * cap + 1, 1, idx.data_ptr(), recv_rows.data_ptr()
        keep = (idx, recv_rows)
        if not record:
            return None, out, keep
        c.local_rows = rows
        c.a2a = A2ARequest(keys=keys, vals=vals, ckey=ckey, idx=idx, n=n, cap=cap, recv_rows=recv_rows,
                           send_grad=None, keep=(ws, bws, recv_counts, recv_ids, ids64, send_ids, counts))
        self.calls.append(c)
        return c, out, keep

    def _shard_lookup_bags(self, seg, rows, record, err_ptr):
        """Pooled bags: all-gather of the ids, per-requester partial bags of the owned rows, a
        reduce-scatter of the [W x rows, D] partial bags (module doc)."""
        from . import ops
        from .dist import all_gather_into, call_shape, pad_ids, reduce_scatter_sum
        W, r = self.shard
        dev = self.param.device
        bag = seg.bag
        if seg.pool_mode not in (_hip.RS_POOL['mean'], _hip.RS_POOL['sum']):
            # lazy_tables() keeps max-pooled tables replicated (their arg-max gradient is exchanged
            # as per-lookup rows): a sharded one here means the table is also max-pooled elsewhere
            raise RuntimeError('row-sharded table looked up with max pooling (mark it _rs_no_shard)')
        mode = SEG_MEAN if seg.pool_mode == _hip.RS_POOL['mean'] else SEG_SUM
        n = rows * bag
        ids32 = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        if n:
            _hip.call('rs_pack_ids', seg.idx, 8, rows, bag, seg.idx_stride, ids32.data_ptr(), _stream())
        # ranks' calls of different shapes (the collate pads to each batch's longest bag): padded to
        # the common [rmax, bmax] with empty slots (dist.EMPTY_ID: no row, no gradient)
        rmax, bmax, ragged = call_shape(rows, bag, getattr(seg, 'agreed', None))
        if ragged and n:
            ids32 = pad_ids(ids32, rows, bag, rmax, bmax)
        nm = rmax * bmax
        all32 = torch.empty(W * max(nm, 1), dtype=torch.int32, device=dev)
        all_gather_into(all32, ids32 if nm else torch.empty(1, dtype=torch.int32, device=dev))
        if nm == 0:
            res = torch.zeros(rows, self.D, device=dev)
            return None, _copy_seg(seg, res), (res,)
        all32 = all32.view(W, -1)[:, :nm].contiguous()
        local = torch.empty(W * nm, dtype=torch.int64, device=dev)
        _hip.call('rs_shard_map_ids', all32.data_ptr(), W * nm, self.V_full, W, r, local.data_ptr(), err_ptr,
                  _stream())
        opt = self.flat.lazy_opt
        if opt is not None:
            _hip.call('rs_lookup_catchup', local.data_ptr(), 8, W * rmax, bmax, bmax, self.V, self.D,
                      self.ptr(self.flat.data), self.ptr(opt['m']), self.ptr(opt['v']), self.last.data_ptr(),
                      opt['step_dev'].data_ptr(), opt['consts'].data_ptr(), *opt['hyper'], _stream())
        # per requesting rank and row: the sum of the owned rows of its bag (others read as 0)
        part = torch.empty(W * rmax, self.D, device=dev)
        ps = _hip.FeatureSeg()
        ps.kind, ps.dim, ps.out_col, ps.pool_mode, ps.bag, ps.pad_idx = (_hip.RS_SEG_POOL, self.D, 0,
                                                                         _hip.RS_POOL['sum'], bmax, -1)
        ps.vocab, ps.idx_stride, ps.idx, ps.table = self.V, bmax, local.data_ptr(), self.ptr(self.flat.data)
        ops.gather_fwd([ps], W * rmax, part, None)
        out = torch.empty(rmax, self.D, device=dev)
        reduce_scatter_sum(out, part)
        if mode == SEG_MEAN:  # this rank's own bag length
            _hip.call('rs_scale_inplace', out.data_ptr(), out.numel(), 1.0 / bag, None, _stream())
        c = None
        if record:
            pad = seg.pad_idx
            pad_local = pad // W if pad >= 0 and pad % W == r else -1
            c = self.sort_call(local.data_ptr(), W * rmax, bmax, bmax, pad_local if pad_local >= 0 else None,
                               SEG_SUM if ragged and mode == SEG_MEAN else mode, id_bytes=8, keep=(local, all32))
            c.local_rows = rmax
            c.own_rows = rows
            if ragged and mode == SEG_MEAN:
                c.prescale = 1.0 / bag
            self.calls.append(c)
        return c, _copy_seg(seg, out), (out,)

    def segsum(self, c, dout_ptr, ldo, accumulate=None):
        """Backward: the table gradient of call c from its output gradient (dout_ptr = the
        feature's first column, row stride ldo floats). Under data parallelism a local call only
        keeps its output gradient rows; dist.exchange_lazy_grads sums every rank's."""
        if c.n == 0:
            return
        dev = self.param.device
        if c.a2a is not None:  # all-to-all sharded call: the gradient of each distinct id, per slot
            self._a2a_local_segsum(c, dout_ptr, ldo)
            return
        if accumulate is None:
            if _dp_active():
                # this rank's output gradient rows (a row-sharded call spans world x local_rows;
                # a ragged one pads them with zero rows and applies a mean bag's 1 / length here)
                own = c.own_rows if c.own_rows is not None else c.local_rows
                c.dseg = (torch.zeros if own != c.local_rows else torch.empty)(c.local_rows, self.D, device=dev)
                _hip.call('rs_pack_rows', dout_ptr, ldo, own, self.D, c.dseg.data_ptr(), _stream())
                if c.prescale is not None:
                    _hip.call('rs_scale_inplace', c.dseg.data_ptr(), own * self.D, c.prescale, None, _stream())
                return
            accumulate = len(self.calls) > 1
        ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(c.n, self.D)) // 4 + 1, dtype=torch.int32,
                         device=dev)
        _hip.call('rs_segsum', c.keys.data_ptr(), c.vals.data_ptr(), c.n, c.bag, c.mode, c.pad,
                  dout_ptr, ldo, self.D, self.ptr(self.flat.grad), int(accumulate), ws.data_ptr(),
                  _stream())

    def segsum_call(self, c, dout_ptr, ldo):
        """The plain (single-process) segsum of call c as an rs_segsum_call_t for rs_segsum_batch
        (functions._grad_tables batches the calls of different tables): (call, ws), or None where
        segsum() takes another path (empty call, all-to-all, data parallelism)."""
        if c.n == 0 or c.a2a is not None or _dp_active():
            return None
        ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(c.n, self.D)) // 4 + 1, dtype=torch.int32,
                         device=self.param.device)
        sc = _hip.SegsumCall(keys=c.keys.data_ptr(), vals=c.vals.data_ptr(), n=c.n, bag=c.bag, mode=c.mode,
                             pad=c.pad, dout=dout_ptr, ldo=ldo, grad=self.ptr(self.flat.grad),
                             accumulate=int(len(self.calls) > 1), ws=ws.data_ptr())
        return sc, ws

    def _a2a_local_segsum(self, c, dout_ptr, ldo):
        """Backward, requester side of an all-to-all call: the call's output gradient summed per
        distinct id into its bucket slot (send_grad [W x cap, D]); dist.exchange_lazy_grads sends
        the buckets to the owners."""
        q = c.a2a
        dev = self.param.device
        W = self.shard[0]
        if dout_ptr % 16 or ldo % 4:  # rs_segsum reads float4 rows
            packed = torch.empty(q.n, self.D, device=dev)
            _hip.call('rs_pack_rows', dout_ptr, ldo, q.n, self.D, packed.data_ptr(), _stream())
            dout_ptr, ldo = packed.data_ptr(), self.D
            q.keep = q.keep + (packed,)
        q.send_grad = torch.empty(W * q.cap, self.D, device=dev)
        ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(q.n, self.D)) // 4 + 1, dtype=torch.int32, device=dev)
        if q.n:
            _hip.call('rs_segsum', q.ckey.data_ptr(), q.vals.data_ptr(), q.n, 1, SEG_ONE, -1, dout_ptr, ldo,
                      self.D, q.send_grad.data_ptr(), 0, ws.data_ptr(), _stream())
        q.keep = q.keep + (ws,)
        c.dseg = q.send_grad  # pending: the exchange sends it to the owners

    def a2a_owner_segsum(self, c, recv_grad, accumulate):
        """Owner side: the received per-slot gradients segment-summed onto the owned rows (the
        owner call's keys are the received slots sorted by local row)."""
        ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(c.n, self.D)) // 4 + 1, dtype=torch.int32,
                         device=self.param.device)
        _hip.call('rs_segsum', c.keys.data_ptr(), c.vals.data_ptr(), c.n, 1, SEG_ONE, c.pad, recv_grad.data_ptr(),
                  self.D, self.D, self.ptr(self.flat.grad), int(accumulate), ws.data_ptr(), _stream())
        c.keep = (c.keep, recv_grad, ws)

    def step_calls(self):
        """The calls whose rows the optimizer steps (the data-parallel union calls once the
        gradients were exchanged). Output gradients kept for an exchange that did not happen
        (a model stepped without dist.allreduce_gradients inside a distributed job) are
        segment-summed locally here, so the gradient is never lost."""
        if self.exchanged is not None:
            return self.exchanged
        if self.shard is not None and any(c.dseg is not None for c in self.calls):
            from .dist import exchange_table  # row-sharded: only the owners can sum (a collective)
            exchange_table(self)
            return self.exchanged
        for c in self.calls:
            if c.dseg is not None:
                g, c.dseg = c.dseg, None
                self.segsum(c, g.data_ptr(), self.D, accumulate=len(self.calls) > 1)
        return self.calls

    def mark_owners(self):
        calls = self.step_calls()
        if len(calls) <= 1:
            return None
        if self.owner is None:
            self.owner = torch.full((self.V,), 0x7fffffff, dtype=torch.int32, device=self.param.device)
        for i, c in enumerate(calls):
            _hip.call('rs_sorted_owner', c.keys.data_ptr(), c.n, self.owner.data_ptr(), i, _stream())
        return self.owner

    def end_step(self):
        self.calls = []
        self.exchanged = None

    def flush(self):
        opt = self.flat.lazy_opt
        if opt is None:
            return
        _hip.call('rs_sparse_flush', self.ptr(self.flat.data), self.ptr(opt['m']), self.ptr(opt['v']),
                  self.last.data_ptr(), self.V, self.D, opt['step_dev'].data_ptr(),
                  opt['consts'].data_ptr(), *opt['hyper'], _stream())

    def zero_grad(self):
        """Zero the gradient rows of pending calls (a backward not followed by an optimizer
        step) and drop them: their rows are current, and a row with a zero gradient needs no
        explicit Adam step (the next catch-up replays it)."""
        for c in self.calls + (self.exchanged or []):
            if c.n > 0:
                _hip.call('rs_sorted_zero_grad', c.keys.data_ptr(), c.n, self.D, self.ptr(self.flat.grad),
                          _stream())
        self.end_step()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dp_active():
    from .dist import is_active  # a rank stepping alone (dist.local_only) is not data parallel
    return is_active()


def _is_lazy(p, lazy_ids):
    return id(p) in lazy_ids


SHARD_AUTO_WORLD = 4  # default: every large (lazy) table row-sharded from this world size on


def shard_threshold(world: int) -> int:
    """Tables with at least this many rows are row-sharded under data parallelism (0: none).
    RSYS_SHARD_ROWS=N sets it; by default every large table is sharded once world >= 4, where
    the replicated form's union row work (world x the rows) would dominate the step."""
    env = os.environ.get('RSYS_SHARD_ROWS')
    if env is not None and env != '':
        return int(env)
    return lazy_rows_threshold() if world >= SHARD_AUTO_WORLD else 0


def shard_spec(param):
    """(world, rank) if this lazy table is row-sharded, else None."""
    if not _dp_active():
        return None
    d = torch.distributed
    thr = shard_threshold(d.get_world_size())
    if thr <= 0 or int(param.shape[0]) < thr or getattr(param, '_rs_no_shard', False):
        return None
    return d.get_world_size(), d.get_rank()


def shard_rows(V: int, world: int, rank: int) -> int:
    """Rows of a V-row table owned by `rank` (ids rank, rank + world, ...)."""
    return (V - rank + world - 1) // world if rank < V else 0


def unshard(parts, V: int):
    """Full [V, D] table from every rank's [shard_rows(V, W, r), D] shard (rank order)."""
    W = len(parts)
    full = parts[0].new_empty(V, parts[0].shape[1])
    for r, p in enumerate(parts):
        full[r::W] = p[:shard_rows(V, W, r)]
    return full


class FlatParams:
    def __init__(self, params, device, lazy=()):
        """params: in module.parameters() order; lazy: the subset (large [V, D] embedding
        weights) trained by lazy-exact Adam, laid out after all other parameters."""
        self.params = list(params)
        lazy_ids = {id(p) for p in lazy}
        # row-sharded lazy tables (module doc): their local shard only, laid out last
        shards = {id(p): shard_spec(p) for p in self.params if _is_lazy(p, lazy_ids)}
        shapes = []
        for p in self.params:
            sp = shards.get(id(p))
            shapes.append(p.shape if sp is None else torch.Size((shard_rows(p.shape[0], *sp), p.shape[1])))
        self.offsets = [0] * len(self.params)
        off = 0
        for group in (0, 1, 2):  # dense, replicated lazy, row-sharded lazy
            for i, p in enumerate(self.params):
                g = 0 if not _is_lazy(p, lazy_ids) else (2 if shards[id(p)] is not None else 1)
                if g == group:
                    self.offsets[i] = off
                    off += (shapes[i].numel() + ALIGN - 1) // ALIGN * ALIGN
            if group == 0:
                self.dense_numel = off
            elif group == 1:
                self.replicated_numel = off  # broadcast / all-reduce never touch the shards
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        with torch.no_grad():
            for p, o, shp in zip(self.params, self.offsets, shapes):
                if p.dtype != torch.float32:
                    raise TypeError(f'only fp32 parameters are supported, got {p.dtype}')
                sp = shards.get(id(p))
                if sp is None:
                    self.data[o:o + p.numel()].copy_(p.detach().reshape(-1))
                else:  # rank 0's initial table, then this rank's rows
                    full = p.detach().to(device).contiguous()
                    torch.distributed.broadcast(full, 0)
                    self.data[o:o + shp.numel()].copy_(full[sp[1]::sp[0]].reshape(-1))
        vocab = {}
        for p, o, shp in zip(self.params, self.offsets, shapes):
            vocab[id(p)] = int(p.shape[0]) if len(p.shape) else 0
            p.data = self.data[o:o + shp.numel()].view(shp)
            p._rs_flat = self
            p._rs_offset = o
        self.lazy = [LazyTable(self, i, p, o, shard=shards[id(p)], vocab=vocab[id(p)])
                     for i, (p, o) in enumerate(zip(self.params, self.offsets)) if _is_lazy(p, lazy_ids)]
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


def _copy_seg(seg, rows_t):
    """A segment copying precomputed rows [rows, D] into seg's columns."""
    s = _hip.FeatureSeg()
    s.kind, s.dim, s.out_col, s.pad_idx = _hip.RS_SEG_COPY, seg.dim, seg.out_col, -1
    s.table = rows_t.data_ptr()
    return s


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
    tables = []
    for owner in module.modules():
        if not isinstance(getattr(owner, 'embeddings', None), torch.nn.ModuleDict):
            continue
        pooling = getattr(owner, 'pooling_config', None) or {}
        for name, m in owner.embeddings.items():
            if pooling.get(name) == 'max' and isinstance(m, torch.nn.Embedding):
                # the arg-max backward has no partial-bag form: a max-pooled table stays replicated
                # under data parallelism (dist.exchange_table, functions._max_as_single)
                m.weight._rs_no_shard = True
            tables.append(m)
    for m in tables:
        # the per-row kernels cover a row with at most 64 lanes x 4 columns (csrc/lookup.hip) and
        # the segment sum works on float4 rows: other widths stay ordinary (dense-Adam) tables
        if isinstance(m, torch.nn.Embedding) and m.num_embeddings >= thr and thr > 0 and \
                m.embedding_dim <= 256 and m.embedding_dim % 4 == 0:
            out.append(m.weight)
            if not getattr(m, '_rs_lazy_hooks', False):
                m.register_state_dict_pre_hook(_flush_hook)
                m._register_state_dict_hook(_shard_state_hook)
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
    t = getattr(module.weight, '_rs_lazy', None)
    k = prefix + 'weight'
    if t is not None and t.shard is not None and k in state_dict and \
            state_dict[k].shape[0] == t.V_full and t.V_full != t.V:
        W, r = t.shard
        state_dict[k] = state_dict[k][r::W]  # a full table: this rank's rows


def _shard_state_hook(module, state_dict, prefix, local_metadata):
    """state_dict() of a row-sharded table: the full [V, D] table, gathered from every rank (a
    collective), so checkpoints keep the reference's shapes."""
    t = getattr(module.weight, '_rs_lazy', None)
    k = prefix + 'weight'
    if t is None or t.shard is None or k not in state_dict:
        return
    state_dict[k] = gather_shards(t.param.detach(), t)


def gather_shards(local, t):
    """The full [V, D] tensor of row-sharded table t from every rank's [shard rows, D] slice
    `local` (its weights or an Adam moment): one all-gather, a collective every rank calls."""
    W, r = t.shard
    n = -(-t.V_full // W)
    pad = torch.zeros(n, t.D, device=t.param.device, dtype=local.dtype)
    pad[:t.V] = local.to(t.param.device)
    parts = [torch.empty_like(pad) for _ in range(W)]
    torch.distributed.all_gather(parts, pad)
    return unshard(parts, t.V_full)


def lookup_table(weight, ids_ptr, rows, bag, row_stride, pad, mode, keep=None, record=True, read_through=False,
                 agreed=None, defer_catchup=False):
    """Forward-side hook of the custom ops for a table lookup: a LookupCall for large
    (lazy-Adam) tables (None for ordinary ones, and for a lookup no backward follows: `record`
    False, the rows are only brought current). `defer_catchup`: a recorded call's sorted catch-up
    is left to the caller (catchup_batch, the call's catchup_due set)."""
    t = getattr(weight, '_rs_lazy', None)
    if t is None or flat_of(weight) is not t.flat:
        return None
    return t.lookup(ids_ptr, rows, bag, row_stride, pad, mode, keep=keep, record=record, read_through=read_through,
                    agreed=agreed, defer_catchup=defer_catchup)


def catchup_batch(items):
    """The deferred forward catch-ups of [(LazyTable, LookupCall)] (calls with catchup_due) as
    rs_sorted_catchup_batch launches: up to 8 calls of one row-width class, one flat buffer and
    DISTINCT tables a launch (two calls of one table touch the same rows: the later one runs in a later launch,
    after the earlier one's rows are current), in the given order."""
    from .optim import _row_class
    todo = [(t, c) for t, c in items if c is not None and c.catchup_due]
    while todo:
        batch, rest, tables, cls = [], [], set(), None
        for t, c in todo:
            k = (_row_class(t.D), id(t.flat))  # one optimizer state per launch
            if len(batch) < 8 and id(t) not in tables and (cls is None or k == cls):
                batch.append((t, c))
                tables.add(id(t))
                cls = k
            else:
                rest.append((t, c))
        opt = batch[0][0].flat.lazy_opt
        arr = (_hip.SortedCall * len(batch))()
        for j, (t, c) in enumerate(batch):
            sc = arr[j]
            sc.keys, sc.n, sc.D, sc.call = c.keys.data_ptr(), c.n, t.D, 0
            sc.p, sc.g = t.ptr(t.flat.data), None
            sc.m, sc.v = t.ptr(opt['m']), t.ptr(opt['v'])
            sc.last, sc.owner = t.last.data_ptr(), None
            c.catchup_due = False
        import ctypes
        _hip.call('rs_sorted_catchup_batch', ctypes.addressof(arr), len(batch), opt['step_dev'].data_ptr(),
                  opt['consts'].data_ptr(), *opt['hyper'], _stream())
        todo = rest


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
