"""Data parallelism over RCCL (torch.distributed 'nccl' backend = RCCL on ROCm), one process
per GPU. The batch is sharded: each rank runs the full training step on its own
B samples (own in-batch negatives, own BatchNorm statistics, as DDP applied to the reference),
then an all-reduce of the flat gradient buffer's dense part (~3.5 MB for the demo schema, 0.9 MB
at C3) and an identical clip + Adam on every rank. Parameters are broadcast from rank 0 at start.
The all-reduce is bucketed per tower and started inside the backward (GradBuckets, `overlap`):
each tower's bucket goes as soon as its last gradient writer has queued its kernels, so it
runs under the other tower's backward and the large-table segment sums.

Below W = 4, large tables trained by lazy-exact Adam (flat.py) stay replicated (a 10M x 128 table
with its Adam state is ~20 GB: it fits 288 GB of HBM many times over) but their gradient is NOT
all-reduced densely (5 GB per table per step). SURVEY §8e's bag-gradient exchange instead: for
every lookup call of such a table the backward keeps the call's OUTPUT gradient ([rows, D]: the
pooled bag gradient, the single-id feature gradient, or the per-token gradient); one all-gather
moves every rank's [rows, bag] int32 ids and [rows, D] gradient (C3 pooled history: 0.8 + 2 MB
per rank), and every rank sorts the gathered ids and runs the deterministic segment sum over
them (csrc/lookup.hip). All ranks therefore hold bitwise-identical gradient rows and step the
same rows in the same order: the clip norm and Adam agree bitwise, with no host sync and no
count exchange.

Row-sharded tables (flat.py; default for every large table at W >= 4): rank r holds only the
rows id % W == r. One-id-per-row lookups exchange the rows of their distinct ids all-to-all (the
backward returns per-id gradient rows to the owners); pooled bags all-gather ids and
reduce-scatter per-rank partial bags, their backward all-gathers the bag gradients
(LazyTable.shard_lookup, exchange below). Per-rank row work stays constant in W.
"""
from __future__ import annotations

import os
import threading

import torch
import torch.distributed as dist

from . import _hip, streams
from .flat import SEG_MEAN, SEG_SUM, ensure_flat, flat_of


def is_active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 and not _AGREE.local


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
    # the row-sharded tables (the end of the buffer) differ by rank by construction
    dist.broadcast(f.data[:f.replicated_numel], src)
    for b in model.buffers():
        if b.dtype in (torch.float32, torch.int64) and b.numel() > 0:
            dist.broadcast(b, src)


def broadcast_buffers(model: torch.nn.Module, src: int = 0):
    """Rank-0 buffers (BatchNorm running statistics, num_batches_tracked) to every rank, as DDP's
    broadcast_buffers=True does before each forward: each rank's training batches move its own
    running statistics, so without this an eval-mode pass (validate) differs by rank."""
    if not is_active():
        return
    for b in model.buffers():
        if b.dtype in (torch.float32, torch.int64) and b.numel() > 0:
            dist.broadcast(b, src)


def broadcast_scalar(x: float, src: int = 0) -> float:
    """Rank src's value of a host scalar on every rank (one decision for all ranks)."""
    if not is_active():
        return x
    dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else torch.device('cpu')
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.broadcast(t, src)
    return float(t.item())


def sync_seed(src: int = 0) -> int:
    """Seed torch's default generator with rank src's initial seed on every rank, so that every
    rank draws the same epoch order (the shards of one permutation)."""
    seed = int(torch.initial_seed()) % (1 << 52)
    seed = int(broadcast_scalar(float(seed), src))
    torch.manual_seed(seed)
    return seed


EMPTY_ID = -(1 << 31)  # the pad slot of a ragged call's id exchange (csrc/lookup.hip kEmptyId)


class _Agreement(threading.local):
    """This forward's batch shapes agreed over the ranks (agree_batch): per batch tensor its
    per-dimension maxima over the ranks and whether any rank's dimension differs."""

    def __init__(self):
        self.table = None   # {(data_ptr, shape): (max dims, ragged)} of this forward's batch; dropped
                            # when the forward ends (end_forward): its keys are allocator addresses
        self.sig = None     # the local shape signature of the last agreed batch
        self.static = False  # the last agreed batch had the same shapes on every rank
        self.step = False   # a batch was agreed since the last allreduce_gradients (clear_agreement)
        self.local = 0      # local_only() depth: this process steps alone (no collective)


_AGREE = _Agreement()


class local_only:
    """`with local_only(): ...` -- the model steps alone inside a distributed job (a single-rank
    emulation or evaluation on one rank): no collective is issued for its shapes or gradients."""

    def __enter__(self):
        _AGREE.local += 1
        return self

    def __exit__(self, *exc):
        _AGREE.local -= 1
        return False


def _batch_tensors(b, out):
    """The tensors of a batch dict in a fixed order (sorted keys; lists in order; a materialised
    hard-negative list's stacked batch): the same order on every rank of one config."""
    if isinstance(b, torch.Tensor):
        out.append(b)
    elif isinstance(b, dict):
        for k in sorted(b, key=str):
            _batch_tensors(b[k], out)
    elif isinstance(b, (list, tuple)):
        for v in b:
            _batch_tensors(v, out)
        st = getattr(b, 'stacked', None)
        if st is not None:
            _batch_tensors(st, out)
    return out


def agree_batch(batch) -> None:
    """One agreement per forward (TwoTowerModel.forward) of every batch tensor's shape -- a
    fixed-size header all-reduce (tensor count, total rank: batches of different structure raise
    before any variable-length collective), then one all-reduce of every dimension: the lookup
    calls of the large tables take their common shapes from it (agreed_dims, valid until the
    forward ends: end_forward) instead of one blocking all-reduce per call. Ranks' batches of equal shapes (the bench's, a loader with
    drop_last and equal list lengths) need nothing more; ragged ones (the collate pads each
    batch's lists to its own longest) pad every call to the per-dimension maxima.
    Inside a hipGraph capture nothing can be exchanged: the batch must have the shapes of the last
    eagerly agreed one, and that one must have been equal on every rank; otherwise this raises
    (the ranks' collectives would not match and the job would hang)."""
    if not is_active() or _AGREE.local:
        return
    ts = _batch_tensors(batch, [])
    sig = tuple(tuple(int(d) for d in t.shape) for t in ts)
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        if sig != _AGREE.sig or not _AGREE.static:
            raise RuntimeError('rsys data parallel: a batch captured into a hipGraph must have the shapes '
                               'of the last eager step, equal on every rank (run one eager step on the '
                               'captured shapes first)')
        _AGREE.table = {(t.data_ptr(), tuple(t.shape)): (tuple(t.shape), False) for t in ts}
        _AGREE.step = True
        return
    dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else torch.device('cpu')
    # a fixed-size header first (tensor count, total rank of the tensors): batches of different
    # structure would otherwise all-reduce vectors of different lengths (a hang, or garbage)
    head = [len(sig), sum(len(x) for x in sig)]
    h = torch.tensor(head + [-x for x in head], dtype=torch.int64, device=dev)
    dist.all_reduce(h, op=dist.ReduceOp.MAX)
    h = h.tolist()
    if h[:2] != [-x for x in h[2:]]:
        raise RuntimeError('rsys data parallel: the ranks\' batches hold different tensors (same config?)')
    flat = [len(sig)] + [len(x) for x in sig] + [d for x in sig for d in x]
    v = torch.tensor(flat + [-x for x in flat], dtype=torch.int64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    v = v.tolist()
    n = len(flat)
    mx, mn = v[:n], [-x for x in v[n:]]
    if mx[:1 + len(sig)] != mn[:1 + len(sig)]:
        raise RuntimeError('rsys data parallel: the ranks\' batches hold different tensors (same config?)')
    table, at = {}, 1 + len(sig)
    for t, shp in zip(ts, sig):
        k = len(shp)
        dims_max = tuple(mx[at:at + k])
        table[(t.data_ptr(), shp)] = (dims_max, dims_max != tuple(mn[at:at + k]))
        at += k
    _AGREE.table = table
    _AGREE.sig = sig
    _AGREE.static = all(not r for _, r in table.values())
    _AGREE.step = True


def end_forward():
    """The forward that agreed its batch is over (TwoTowerModel.forward): its table keyed by batch
    tensor addresses is dropped, so a later lookup outside a TwoTowerModel forward (validate()'s
    item indexing through get_item_embeddings, a tower called on its own) can never match a
    reused allocator address of the same shape and take another batch's dims; it agrees per call
    (agree_max) instead. The step's `static` verdict stays until clear_agreement."""
    _AGREE.table = None


def agreed_dims(t):
    """(per-dimension maxima over the ranks, ragged?) of batch tensor t as this forward's
    agree_batch saw it, or None (not a batch tensor, or no agreement this step)."""
    if _AGREE.table is None or t is None:
        return None
    return _AGREE.table.get((t.data_ptr(), tuple(int(d) for d in t.shape)))


def clear_agreement():
    """End of the step's collectives (allreduce_gradients): later lookups outside a
    TwoTowerModel forward agree per call again."""
    _AGREE.table = None
    _AGREE.step = False


def agree_max(*vals):
    """The max over ranks of each host int (one tiny all-reduce + host sync): the fallback for a
    lookup call whose shape agree_batch did not cover (a tower called outside TwoTowerModel).
    Inside a hipGraph capture no exchange is possible: raises unless this step's batch was
    agreed equal on every rank (then the local values are everyone's)."""
    if not is_active() or _AGREE.local:
        return list(vals)
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        if _AGREE.step and _AGREE.static:
            return list(vals)
        raise RuntimeError('rsys data parallel: a lookup shape cannot be agreed inside a hipGraph capture')
    dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend() == 'nccl' else torch.device('cpu')
    t = torch.tensor(vals, dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [int(x) for x in t.tolist()]


def call_shape(rows, bag, agreed=None):
    """(rows_max, bag_max, ragged) over the ranks for a [rows, bag] lookup call; `agreed`: the
    same triple derived from agree_batch (no collective)."""
    if agreed is not None:
        return agreed
    rmax, rmin, bmax, bmin = agree_max(rows, -rows, bag, -bag)
    return rmax, bmax, rmax != -rmin or bmax != -bmin


def pad_ids(ids32, rows, bag, rmax, bmax):
    """A [rows, bag] int32 id matrix padded to [rmax, bmax] with EMPTY_ID."""
    if (rows, bag) == (rmax, bmax):
        return ids32
    out = torch.full((rmax, bmax), EMPTY_ID, dtype=torch.int32, device=ids32.device)
    out[:rows, :bag] = ids32.view(rows, bag)
    return out.view(-1)


def allreduce_flat_grad(flat_grad: torch.Tensor):
    """Sum the flat gradient over ranks (the mean is folded into the optimizer's grad_scale)."""
    with streams.on_root():
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)


class GradBuckets:
    """The dense part of a flat gradient [0, dense_numel) split into buckets, one per tower: a
    tower's non-lazy parameters are contiguous in the flat buffer (module.parameters() order).
    Every op that writes a bucket's gradient in the backward registers itself in its forward
    (`note_writer`) and reports in its backward once its dense-gradient kernels are queued
    (`note_writer(..., written=True)`), before any large-table work. While armed (`overlap`), the last writer of a
    bucket starts the bucket's all-reduce asynchronously: RCCL's stream waits for the writer's
    stream and the all-reduce runs while the rest of the backward (the other tower, the
    large-table sort / segment sums) does. allreduce_gradients then only waits for those
    and all-reduces what no writer covered. The launch order is the autograd engine's node order,
    the same on every rank (same graph), so the ranks' collectives match."""

    def __init__(self, f, spans):
        self.f = f
        self.spans = spans       # [(lo, hi)] per bucket, disjoint, inside [0, dense_numel)
        self.pending = [0] * len(spans)
        self.armed = 0
        self.works = []          # (bucket, async work) launched in this backward
        self.launched = 0        # buckets started inside a backward, all steps (tests)

    def reset(self):
        self.pending = [0] * len(self.spans)
        self.works = []

    def _launch(self, b):
        lo, hi = self.spans[b]
        self.launched += 1
        # issued from the root stream when a tower's side stream is current (streams.on_root: RCCL's
        # stream forked from a side stream breaks the captured step); waited for on the root
        with streams.on_root(sync=False):
            self.works.append((b, dist.all_reduce(self.f.grad[lo:hi], op=dist.ReduceOp.SUM, async_op=True)))

    def writer(self, params, delta):
        b = _bucket_of(params)
        if b is None:
            return
        if delta > 0 and any(w[0] == b for w in self.works):
            # a second forward before allreduce_gradients: its gradient would be added after
            # the bucket's all-reduce (gradient accumulation needs the backward outside overlap)
            raise RuntimeError('rsys data parallel: a forward writing an already all-reduced gradient '
                               'bucket (call allreduce_gradients after each backward run under '
                               'dist.overlap)')
        self.pending[b] += delta
        if delta < 0 and self.pending[b] == 0 and self.armed and all(w[0] != b for w in self.works):
            self._launch(b)

    def finish(self):
        """Wait (stream order) for the buckets launched in the backward; -> their spans."""
        done = []
        for b, w in self.works:
            w.wait()
            done.append(self.spans[b])
        self.reset()
        return done


def _bucket_of(params):
    for p in params:
        b = getattr(p, '_rs_dp_bucket', None)
        if b is not None:
            return b
    return None


def setup_buckets(model: torch.nn.Module, groups) -> GradBuckets | None:
    """One gradient bucket per module of `groups` (the towers) over the model's flat buffer;
    None if a group's dense parameters do not form one span of their own."""
    f = flat_of(next(model.parameters()))
    if f is None:
        return None
    gb = getattr(f, 'dp_buckets', None)
    if gb is not None or getattr(f, 'dp_buckets_tried', False):
        return gb
    f.dp_buckets_tried = True
    lazy = {id(t.param) for t in f.lazy}
    off = {id(p): (o, o + p.numel()) for p, o in zip(f.params, f.offsets)}
    owner, spans = {}, []
    for b, m in enumerate(groups):
        ps = [p for p in m.parameters() if id(p) not in lazy and id(p) in off]
        if not ps or any(id(p) in owner for p in ps):
            return None
        for p in ps:
            owner[id(p)] = b
        spans.append((min(off[id(p)][0] for p in ps), max(off[id(p)][1] for p in ps)))
    # a span may hold no other group's (or ungrouped) parameter: its all-reduce would sum a
    # gradient some other writer is still producing
    for p in f.params:
        if id(p) in lazy:
            continue
        lo, hi = off[id(p)]
        for b, (s0, s1) in enumerate(spans):
            if lo < s1 and hi > s0 and owner.get(id(p)) != b:
                return None
    for p in f.params:
        if id(p) in owner:
            p._rs_dp_bucket = owner[id(p)]
    f.dp_buckets = GradBuckets(f, spans)
    return f.dp_buckets


def note_writer(params, written=False):
    """Forward (written=False) / backward (written=True) of an op writing dense gradients of
    `params` (GradBuckets). No-op without data parallelism or buckets."""
    if not params:
        return
    f = flat_of(params[0])
    gb = getattr(f, 'dp_buckets', None) if f is not None else None
    if gb is not None:
        gb.writer(params, -1 if written else 1)


class overlap:
    """`with overlap(model): loss.backward()` -- start each tower's gradient all-reduce inside
    the backward (GradBuckets). allreduce_gradients must follow, as without it."""

    def __init__(self, model):
        f = flat_of(next(model.parameters())) if is_active() else None
        self.gb = getattr(f, 'dp_buckets', None) if f is not None else None
        if (self.gb is not None and dist.get_backend() != 'nccl' and torch.cuda.is_available()
              and torch.cuda.is_current_stream_capturing()):
            self.gb = None  # host-staged collectives (gloo) cannot be captured

    def __enter__(self):
        if self.gb is not None:
            self.gb.armed += 1
        return self

    def __exit__(self, *exc):
        if self.gb is not None:
            self.gb.armed -= 1
        return False


def _complement(n, spans):
    out, at = [], 0
    for lo, hi in sorted(spans):
        if lo > at:
            out.append((at, lo))
        at = max(at, hi)
    if at < n:
        out.append((at, n))
    return out


def allreduce_gradients(model: torch.nn.Module, optimizer=None):
    """After backward: RCCL all-reduce of the model's flat gradient -- the buckets the backward
    started (overlap) are waited for, the rest is reduced here, in as few calls as it spans;
    the optimizer scales by 1/world (so clip + Adam see the average gradient, as DDP)."""
    if not is_active():
        return
    params = list(model.parameters())
    f = flat_of(params[0])
    if f is None:
        raise RuntimeError('model is not flattened')
    gb = getattr(f, 'dp_buckets', None)
    done = gb.finish() if gb is not None else []
    for lo, hi in _complement(f.dense_numel, done):
        allreduce_flat_grad(f.grad[lo:hi])
    if f.lazy:
        exchange_lazy_grads(f)
    clear_agreement()
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


class _ExchangeBuffers:
    """Per (table, call) all-gather buffers, reused while the call shapes stay the same."""

    def __init__(self):
        self.bufs = {}

    def get(self, key, shape, dtype, dev):
        b = self.bufs.get(key)
        if b is None or b.shape != shape or b.dtype != dtype or b.device != dev:
            b = torch.empty(shape, dtype=dtype, device=dev)
            self.bufs[key] = b
        return b


def _all_gather(out, inp):
    with streams.on_root():
        if dist.get_backend() == 'nccl':
            dist.all_gather_into_tensor(out, inp)
        else:
            dist.all_gather(list(out.chunk(dist.get_world_size())), inp)


all_gather_into = _all_gather


def all_to_all(out, inp):
    """out block s = rank s's inp block `rank` (equal splits along dim 0): RCCL's all-to-all; on
    other backends (gloo: ranks sharing one GPU in tests) through host copies."""
    if dist.get_backend() == 'nccl':
        with streams.on_root():
            dist.all_to_all_single(out, inp)
        return
    o = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(o, inp.cpu())
    out.copy_(o)


def reduce_scatter_sum(out, inp):
    """out = sum over ranks of inp's block `rank` (inp: world blocks of out's size). RCCL's
    reduce-scatter; other backends (gloo sharing one GPU in tests): an all-reduce of inp and the
    block."""
    if dist.get_backend() == 'nccl':
        with streams.on_root():
            dist.reduce_scatter_tensor(out, inp)
        return
    dist.all_reduce(inp)
    r = dist.get_rank()
    n = out.numel()
    out.view(-1).copy_(inp.view(-1)[r * n:(r + 1) * n])


def _exchange_sharded(t, bufs, world, dev):
    """Row-sharded table. All-to-all calls: each rank's per-slot gradient buckets go to the
    owners (all_to_all_single), which segment-sum them onto their rows. Pooled-bag calls:
    all-gather each call's output gradient rows; the call's sorted keys are the union's local
    rows, so the segment sum lands on the rows this rank owns."""
    calls = [c for c in t.calls if c.dseg is not None]
    for i, c in enumerate(calls):
        acc = len(calls) > 1
        if c.a2a is not None:
            recv = bufs.get(('shard_a2a', i), tuple(c.dseg.shape), torch.float32, dev)
            all_to_all(recv, c.dseg)
            c.dseg = None
            t.a2a_owner_segsum(c, recv, acc)
            continue
        all_g = bufs.get(('shard_g', i), (world * c.local_rows, t.D), torch.float32, dev)
        _all_gather(all_g, c.dseg)
        c.dseg = None
        c.keep = (c.keep, all_g)
        t.segsum(c, all_g.data_ptr(), t.D, accumulate=acc)
    t.exchanged = calls


def exchange_lazy_grads(f):
    """Bag-gradient exchange of every lazy table of flat buffer f (see module doc)."""
    for t in f.lazy:
        if t.calls:
            exchange_table(t)


def exchange_table(t):
    """The gradient exchange of one lazy table's calls this step (module doc): every rank calls
    it for the same tables in the same order."""
    world = dist.get_world_size()
    dev = t.flat.data.device
    bufs = getattr(t, '_dp_bufs', None)
    if bufs is None:
        bufs = t._dp_bufs = _ExchangeBuffers()
    if t.shard is not None:
        _exchange_sharded(t, bufs, world, dev)
        return
    union = []
    for i, c in enumerate(t.calls):
        if c.dseg is None:  # looked up without a backward (e.g. under no_grad)
            continue
        ids = bufs.get(('ids', i), (c.n,), torch.int32, dev)
        _hip.call('rs_pack_ids', c.ids_ptr, c.id_bytes, c.rows, c.bag, c.row_stride, ids.data_ptr(),
                  _stream())
        rmax, bmax, ragged = call_shape(c.rows, c.bag, c.agreed)
        g, mode = c.dseg, c.mode
        if ragged:
            # pad to the ranks' common shape: pad ids sort last (skipped), pad rows are zero; a
            # mean bag's 1 / length is applied to this rank's rows here and the union sums
            ids = pad_ids(ids, c.rows, c.bag, rmax, bmax)
            g = torch.zeros(rmax, t.D, device=dev)
            g[:c.rows] = c.dseg
            if mode == SEG_MEAN:
                _hip.call('rs_scale_inplace', g.data_ptr(), c.rows * t.D, 1.0 / c.bag, None, _stream())
                mode = SEG_SUM
        all_ids = bufs.get(('all_ids', i), (world * rmax * bmax,), torch.int32, dev)
        all_g = bufs.get(('all_g', i), (world * rmax, t.D), torch.float32, dev)
        _all_gather(all_ids, ids)
        _all_gather(all_g, g)
        union.append((all_ids, all_g, c, rmax, bmax, mode))
    calls = []
    for all_ids, all_g, c, rmax, bmax, mode in union:
        u = t.sort_call(all_ids.data_ptr(), world * rmax, bmax, bmax, c.pad, mode, id_bytes=4,
                        keep=(all_ids, all_g))
        calls.append((u, all_g))
    t.exchanged = [u for u, _ in calls]
    for u, all_g in calls:
        t.segsum(u, all_g.data_ptr(), t.D, accumulate=len(calls) > 1)
