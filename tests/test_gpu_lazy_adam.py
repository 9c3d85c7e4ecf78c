"""Sorted lookups and lazy-exact Adam for large tables (csrc/lookup.hip, csrc/sparse.hip, flat.py;
SURVEY.md §7.2 / trap T16).

The reference trains its embeddings with dense gradients (nn.Embedding -> embedding_dense_backward)
and torch.optim.Adam, so every row moves every step once its exp_avg is non-zero. Here a large
table's lookups are radix-sorted by row; the gradient is a deterministic segment sum over the
sorted lookups, and only looked-up rows are stepped (skipped zero-gradient steps are replayed when
a row is next read). These tests hold:
  * the sort bit-exact against numpy's stable argsort (int64 / int32 ids, pad, out-of-range ids,
    one-tile and multi-tile sizes, 300 .. 100M-row vocabularies);
  * the segment sum against a float64 restatement of embedding_dense_backward (single ids, mean
    and sum bags, Zipf-skewed ids whose hot rows span hundreds of chunks), bitwise reproducible;
  * lazy Adam BITWISE equal to the dense kernel on the same gradients, at every read and after a
    flush, with one and with several lookup calls per step.
"""
import numpy as np
import pytest
import torch

from recommendsystemproject_amd import _hip, ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
LR, B1, B2, EPS = 1e-2, 0.9, 0.999, 1e-8
SENT = 0xFFFFFFFF


def _sort(ids, vocab, bag=None, stride=None, no_ws=False):
    """rs_lookup_sort of a [rows, bag] id tensor on the device -> (keys, vals) as numpy uint32.
    no_ws: no workspace (n <= 4096: the one-workgroup radix sort instead of the counting sort)."""
    rows = ids.shape[0]
    bag = bag or (ids.shape[1] if ids.dim() == 2 else 1)
    stride = stride or (ids.stride(0) if ids.dim() == 2 else 1)
    n = rows * bag
    keys = torch.empty(max(n, 1), dtype=torch.int32, device=DEV)
    vals = torch.empty(max(n, 1), dtype=torch.int32, device=DEV)
    wsb = 0 if no_ws else int(_hip.lib().rs_lookup_sort_ws_bytes(n, vocab))
    ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=DEV) if wsb else None
    _hip.call('rs_lookup_sort', ids.data_ptr(), ids.element_size(), rows, bag, stride, vocab,
              keys.data_ptr(), vals.data_ptr(), None if ws is None else ws.data_ptr(), ops.stream())
    return keys, vals


def _expect(ids_np, vocab):
    flat = ids_np.reshape(-1).astype(np.int64)
    key = np.where((flat >= 0) & (flat < vocab), flat, SENT).astype(np.uint64)
    order = np.argsort(key, kind='stable')
    return key[order].astype(np.uint32), order.astype(np.uint32)


@pytest.mark.parametrize('n,bag,vocab,dtype,no_ws', [
    (1, 1, 300, torch.int64, False), (4096, 1, 1_000_000, torch.int64, False), (3000, 3, 19, torch.int64, False),
    (4096, 1, 10_000_000, torch.int64, True), (3000, 3, 19, torch.int64, True), (257, 1, 1000, torch.int32, False),
    (8192, 1, 10_000_000, torch.int64, False), (6000, 2, 1_000_000, torch.int32, False),
    (8193, 1, 10_000_000, torch.int64, False),
    (4097, 1, 10_000_000, torch.int64, False), (204_800, 50, 10_000_000, torch.int64, False),
    (100_000, 1, 100_000_000, torch.int32, False), (65_536, 4, 65_536, torch.int64, False),
    (819_200, 1, 100_000_000, torch.int64, False)])
def test_lookup_sort_bit_exact(n, bag, vocab, dtype, no_ws):
    g = np.random.default_rng(n + bag)
    rows = max(n // bag, 1)
    ids = g.integers(0, vocab, size=(rows, bag))
    ids[g.random((rows, bag)) < 0.1] = 0                    # padding-like repeats
    ids[g.random((rows, bag)) < 0.05] = g.integers(0, 50, size=1)  # a hot row
    if ids.size > 10:
        ids.reshape(-1)[3] = vocab + 5                       # out of range
        ids.reshape(-1)[7] = -2
    t = torch.from_numpy(ids).to(dtype).to(DEV)
    keys, vals = _sort(t, vocab, no_ws=no_ws)
    ek, ev = _expect(ids, vocab)
    assert np.array_equal(keys.cpu().numpy().view(np.uint32)[:ids.size], ek)
    assert np.array_equal(vals.cpu().numpy().view(np.uint32)[:ids.size], ev)


def test_lookup_sort_strided_column():
    """A single-id feature is a column of the [B, S] sparse matrix, read in place (stride S)."""
    g = np.random.default_rng(5)
    m = g.integers(0, 5_000_000, size=(6000, 5))
    t = torch.from_numpy(m).to(DEV)
    col = 3
    keys = torch.empty(6000, dtype=torch.int32, device=DEV)
    vals = torch.empty(6000, dtype=torch.int32, device=DEV)
    wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(6000, 5_000_000))
    ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=DEV)
    _hip.call('rs_lookup_sort', t.data_ptr() + 8 * col, 8, 6000, 1, 5, 5_000_000, keys.data_ptr(),
              vals.data_ptr(), ws.data_ptr(), ops.stream())
    ek, ev = _expect(m[:, col], 5_000_000)
    assert np.array_equal(keys.cpu().numpy().view(np.uint32), ek)
    assert np.array_equal(vals.cpu().numpy().view(np.uint32), ev)


def _segsum(keys, vals, n, bag, mode, pad, dout, V, D, acc=0, grad=None):
    grad = torch.zeros(V, D, device=DEV) if grad is None else grad
    ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(n, D)) // 4 + 1, dtype=torch.int32, device=DEV)
    _hip.call('rs_segsum', keys.data_ptr(), vals.data_ptr(), n, bag, mode, pad, dout.data_ptr(),
              dout.stride(0), D, grad.data_ptr(), acc, ws.data_ptr(), ops.stream())
    return grad


def _ref_grad(ids, dout, V, mode, pad):
    """float64 embedding_dense_backward of the lookup (mean: grad / bag per lookup)."""
    ids = ids.reshape(ids.shape[0], -1)
    bag = ids.shape[1]
    g = np.zeros((V, dout.shape[1]))
    d = dout.astype(np.float64) / (bag if mode == 1 else 1)
    for l in range(bag):
        col = ids[:, l]
        ok = (col >= 0) & (col < V) & (col != pad)
        np.add.at(g, col[ok], d[ok])
    return g


@pytest.mark.parametrize('mode,bag,D,zipf', [(0, 1, 128, False), (1, 50, 128, False), (2, 3, 40, False),
                                             (1, 50, 128, True), (0, 1, 64, True), (1, 20, 200, True),
                                             (0, 1, 16, False)])
def test_segsum_matches_dense_backward(mode, bag, D, zipf):
    g = np.random.default_rng(D + bag)
    V, B, pad = 300_000, 4096, 0
    if zipf:
        ids = np.minimum(g.zipf(1.05, size=(B, bag)) - 1, V - 1)
    else:
        ids = g.integers(0, V, size=(B, bag))
    ids[g.random((B, bag)) < 0.3] = pad
    ids[0, 0] = V + 1  # out of range: no gradient
    t = torch.from_numpy(ids).to(DEV)
    dout = torch.randn(B, D + 8, device=DEV)[:, 4:4 + D]  # a column slice of a wider gradient
    keys, vals = _sort(t, V)
    got = _segsum(keys, vals, B * bag, bag, mode, pad, dout, V, D)
    want = _ref_grad(ids, dout.cpu().numpy(), V, mode, pad)
    err = np.abs(got.cpu().numpy() - want).max()
    assert err <= 1e-5 * max(1.0, np.abs(want).max()), err
    again = _segsum(keys, vals, B * bag, bag, mode, pad, dout, V, D)
    assert torch.equal(got, again)  # deterministic
    assert not got[pad].any()
    # accumulate = 1 adds to what is there
    base = torch.randn(V, D, device=DEV)
    acc = _segsum(keys, vals, B * bag, bag, mode, pad, dout, V, D, acc=1, grad=base.clone())
    assert torch.allclose(acc, base + got, atol=1e-5)


@pytest.mark.parametrize('D', [128, 64, 40])
def test_segsum_batch_bitwise(D):
    """rs_segsum_batch (several tables' calls in one launch pair, functions._grad_tables) gives
    the bits of the calls one by one: single ids, a mean bag of 50 (C3's user side), a sum bag,
    accumulate on and off, n from 1 to 204,800."""
    g = np.random.default_rng(D)
    specs = [(1_000_000, 4096, 1, 0, 0, 0), (300_000, 4096, 50, 1, 0, 1), (5000, 777, 3, 2, 2, 0), (10, 1, 1, 0, -1, 1)]
    calls, singles, keep = [], [], []
    for V, B, bag, mode, pad, acc in specs:
        ids = g.integers(0, V, size=(B, bag))
        ids[g.random((B, bag)) < 0.2] = max(pad, 0)
        t = torch.from_numpy(ids).to(DEV)
        dout = torch.randn(B, D + 8, device=DEV)[:, 4:4 + D]
        keys, vals = _sort(t, V)
        base = torch.randn(V, D, device=DEV)
        n = B * bag
        singles.append(_segsum(keys, vals, n, bag, mode, pad, dout, V, D, acc=acc, grad=base.clone()))
        grad = base.clone()
        ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(n, D)) // 4 + 1, dtype=torch.int32, device=DEV)
        keep += [t, dout, keys, vals, grad, ws]
        calls.append(_hip.SegsumCall(keys=keys.data_ptr(), vals=vals.data_ptr(), n=n, bag=bag, mode=mode, pad=pad,
                                     dout=dout.data_ptr(), ldo=dout.stride(0), grad=grad.data_ptr(), accumulate=acc,
                                     ws=ws.data_ptr()))
    arr = (_hip.SegsumCall * len(calls))(*calls)
    import ctypes
    _hip.call('rs_segsum_batch', ctypes.addressof(arr), len(calls), D, ops.stream())
    torch.cuda.synchronize()
    for i, want in enumerate(singles):
        assert torch.equal(keep[6 * i + 4], want), i
    # one table twice in a batch is refused
    arr2 = (_hip.SegsumCall * 2)(calls[0], calls[0])
    with pytest.raises(RuntimeError):
        _hip.call('rs_segsum_batch', ctypes.addressof(arr2), 2, D, ops.stream())


def test_segsum_equals_atomic_scatter():
    """rs_segsum == the atomic scatter of rs_gather_bwd (ordinary tables) up to summation order."""
    from recommendsystemproject_amd.functions import _seg
    V, D, B, bag, pad = 200_000, 128, 512, 7, 3
    gen = torch.Generator().manual_seed(11)
    ids = torch.randint(0, V, (B, bag), generator=gen)
    ids[:40] = torch.randint(0, 50, (40, bag), generator=gen)
    ids[0, :3] = pad
    ids = ids.to(DEV)
    table = torch.randn(V, D, device=DEV)
    dout = torch.randn(B, D, device=DEV)
    g1 = torch.zeros(V, D, device=DEV)
    s = _seg(kind=_hip.RS_SEG_POOL, dim=D, out_col=0, vocab=V, idx_stride=bag, bag=bag,
             pool_mode=_hip.RS_POOL['mean'], idx=ids.data_ptr(), table=table.data_ptr(), pad_idx=pad)
    s.grad = g1.data_ptr()
    ops.gather_bwd([s], B, dout)
    keys, vals = _sort(ids, V)
    g2 = _segsum(keys, vals, B * bag, bag, 1, pad, dout, V, D)
    assert torch.allclose(g1, g2, atol=1e-6, rtol=1e-5)


def _sorted_rows(keys):
    k = keys.cpu().numpy().view(np.uint32)
    return sorted(set(int(x) for x in k if x != SENT))


def _gather_pair(ids_d, D, V, pad, table, lazy=None, lazy_last=None):
    """The call's rows gathered two ways: mean bags of 3 and one id per row (rs_gather_fwd, or
    rs_gather_fwd_lazy reading through the catch-up when `lazy` is given)."""
    rows = ids_d.shape[0]
    outs = []
    for kind in (_hip.RS_SEG_POOL, _hip.RS_SEG_SPARSE):
        s = _hip.FeatureSeg()
        s.kind, s.dim, s.out_col, s.vocab, s.pad_idx, s.table = kind, D, 0, V, pad, table.data_ptr()
        if kind == _hip.RS_SEG_POOL:
            s.pool_mode, s.bag, s.idx_stride, s.idx, n = _hip.RS_POOL['mean'], 3, 3, ids_d.data_ptr(), rows
        else:
            s.idx_stride, s.idx, n = 1, ids_d.data_ptr(), rows * 3
        if lazy_last is not None:
            s.lazy_last = lazy_last.data_ptr()
        out = torch.full((n, D), 7.0, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        ops.gather_fwd([s], n, out, err, lazy=lazy)
        outs.append(out)
    return outs


@pytest.mark.parametrize('catch', ['sorted', 'ids', 'read'])
@pytest.mark.parametrize('D,wd,clip,calls', [(40, 0.0, False, 1), (128, 0.0, True, 1), (16, 0.0, False, 1),
                                             (64, 0.01, True, 1), (32, 0.0, True, 2), (6, 0.01, False, 2)])
def test_lazy_adam_bitwise_equals_dense(D, wd, clip, calls, catch):
    """Forward catch-up either over the sorted keys (rs_sorted_catchup), straight from the id
    matrix (rs_lookup_catchup: one compare-and-swap per row picks the replaying lookup), or read
    through inside the gather (rs_gather_fwd_lazy: nothing written; the gathered bags and rows
    equal the dense weights' bitwise, and the optimizer step's replay stores the same state)."""
    V, pad, steps, cap = 3000, 7, 9, 64
    gen = torch.Generator().manual_seed(D + calls)
    p0 = torch.randn(V, D, generator=gen).to(DEV)
    pd, md, vd = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    pl, ml, vl = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    gl = torch.zeros_like(p0)
    last = torch.zeros(V, 2, dtype=torch.int32, device=DEV)  # (moments' step, parameters' step)
    owner = torch.full((V,), 0x7fffffff, dtype=torch.int32, device=DEV)
    step_d = torch.zeros((), dtype=torch.int64, device=DEV)
    step_l = torch.zeros((), dtype=torch.int64, device=DEV)
    consts = torch.zeros(cap, 2, device=DEV)
    consts.view(torch.int32)[0, 0] = cap
    coef = torch.tensor(0.37, device=DEV) if clip else None
    cptr = coef.data_ptr() if clip else None
    S = ops.stream()
    hyper = (B1, B2, EPS, wd)
    for t in range(1, steps + 1):
        # this step's lookups (calls x [rows, 3] ids with repeats, the padding id and
        # out-of-range ids); step 4 touches nothing at all (rows must still replay step 4 later)
        sorted_calls, rows = [], set()
        for c in range(calls):
            n_ids = 0 if t == 4 else 300
            ids = torch.randint(0, V // (1 if t % 2 else 6), (300,), generator=gen)
            ids[:5] = pad
            ids[5] = V + 3
            ids = ids[:n_ids].view(-1, 3)
            if n_ids == 0:
                continue
            ids_d = ids.to(DEV)
            keys, _ = _sort(ids_d, V)
            sorted_calls.append(keys)
            if catch == 'read':
                lz = ((ml.data_ptr() - pl.data_ptr()) // 4, (vl.data_ptr() - pl.data_ptr()) // 4, step_l.data_ptr(),
                      consts.data_ptr(), *hyper)
                got = _gather_pair(ids_d, D, V, pad, pl, lazy=lz, lazy_last=last)
                want = _gather_pair(ids_d, D, V, pad, pd)
                assert all(torch.equal(a, b) for a, b in zip(got, want)), t
            elif catch == 'sorted':
                _hip.call('rs_sorted_catchup', keys.data_ptr(), ids.numel(), D, pl.data_ptr(), ml.data_ptr(),
                          vl.data_ptr(), last.data_ptr(), step_l.data_ptr(), consts.data_ptr(), *hyper, S)
            else:
                _hip.call('rs_lookup_catchup', ids_d.data_ptr(), 8, ids.shape[0], 3, 3, V, D, pl.data_ptr(),
                          ml.data_ptr(), vl.data_ptr(), last.data_ptr(), step_l.data_ptr(), consts.data_ptr(),
                          *hyper, S)
            rows |= set(_sorted_rows(keys))
        rows = sorted(rows)
        # what the forward reads: touched rows (pad included) equal the dense weights exactly
        r = torch.tensor(rows, device=DEV) if rows else None
        if rows and catch != 'read':
            assert torch.equal(pl[r], pd[r]), t
        # gradient of the touched rows except the pad row (what the segment sum leaves)
        g = torch.zeros(V, D)
        grows = [x for x in rows if x != pad]
        if grows:
            g[grows] = torch.randn(len(grows), D, generator=gen)
        g = g.to(DEV)
        gl.copy_(g)
        _hip.call('rs_counter_add', step_d.data_ptr(), 1, S)
        _hip.call('rs_adam_step', pd.data_ptr(), g.data_ptr(), md.data_ptr(), vd.data_ptr(), V * D, LR,
                  B1, B2, EPS, wd, 0, step_d.data_ptr(), 0.5, cptr, 0, S)
        _hip.call('rs_adam_prepare', step_l.data_ptr(), consts.data_ptr(), cap, LR, B1, B2, S)
        multi = len(sorted_calls) > 1
        if multi:
            for i, keys in enumerate(sorted_calls):
                _hip.call('rs_sorted_owner', keys.data_ptr(), keys.numel(), owner.data_ptr(), i, S)
        for i, keys in enumerate(sorted_calls):
            _hip.call('rs_sorted_adam', keys.data_ptr(), keys.numel(), D, pl.data_ptr(), gl.data_ptr(),
                      ml.data_ptr(), vl.data_ptr(), last.data_ptr(), owner.data_ptr() if multi else None,
                      i, step_l.data_ptr(), consts.data_ptr(), *hyper, 0.5, cptr, S)
        assert not gl.any().item()  # stepped gradient rows re-zeroed
        assert int(owner.min().item()) == 0x7fffffff  # owners reset by the step
        if rows:  # every touched row stepped exactly once
            assert torch.equal(pl[r], pd[r]), t
    assert step_l.item() == steps
    _hip.call('rs_sparse_flush', pl.data_ptr(), ml.data_ptr(), vl.data_ptr(), last.data_ptr(), V, D,
              step_l.data_ptr(), consts.data_ptr(), *hyper, S)
    assert torch.equal(pl, pd)
    assert torch.equal(ml, md)
    assert torch.equal(vl, vd)
    assert int(last.min().item()) == steps


def test_consts_overflow_clamped():
    """Past the constants capacity (graph replays skip the host check) the step index is clamped
    on the device and the overflow flag set."""
    cap = 4
    consts = torch.zeros(cap, 2, device=DEV)
    consts.view(torch.int32)[0, 0] = cap
    step = torch.zeros((), dtype=torch.int64, device=DEV)
    for _ in range(cap + 2):
        _hip.call('rs_adam_prepare', step.data_ptr(), consts.data_ptr(), cap, LR, B1, B2, ops.stream())
    assert int(consts.view(torch.int32)[0, 1].item()) == 1
    V, D = 10, 8
    p = torch.randn(V, D, device=DEV)
    m, v = torch.ones_like(p), torch.ones_like(p)
    last = torch.zeros(V, 2, dtype=torch.int32, device=DEV)  # (moments' step, parameters' step)
    _hip.call('rs_sparse_flush', p.data_ptr(), m.data_ptr(), v.data_ptr(), last.data_ptr(), V, D,
              step.data_ptr(), consts.data_ptr(), B1, B2, EPS, 0.0, ops.stream())
    assert int(last.max().item()) == cap - 1


def test_sorted_sqnorm_matches_dense():
    V, D = 5000, 64
    g = torch.zeros(V, D, device=DEV)
    rows = torch.randperm(V)[:700]
    g[rows.to(DEV)] = torch.randn(700, D, device=DEV)
    ids = torch.cat([rows, rows[:100]]).to(DEV)  # repeats: each row counted once
    keys, _ = _sort(ids.view(-1, 1), V)
    ns = int(_hip.lib().rs_sorted_sqnorm_parts())
    ws = torch.zeros(ns, dtype=torch.float64, device=DEV)
    _hip.call('rs_sorted_sqnorm', keys.data_ptr(), ids.numel(), D, g.data_ptr(), None, 0, 2.0,
              ws.data_ptr(), ops.stream())
    norm, coef = torch.zeros((), device=DEV), torch.zeros((), device=DEV)
    _hip.call('rs_clip_coef', ws.data_ptr(), ns, 1.0, norm.data_ptr(), coef.data_ptr(), ops.stream())
    want = (2.0 * g.double()).norm().item()
    assert abs(norm.item() - want) < 1e-6 * want


def test_pack_ids_and_rows():
    g = np.random.default_rng(2)
    m = torch.from_numpy(g.integers(0, 1 << 30, size=(300, 9))).to(DEV)
    out = torch.empty(300 * 4, dtype=torch.int32, device=DEV)
    _hip.call('rs_pack_ids', m.data_ptr() + 8 * 2, 8, 300, 4, 9, out.data_ptr(), ops.stream())
    assert torch.equal(out.view(300, 4).long(), m[:, 2:6])
    x = torch.randn(300, 50, device=DEV)
    y = torch.empty(300, 16, device=DEV)
    _hip.call('rs_pack_rows', x.data_ptr() + 4 * 7, 50, 300, 16, y.data_ptr(), ops.stream())
    assert torch.equal(y, x[:, 7:23])


def test_sorted_catchup_batch_bitwise():
    """rs_sorted_catchup_batch (round 6: a gather's tables caught up in one launch) against one
    rs_sorted_catchup per call: two tables of different widths in one row class (D = 128, 100)
    and a third call on the first table in a second launch, rows several steps stale -- the same
    parameters, moments and `last` bit for bit."""
    V, cap, pad = 5000, 64, 3
    gen = torch.Generator().manual_seed(11)
    S = ops.stream()
    hyper = (B1, B2, EPS, 0.0)
    step = torch.zeros((), dtype=torch.int64, device=DEV)
    consts = torch.zeros(cap, 2, device=DEV)
    consts.view(torch.int32)[0, 0] = cap
    for _ in range(6):
        _hip.call('rs_adam_prepare', step.data_ptr(), consts.data_ptr(), cap, LR, B1, B2, S)
    state = {}
    for name, D in (('a', 128), ('b', 100)):
        p = torch.randn(V, D, generator=gen).to(DEV)
        m = (0.01 * torch.randn(V, D, generator=gen)).to(DEV)
        v = (0.001 * torch.rand(V, D, generator=gen)).to(DEV)
        last = torch.randint(0, 5, (V, 1), generator=gen, dtype=torch.int32).repeat(1, 2).to(DEV)
        state[name] = (D, p, m, v, last)
    calls = []
    for name in ('a', 'b', 'a'):
        ids = torch.randint(0, V, (700,), generator=gen)
        ids[:4] = pad
        keys, _ = _sort(ids.to(DEV), V)
        calls.append((name, keys, ids.numel()))
    copies = {k: (D, p.clone(), m.clone(), v.clone(), last.clone()) for k, (D, p, m, v, last) in state.items()}
    for name, keys, n in calls:  # one launch per call
        D, p, m, v, last = copies[name]
        _hip.call('rs_sorted_catchup', keys.data_ptr(), n, D, p.data_ptr(), m.data_ptr(), v.data_ptr(),
                  last.data_ptr(), step.data_ptr(), consts.data_ptr(), *hyper, S)

    def launch(group):
        arr = (_hip.SortedCall * len(group))()
        for j, (name, keys, n) in enumerate(group):
            D, p, m, v, last = state[name]
            sc = arr[j]
            sc.keys, sc.n, sc.D, sc.call = keys.data_ptr(), n, D, 0
            sc.p, sc.g, sc.m, sc.v, sc.last, sc.owner = p.data_ptr(), None, m.data_ptr(), v.data_ptr(), \
                last.data_ptr(), None
        import ctypes
        _hip.call('rs_sorted_catchup_batch', ctypes.addressof(arr), len(group), step.data_ptr(),
                  consts.data_ptr(), *hyper, S)
    launch(calls[:2])   # tables a and b together
    launch(calls[2:])   # a's second call after
    torch.cuda.synchronize()
    for name in state:
        for x, y in zip(state[name][1:], copies[name][1:]):
            assert torch.equal(x, y), name
    assert int(state['a'][4][:, 1].max().item()) == 6
