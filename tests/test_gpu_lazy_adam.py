"""Lazy-exact Adam for large tables (csrc/sparse.hip, flat.py; SURVEY.md §7.2 / trap T16).

The reference trains its embeddings with dense gradients and torch.optim.Adam, so every row
moves every step once its exp_avg is non-zero. The lazy path touches only looked-up rows and
replays the skipped zero-gradient steps when a row is next read; these tests require it to be
BITWISE equal to the dense kernel on the same gradients, at every read and after a flush.
"""
import pytest
import torch

from recommendsystemproject_amd import _hip, ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
LR, B1, B2, EPS = 1e-2, 0.9, 0.999, 1e-8


def _i32(n):
    return torch.zeros(n, dtype=torch.int32, device=DEV)


@pytest.mark.parametrize('D,wd,clip', [(40, 0.0, False), (128, 0.0, True), (16, 0.0, False)])
def test_lazy_adam_bitwise_equals_dense(D, wd, clip):
    V, pad, steps, cap = 3000, 7, 9, 64
    gen = torch.Generator().manual_seed(D)
    p0 = torch.randn(V, D, generator=gen).to(DEV)
    pd, md, vd = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    pl, ml, vl = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    gl = torch.zeros_like(p0)
    flag, lst, cnt, last = _i32(V), _i32(V), _i32(1), _i32(V)
    step_d = torch.zeros((), dtype=torch.int64, device=DEV)
    step_l = torch.zeros((), dtype=torch.int64, device=DEV)
    consts = torch.zeros(cap, 2, device=DEV)
    coef = torch.tensor(0.37, device=DEV) if clip else None
    cptr = coef.data_ptr() if clip else None
    S = ops.stream()
    hyper = (B1, B2, EPS, wd)
    for t in range(1, steps + 1):
        # this step's lookups: [rows, bag] ids with repeats, the padding id and out-of-range ids;
        # step 4 touches nothing at all (rows must still replay step 4 later)
        n_ids = 0 if t == 4 else 300
        ids = torch.randint(0, V // (1 if t % 2 else 6), (300,), generator=gen)
        ids[:5] = pad
        ids[5] = V + 3
        ids = ids[:n_ids].view(-1, 3)
        idsd = ids.to(DEV)
        _hip.call('rs_sparse_touch', idsd.data_ptr(), ids.shape[0], 3, 3, V, pad, flag.data_ptr(),
                  lst.data_ptr(), cnt.data_ptr(), S) if n_ids else None
        _hip.call('rs_sparse_catchup', pl.data_ptr(), ml.data_ptr(), vl.data_ptr(), last.data_ptr(),
                  lst.data_ptr(), cnt.data_ptr(), D, step_l.data_ptr(), consts.data_ptr(), *hyper, S)
        # what the forward reads: touched rows equal the dense weights exactly
        rows = sorted({int(i) for i in ids.reshape(-1).tolist() if 0 <= i < V and i != pad})
        if rows:
            r = torch.tensor(rows, device=DEV)
            assert torch.equal(pl[r], pd[r]), t
        # gradient of the touched rows (what the scatter-add would leave)
        g = torch.zeros(V, D)
        if rows:
            g[rows] = torch.randn(len(rows), D, generator=gen)
        g = g.to(DEV)
        gl.copy_(g)
        _hip.call('rs_counter_add', step_d.data_ptr(), 1, S)
        _hip.call('rs_adam_step', pd.data_ptr(), g.data_ptr(), md.data_ptr(), vd.data_ptr(), V * D, LR,
                  B1, B2, EPS, wd, 0, step_d.data_ptr(), 0.5, cptr, 0, S)
        _hip.call('rs_adam_prepare', step_l.data_ptr(), consts.data_ptr(), cap, LR, B1, B2, S)
        _hip.call('rs_sparse_adam', pl.data_ptr(), gl.data_ptr(), ml.data_ptr(), vl.data_ptr(),
                  last.data_ptr(), flag.data_ptr(), lst.data_ptr(), cnt.data_ptr(), D,
                  step_l.data_ptr(), consts.data_ptr(), *hyper, 0.5, cptr, S)
        assert cnt.item() == 0 and int(flag.sum().item()) == 0
        assert not gl.any().item()  # listed gradient rows re-zeroed
    assert step_l.item() == steps
    _hip.call('rs_sparse_flush', pl.data_ptr(), ml.data_ptr(), vl.data_ptr(), last.data_ptr(), V, D,
              step_l.data_ptr(), consts.data_ptr(), *hyper, S)
    assert torch.equal(pl, pd)
    assert torch.equal(ml, md)
    assert torch.equal(vl, vd)
    assert int(last.min().item()) == steps


def test_sparse_sqnorm_matches_dense():
    V, D = 5000, 64
    g = torch.zeros(V, D, device=DEV)
    rows = torch.randperm(V)[:700].to(DEV)
    g[rows] = torch.randn(700, D, device=DEV)
    flag, lst, cnt = _i32(V), _i32(V), _i32(1)
    ids = rows.long()
    _hip.call('rs_sparse_touch', ids.data_ptr(), 700, 1, 1, V, -1, flag.data_ptr(), lst.data_ptr(),
              cnt.data_ptr(), ops.stream())
    ns = int(_hip.lib().rs_sparse_sqnorm_parts())
    ws = torch.zeros(ns, dtype=torch.float64, device=DEV)
    _hip.call('rs_sparse_sqnorm', g.data_ptr(), lst.data_ptr(), cnt.data_ptr(), D, 2.0, ws.data_ptr(),
              ops.stream())
    norm, coef = torch.zeros((), device=DEV), torch.zeros((), device=DEV)
    _hip.call('rs_clip_coef', ws.data_ptr(), ns, 1.0, norm.data_ptr(), coef.data_ptr(), ops.stream())
    want = (2.0 * g.double()).norm().item()
    assert abs(norm.item() - want) < 1e-6 * want


def test_compact_pack_unpack_roundtrip():
    """Row-sparse DP exchange kernels: ordered compaction, pack, rank-ordered unpack-add."""
    V, D, cap = 20000, 24, 512
    gen = torch.Generator().manual_seed(3)
    S = ops.stream()
    gsum = torch.zeros(V, D, device=DEV)
    bufs, union = [], set()
    for r in range(3):  # three "ranks"
        rows = torch.randperm(V, generator=gen)[:300 + 50 * r]
        union |= set(rows.tolist())
        g = torch.zeros(V, D)
        g[rows] = torch.randn(len(rows), D, generator=gen)
        g = g.to(DEV)
        gsum += g
        flag, lst, cnt = _i32(V), _i32(V), _i32(1)
        ids = rows.to(DEV)
        _hip.call('rs_sparse_touch', ids.data_ptr(), len(rows), 1, 1, V, -1, flag.data_ptr(),
                  lst.data_ptr(), cnt.data_ptr(), S)
        buf = torch.empty(cap * (D + 1), device=DEV)
        err = _i32(1)
        _hip.call('rs_sparse_pack', g.data_ptr(), lst.data_ptr(), cnt.data_ptr(), D, cap, buf.data_ptr(),
                  err.data_ptr(), S)
        assert err.item() == 0
        ids_back = buf[:cap].view(torch.int32)
        assert sorted(x for x in ids_back.tolist() if x >= 0) == sorted(rows.tolist())
        bufs.append(buf)
    out = torch.zeros(V, D, device=DEV)
    flag = _i32(V)
    for buf in bufs:
        _hip.call('rs_sparse_unpack_add', out.data_ptr(), flag.data_ptr(), buf.data_ptr(), D, cap, S)
    assert torch.allclose(out, gsum, atol=1e-6)
    lst, cnt = _i32(V), _i32(1)
    ws = torch.empty(int(_hip.lib().rs_sparse_compact_ws_bytes(V)) // 4 + 1, dtype=torch.int32, device=DEV)
    _hip.call('rs_sparse_compact', flag.data_ptr(), V, lst.data_ptr(), cnt.data_ptr(), ws.data_ptr(), S)
    n = cnt.item()
    assert n == len(union)
    assert lst[:n].tolist() == sorted(union)
    # overflow is flagged
    err = _i32(1)
    cnt.fill_(cap + 1)
    _hip.call('rs_sparse_pack', out.data_ptr(), lst.data_ptr(), cnt.data_ptr(), D, cap,
              torch.empty(cap * (D + 1), device=DEV).data_ptr(), err.data_ptr(), S)
    assert err.item() == 2


def test_compact_large_vocab():
    V = 10_000_019
    flag = torch.zeros(V, dtype=torch.int32, device=DEV)
    idx = torch.unique(torch.randint(0, V, (200000,), device=DEV))
    flag[idx] = 1
    lst, cnt = _i32(V), _i32(1)
    ws = torch.empty(int(_hip.lib().rs_sparse_compact_ws_bytes(V)) // 4 + 1, dtype=torch.int32, device=DEV)
    _hip.call('rs_sparse_compact', flag.data_ptr(), V, lst.data_ptr(), cnt.data_ptr(), ws.data_ptr(),
              ops.stream())
    n = cnt.item()
    assert n == idx.numel()
    assert torch.equal(lst[:n].long(), idx)


@pytest.mark.parametrize('kind', ['sparse', 'pool_mean', 'pool_sum'])
def test_scatter_store_for_single_lookup_rows(kind):
    """rs_gather_bwd with touch counts: rows looked up once this step are stored, the others
    atomically added; the table gradient must equal the all-atomic scatter."""
    from recommendsystemproject_amd.functions import _seg
    V, D, B, bag, pad = 200_000, 128, 512, 7, 3
    gen = torch.Generator().manual_seed(11)
    ids = torch.randint(0, V, (B, bag), generator=gen)
    ids[:40] = torch.randint(0, 50, (40, bag), generator=gen)  # heavy repeats
    ids[0, :3] = pad
    ids = ids.to(DEV)
    if kind == 'sparse':
        ids = ids[:, :1].contiguous()
    nb = ids.shape[1]
    table = torch.randn(V, D, device=DEV)
    dout = torch.randn(B, D, device=DEV)
    grads = []
    for use_count in (False, True):
        g = torch.zeros(V, D, device=DEV)
        flag, lst, cnt = _i32(V), _i32(V), _i32(1)
        if kind == 'sparse':
            s = _seg(kind=_hip.RS_SEG_SPARSE, dim=D, out_col=0, vocab=V, idx_stride=1, idx=ids.data_ptr(),
                     table=table.data_ptr(), pad_idx=pad)
        else:
            s = _seg(kind=_hip.RS_SEG_POOL, dim=D, out_col=0, vocab=V, idx_stride=nb, bag=nb,
                     pool_mode=_hip.RS_POOL[kind[5:]], idx=ids.data_ptr(), table=table.data_ptr(), pad_idx=pad)
        s.grad = g.data_ptr()
        if use_count:
            _hip.call('rs_sparse_touch', ids.data_ptr(), B, nb, nb, V, pad, flag.data_ptr(), lst.data_ptr(),
                      cnt.data_ptr(), ops.stream())
            s.touch_count = flag.data_ptr()
            assert int(flag.max().item()) > 1
        ops.gather_bwd([s], B, dout)
        grads.append(g)
    assert torch.allclose(grads[0], grads[1], atol=1e-5, rtol=1e-6)
    assert not grads[1][pad].any()
