"""The benched workloads end to end on the GPU (BASELINE.json configs[1], [2], [4]):

* logits of the HIP path against the reference's golden logits (fp32, 1e-4; collision mask
  exact);
* the benched bf16 compute mode against every golden fixture and against the fp32 oracle at the
  C2 (B = 1024, L = 50), C3-capped (B = 1024) and C5-capped (B = 256, L = 200, N = 10) shapes,
  where every bf16 path engages (streaming GEMMs, fused FFN, short and long bf16 attention, bf16
  qkv storage, the bf16 tower chain, the fused CE with and without hard negatives);
* the fp32 step against the oracle at the configured batch B = 4096 (C2);
* C3 at its real sizes (1M / 10M / 10M-row tables, pooled 50-long history, lazy-exact Adam over
  sorted lookups) for several steps with distinct batches against a dense-Adam HIP control, and
  the C3 schema with the tables capped to 1M rows against the oracle;
* C5 (L = 200 encoder, N = 10 hard negatives materialised from a device catalog, grouped per-slot
  BatchNorm, bf16 long-history attention) at its real 100M-row size, and capped against the
  oracle (fp32) and against a dense-Adam control.

bf16 bounds (all derived, none fitted). Every GEMM operand the bf16 mode rounds carries a relative
error of at most u = 2^-8. Embeddings: elementwise within TOL_EMB = 4u (unit vectors). Logits:
|dS_ij| <= (|dU_i| + |dI_j| + |dU_i||dI_j| + 2u(1 + |dU_i|)(1 + |dI_j|)) / T elementwise, from the
measured embedding errors by Cauchy-Schwarz (_logit_bound). Loss: the mean over rows of twice the
row's largest logit bound (a row loss is 1-Lipschitz in the max-norm of its logits, once more for
the label logit). Bias: rounding noise is unbiased, so the mean of the per-row loss differences
must sit within 4 standard errors of zero. Gradients: per tensor, a relative error within
4u sqrt(depth) plus the ReLU-decision term and a regression slope on the oracle's gradient within
its derived band (tests/bf16_check.py; tools/bf16_grad_stats.py prints the measured values).
"""
import os

import numpy as np
import pytest
import torch
import yaml

import bf16_check as bc
import golden_util as gu
from oracle.twotower_oracle import OracleTrainer, model_forward, model_state_shapes, inbatch_logits
from recommendsystemproject_amd import precision, synth
from recommendsystemproject_amd.flat import ensure_flat
from recommendsystemproject_amd.optim import Adam
from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
from recommendsystemproject_amd.project.utils.training_utils import extract_item_id, train_step

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = gu.training_fixtures(os.path.join(ROOT, 'tests', 'golden'))
DEV = torch.device('cuda:0')
U_BF16 = 2.0 ** -8
TOL_EMB = 4 * U_BF16


def cfg_of(name, dropout0=True):
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', f'{name}.yaml')))
    if dropout0:
        for t in cfg['two_tower'].values():
            t['dropout'] = 0.0
            if 'transformer_parameters' in t:
                t['transformer_parameters']['dropout'] = 0.0
    return cfg


def maps_of(cfg):
    return {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}


def build(cfg, state=None, on_device=False):
    maps = maps_of(cfg)
    if on_device:
        torch.manual_seed(0)
        with torch.device(DEV):
            m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                              maps['user'], maps['item'])
    else:
        m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                          maps['user'], maps['item'])
    if state is not None:
        m.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state.items()})
    return m.to(DEV), maps


def cap_vocab(cfg, cap):
    for t in cfg['two_tower'].values():
        for f in (t.get('sparse_features') or []) + (t.get('sequence_features') or []):
            f['vocab_size'] = min(int(f['vocab_size']), cap)
    return cfg


@pytest.fixture
def bf16():
    precision.set_compute_dtype('bf16')
    yield
    precision.set_compute_dtype('fp32')


# ---------------------------------------------------------------------------------- logits
@pytest.mark.parametrize('path', GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_logits_match_golden(path):
    cfg, meta, data = gu.load(path)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    model, _ = build(cfg, synth.make_state(shapes, seed=meta['weight_seed']))
    model.train()
    tb = synth.batch_to_torch(gu.batches(meta, data)[0], DEV)
    U, I, H = model(tb)
    logits = model.compute_logits(U, I, extract_item_id(tb['item_tower']), H, meta['temperature'])
    want = data['logits']
    got = logits.cpu().numpy()
    assert got.shape == want.shape
    masked = want <= -1e8
    assert np.array_equal(got <= -1e8, masked)          # the collision mask, exactly
    assert np.array_equal(got[masked], want[masked])    # -1e9
    np.testing.assert_allclose(got[~masked], want[~masked], rtol=0, atol=1e-4)


# ---------------------------------------------------------------------------------- bf16 mode
def _logit_bound(h, f, T):
    """|dS_ij| <= (|dU_i| + |dI_j| + |dU_i| |dI_j| + 2u (1 + |dU_i|)(1 + |dI_j|)) / T elementwise
    (Cauchy-Schwarz on unit vectors, with the measured embedding errors; 2u: the similarity's
    own rounded operands). Hard-negative columns likewise with |dH_in|."""
    nU = (h['U'] - f['U']).double().norm(dim=1)
    nI = (h['I'] - f['I']).double().norm(dim=1)
    cols = [nI[None, :].expand(nU.shape[0], -1)]
    if f['H'] is not None:
        cols.append((h['H'] - f['H']).double().norm(dim=2))
    nC = torch.cat(cols, dim=1)
    nR = nU[:, None]
    return (nR + nC + nR * nC + 2 * U_BF16 * (1 + nR) * (1 + nC)) / T


def _assert_bf16_vs_oracle(r, cfg, T):
    """The bf16 step against the fp32 oracle: embeddings elementwise within TOL_EMB, every logit
    within its derived bound, the loss within the mean of the rows' bounds (a row loss is
    1-Lipschitz in the max-norm of its logits, twice for the label logit), the per-row loss
    differences unbiased (4 standard errors), and every gradient tensor within
    bf16_check.check_grads' derived bounds (relative error and regression slope)."""
    h, f = r['hip'], r['ref']
    for k in ('U', 'I', 'H'):
        if f[k] is not None:
            err = (h[k] - f[k]).abs().max().item()
            assert err <= TOL_EMB, (k, err)
    bound = _logit_bound(h, f, T)
    ok = f['logits'] > -1e8
    assert torch.equal(h['logits'] > -1e8, ok)  # the collision mask, exactly
    dl = (h['logits'] - f['logits']).abs()
    assert bool((dl[ok] <= bound[ok]).all()), (dl[ok].max().item(), (dl - bound)[ok].max().item())
    row_bound = 2 * torch.where(ok, bound, torch.zeros_like(bound)).max(dim=1).values
    assert abs(h['loss'] - f['loss']) <= row_bound.mean().item(), (h['loss'], f['loss'], row_bound.mean().item())
    d = bc.row_losses(h['logits']) - bc.row_losses(f['logits'])
    se = d.std().item() / np.sqrt(d.numel())
    assert abs(d.mean().item()) <= 4 * se + 1e-5, (d.mean().item(), se)
    bad = bc.check_grads(h['grads'], f['grads'], cfg, f['kappa'], batch=h['U'].shape[0])
    assert not bad, bad


@pytest.mark.parametrize('path', GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_bf16_step_matches_golden(path, bf16):
    """Every golden fixture's first step in the bf16 compute mode: U, I, H and the logits against
    the reference's own (golden) values, the gradients against the oracle's (itself pinned to the
    same fixtures by tests/test_oracle_golden.py)."""
    cfg, meta, data = gu.load(path)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    T = meta['temperature']
    b0 = gu.batches(meta, data)[0]
    r = bc.bf16_vs_oracle(cfg, len(b0['item_tower']['sparse']), DEV, 0,
                          state=synth.make_state(shapes, seed=meta['weight_seed']), batch=b0, T=T)
    for name in ('U', 'I', 'H'):
        if name in data:
            err = np.abs(r['hip'][name].numpy() - data[name]).max()
            assert err <= TOL_EMB, (name, err)
    want = data['logits']
    ok = want > -1e8
    bound = _logit_bound(r['hip'], r['ref'], T).numpy()
    assert np.all(np.abs(r['hip']['logits'].numpy() - want)[ok] <= bound[ok])
    assert abs(r['hip']['loss'] - float(data['loss1'])) <= 2 * bound.max(axis=1).mean()
    _assert_bf16_vs_oracle(r, cfg, T)


def test_bf16_c2_step_matches_oracle(bf16):
    """C2 shapes with every bf16 path engaged (B * L = 51,200 token rows: bf16 streaming GEMMs,
    fused FFN, bf16 attention and qkv storage, fused CE) against the fp32 oracle."""
    cfg = cfg_of('c2')
    _assert_bf16_vs_oracle(bc.bf16_vs_oracle(cfg, 1024, DEV, 21), cfg, float(cfg['train']['temperature']))


def test_bf16_c3_capped_matches_oracle(bf16):
    """The C3 schema in the benched precision (bf16 tower chain on 128-wide tables, pooled-mean
    50-long history, fused bf16 in-batch CE), the large tables capped to 1M rows (still lazy-Adam
    tables), B = 1024, against the fp32 oracle."""
    cfg = cap_vocab(cfg_of('c3'), 1_000_000)
    _assert_bf16_vs_oracle(bc.bf16_vs_oracle(cfg, 1024, DEV, 71), cfg, float(cfg['train']['temperature']))


def test_bf16_c5_capped_matches_oracle(bf16):
    """The C5 schema in the benched precision: L = 200 history through the bf16 long-history
    attention (B * L = 51,200 tokens: bf16 qkv storage too), N = 10 hard negatives from a device
    catalog in the fused bf16 CE, grouped per-slot BatchNorm; tables capped to 1M rows, B = 256,
    against the fp32 oracle (N separate item-tower passes there)."""
    from recommendsystemproject_amd import ops
    cfg = cap_vocab(cfg_of('c5'), 1_000_000)
    B, L = 256, 200
    assert ops.qkv_bf16_ok(L, 64, 4, B * L)  # the benched storage and kernels engage at this size
    _assert_bf16_vs_oracle(bc.bf16_vs_oracle(cfg, B, DEV, 81, n_neg=10), cfg, float(cfg['train']['temperature']))


def test_fp32_c2_configured_batch_matches_oracle():
    """The configured batch (B = 4096, L = 50) in the parity precision: loss, embeddings and the
    updated weights after one step against the oracle."""
    B = 4096
    cfg = cfg_of('c2')
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=31)
    model, maps = build(cfg, state)
    opt = Adam(model.parameters(), lr=float(cfg['train']['learning_rate']))
    ref = OracleTrainer(cfg, state, lr=float(cfg['train']['learning_rate']))
    T = float(cfg['train']['temperature'])
    b = synth.make_batch(cfg, B, seed=32, edge_cases=True)
    got = train_step(model, synth.batch_to_torch(b, DEV), opt, 1.0, T).item()
    want = float(ref.step(synth.batch_to_torch(b), maps, temperature=T))
    assert abs(got - want) < 1e-4, (got, want)
    sd = model.state_dict()
    for k in ('user_tower.seq_encoder.transformer_backbone.layers.1.linear1.weight',
              'user_tower.seq_encoder.feature_embedder.feature_projection.0.weight',
              'user_tower.mlp.mlp.0.weight', 'item_tower.mlp.mlp.8.weight',
              'item_tower.embeddings.movie_id_enc.weight'):
        err = (sd[k].cpu() - ref.S[k].detach()).abs().max().item()
        assert err < 1e-4, (k, err)


# ---------------------------------------------------------------------------------- C3
def _c3_steps(cfg, model, batches, T):
    opt = Adam(model.parameters(), lr=float(cfg['train']['learning_rate']))
    return [train_step(model, synth.batch_to_torch(b, DEV), opt, 1.0, T).item() for b in batches]


@pytest.fixture
def deterministic():
    """torch.use_deterministic_algorithms(True): every table gradient through a fixed-order kernel
    (slot-image / ranged LDS images, sorted segment sums for the large ones, lazy or not:
    functions._sorted_ordinary), so two runs that compute the same sums agree bitwise."""
    from recommendsystemproject_amd import ops
    torch.use_deterministic_algorithms(True, warn_only=True)
    ops.sync_deterministic()
    yield
    torch.use_deterministic_algorithms(False)
    ops.sync_deterministic()


def test_c3_real_tables_lazy_matches_dense_adam(monkeypatch, deterministic):
    """C3 at its real sizes: lazy-exact Adam over sorted lookups (1M / 10M / 10M rows) against
    the same model trained with dense Adam over every row, 5 steps of distinct batches, in
    deterministic mode: the table gradients are the same fixed-order sums in both runs, so the
    losses and the tables agree bitwise (up to 1e-6 where the clip coefficient's last bit may
    differ: the dense run's norm sums 2.69B squares, the lazy one only the touched rows')."""
    cfg = cfg_of('c3')
    T = float(cfg['train']['temperature'])
    batches = [synth.make_batch(cfg, 4096, seed=300 + s) for s in range(5)]
    monkeypatch.setenv('RSYS_LAZY_ROWS', '65536')
    lazy, _ = build(cfg, on_device=True)
    assert len(ensure_flat(lazy).lazy) == 3
    init = {k: v.detach().clone() for k, v in lazy.state_dict().items() if 'embeddings' in k and v.dim() == 2
            and v.shape[0] >= 1_000_000}
    l_lazy = _c3_steps(cfg, lazy, batches, T)
    monkeypatch.setenv('RSYS_LAZY_ROWS', '0')
    dense, _ = build(cfg, on_device=True)
    with torch.no_grad():
        dense.load_state_dict({k: v for k, v in init.items()}, strict=False)
    assert not ensure_flat(dense).lazy
    l_dense = _c3_steps(cfg, dense, batches, T)
    np.testing.assert_allclose(l_lazy, l_dense, rtol=0, atol=1e-6)
    sl, sd = lazy.state_dict(), dense.state_dict()  # lazy: flushed to the current step
    for k, w0 in init.items():
        a, b = sl[k], sd[k]
        d = (a - b).abs()
        assert d.max().item() <= 1e-6, (k, d.max().item(), int((d > 0).sum()))
        # rows no batch looked up moved by neither (their Adam state is zero)
        rows = torch.randint(0, a.shape[0], (4096,), device=DEV)
        touched = torch.zeros(a.shape[0], dtype=torch.bool, device=DEV)
        for bt in batches:
            for t in (synth.batch_to_torch(bt, DEV)['user_tower'], synth.batch_to_torch(bt, DEV)['item_tower']):
                for x in [t.get('sparse')] + list((t.get('sequence') or {}).values()):
                    if x is not None:
                        ids = x.reshape(-1)
                        touched[ids[(ids >= 0) & (ids < a.shape[0])]] = True
        cold = rows[~touched[rows]]
        assert torch.equal(a[cold], w0[cold]) and torch.equal(b[cold], w0[cold])


def test_eval_lookups_catch_up_in_id_order(monkeypatch):
    """A forward without a backward (validation) brings its rows current straight from the ids
    (rs_lookup_catchup, no sort) and records no call for the optimizer; its output equals the
    output after a full flush of the lazy state (every row brought current by rs_sparse_flush)."""
    cfg = cap_vocab(cfg_of('c3'), 200_000)
    monkeypatch.setenv('RSYS_LAZY_ROWS', '65536')
    model, _ = build(cfg, on_device=True)
    f = ensure_flat(model)
    assert f.lazy
    T = float(cfg['train']['temperature'])
    batches = [synth.make_batch(cfg, 1024, seed=500 + s) for s in range(4)]
    _c3_steps(cfg, model, batches[:3], T)
    model.eval()
    b = synth.batch_to_torch(batches[3], DEV)
    with torch.no_grad():
        u1, i1, _ = model(b)
    assert all(not t.calls for t in f.lazy)
    f.flush()
    with torch.no_grad():
        u2, i2, _ = model(b)
    assert torch.equal(u1, u2) and torch.equal(i1, i2)


def _assert_adam_close(name, diff, lr, steps, tol=1e-4):
    """Weights after `steps` Adam steps within tol of the oracle's. Adam's normalised step of an
    element whose gradient is ~0 is set by fp32 rounding noise (either implementation may land
    anywhere in +-lr per step), so a few isolated elements may differ by up to 2 lr per step; a
    wrong gradient moves many elements."""
    d = diff.abs()
    off = int((d > tol).sum())
    assert off == 0 or (off <= 16 and d.max().item() <= 2 * lr * steps * 1.01), \
        (name, d.max().item(), off)


def test_c3_capped_matches_oracle():
    """The C3 schema (pooled-mean 50-long history as a sparse feature, 128-wide tables) with the
    large tables capped to 1M rows -- still lazy-Adam tables -- against the oracle."""
    cfg = cap_vocab(cfg_of('c3'), 1_000_000)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=41)
    model, maps = build(cfg, state)
    assert len(ensure_flat(model).lazy) == 3
    opt = Adam(model.parameters(), lr=1e-3)
    ref = OracleTrainer(cfg, state, lr=1e-3)
    for s in range(2):
        b = synth.make_batch(cfg, 256, seed=42 + s, edge_cases=True)
        got = train_step(model, synth.batch_to_torch(b, DEV), opt, 1.0, 0.15).item()
        want = float(ref.step(synth.batch_to_torch(b), maps, temperature=0.15))
        assert abs(got - want) < 1e-4, (s, got, want)
    sd = model.state_dict()
    for k in ('user_tower.embeddings.hist_item_ids.weight', 'item_tower.embeddings.item_id_enc.weight',
              'user_tower.mlp.mlp.0.weight', 'item_tower.mlp.mlp.4.weight'):
        _assert_adam_close(k, sd[k].cpu() - ref.S[k].detach(), lr=1e-3, steps=2)


def _clone_batch(b):
    if isinstance(b, torch.Tensor):
        return b.clone()
    return {k: _clone_batch(v) for k, v in b.items()} if isinstance(b, dict) else b


def _copy_batch(dst, src):
    if isinstance(src, torch.Tensor):
        dst.copy_(src)
    elif isinstance(src, dict):
        for k, v in src.items():
            _copy_batch(dst[k], v)


@pytest.mark.parametrize('mode', ['high', '1'])
def test_c3_capped_user_tower_own_stream_captured(monkeypatch, mode):
    """The user tower on a stream of its own (RSYS_USER_STREAM: 'high' = the highest priority),
    the item tower on the side stream: two eager steps, then the whole step (forward, backward,
    clip, lazy Adam) captured into one hipGraph and replayed on two new batches -- every loss
    against the oracle's. Round 4's core dump of this mode was a fork of a fork inside the capture
    (the user tower's per-table lookup stream forked from its own side stream): side streams no
    longer fork (streams.py)."""
    monkeypatch.setenv('RSYS_USER_STREAM', mode)
    cfg = cap_vocab(cfg_of('c3'), 1_000_000)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=43)
    model, maps = build(cfg, state)
    assert len(ensure_flat(model).lazy) == 3
    opt = Adam(model.parameters(), lr=1e-3)
    ref = OracleTrainer(cfg, state, lr=1e-3)
    raw = [synth.make_batch(cfg, 256, seed=60 + s, edge_cases=True) for s in range(4)]
    dev = [synth.batch_to_torch(b, DEV) for b in raw]
    got, want = [], []
    for s in range(2):
        got.append(train_step(model, dev[s], opt, 1.0, 0.15).item())
        want.append(float(ref.step(synth.batch_to_torch(raw[s]), maps, temperature=0.15)))
    assert model._rs_user_stream is not None
    slot = _clone_batch(dev[1])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode='thread_local'):
        loss_static = train_step(model, slot, opt, 1.0, 0.15)
    for s in (2, 3):
        _copy_batch(slot, dev[s])
        g.replay()
        got.append(loss_static.item())
        want.append(float(ref.step(synth.batch_to_torch(raw[s]), maps, temperature=0.15)))
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-4)
    sd = model.state_dict()
    for k in ('user_tower.embeddings.hist_item_ids.weight', 'item_tower.mlp.mlp.4.weight'):
        _assert_adam_close(k, sd[k].cpu() - ref.S[k].detach(), lr=1e-3, steps=4)


# ---------------------------------------------------------------------------------- C5
def _catalog(cfg, seed=7):
    from recommendsystemproject_amd.project.utils.hard_negatives import ItemCatalog
    item = cfg['two_tower']['item_tower']
    V = int(item['sparse_features'][0]['vocab_size'])
    g = torch.Generator(device=DEV).manual_seed(seed)
    cols = [f for f in item['sparse_features'] if 'pooling' not in f]
    sparse = torch.stack([torch.arange(V, device=DEV, dtype=torch.int32) if i == 0 else
                          torch.randint(1, int(f['vocab_size']), (V,), device=DEV, generator=g, dtype=torch.int32)
                          for i, f in enumerate(cols)], 1)
    seqc = {f['name']: torch.randint(0, int(f['vocab_size']), (V, 3), device=DEV, generator=g, dtype=torch.int32)
            for f in item['sparse_features'] if 'pooling' in f}
    return ItemCatalog(sparse=sparse, sequence=seqc, device=DEV), V


def _c5_step(model, opt, cfg, b, catalog, neg):
    tb = synth.batch_to_torch(b, DEV)
    tb['hard_negatives'] = catalog.materialize(neg)
    return train_step(model, tb, opt, 1.0, float(cfg['train']['temperature'])).item()


def test_c5_real_size_bf16_steps(bf16):
    """C5 at its real size (100M-row history and item tables, L = 200, N = 10 hard negatives from
    a device catalog, grouped per-slot BatchNorm, bf16 long-history attention): 3 steps of
    distinct batches run, the loss is finite, and after a flush every row the steps looked up
    is at the current optimizer step."""
    cfg = cfg_of('c5', dropout0=False)
    model, _ = build(cfg, on_device=True)
    f = ensure_flat(model)
    assert len(f.lazy) == 2 and all(t.V == 100_000_000 for t in f.lazy)
    opt = Adam(model.parameters(), lr=float(cfg['train']['learning_rate']))
    catalog, V = _catalog(cfg)
    g = torch.Generator(device=DEV).manual_seed(3)
    losses = []
    looked = []
    for s in range(3):
        b = synth.make_batch(cfg, 4096, seed=500 + s)
        neg = torch.randint(1, V, (4096, 10), device=DEV, generator=g)
        losses.append(_c5_step(model, opt, cfg, b, catalog, neg))
        looked.append(torch.as_tensor(b['item_tower']['sparse'][:, 0]))
    assert all(np.isfinite(losses)), losses
    model.check_errors()
    f.flush()
    steps = int(opt._flat_state[id(f)]['step_dev'].item())
    assert steps == 3
    item_table = model.item_tower.embeddings['item_id_enc'].weight
    t = next(t for t in f.lazy if t.param is item_table)
    rows = torch.cat(looked).to(DEV)
    assert int(t.last[rows].min().item()) == steps
    assert int(t.last.max().item()) == steps


def test_c5_capped_matches_oracle():
    """The C5 schema (L = 200 encoder with hist_genre_ids tag pooling, N = 10 hard negatives) with
    the tables capped to 1M rows (lazy tables), fp32, against the oracle (N separate item-tower
    passes there, one grouped pass here)."""
    cfg = cap_vocab(cfg_of('c5'), 1_000_000)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=51)
    model, maps = build(cfg, state)
    assert len(ensure_flat(model).lazy) == 2
    opt = Adam(model.parameters(), lr=1e-3)
    ref = OracleTrainer(cfg, state, lr=1e-3)
    catalog, V = _catalog(cfg)
    cat_sparse = catalog.sparse.long().cpu()
    cat_seq = {k: v.long().cpu() for k, v in catalog.sequence.items()}
    g = torch.Generator().manual_seed(4)
    for s in range(2):
        b = synth.make_batch(cfg, 64, seed=52 + s, edge_cases=True)
        neg = torch.randint(1, V, (64, 10), generator=g)
        got = _c5_step(model, opt, cfg, b, catalog, neg.to(DEV))
        rb = synth.batch_to_torch(b)
        rb['hard_negatives'] = [{'sparse': cat_sparse[neg[:, n]],
                                 'sequence': {k: v[neg[:, n]] for k, v in cat_seq.items()}}
                                for n in range(10)]
        want = float(ref.step(rb, maps, temperature=float(cfg['train']['temperature'])))
        assert abs(got - want) < 1e-4, (s, got, want)
    sd = model.state_dict()
    for k in ('user_tower.seq_encoder.feature_embedder.embeddings.hist_item_ids.weight',
              'item_tower.embeddings.item_id_enc.weight', 'item_tower.mlp.mlp.0.weight'):
        _assert_adam_close(k, sd[k].cpu() - ref.S[k].detach(), lr=1e-3, steps=2)


@pytest.mark.timeout(600)
def test_c5_configured_batch_matches_oracle():
    """C5 at its configured batch in the parity precision: B = 4096, L = 200, N = 10 hard
    negatives from a device catalog, fp32, the tables capped to 10M rows (the bench's CPU leg runs
    the oracle at exactly this size; 100M rows with the oracle's dense Adam state exceed the box's
    host memory). One step: the loss within 1e-4 of the oracle's and three updated weight tensors
    (the history table, the item-id table, the item tower's first Linear)."""
    cfg = cap_vocab(cfg_of('c5'), 10_000_000)
    B, N = 4096, 10
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=55)
    model, maps = build(cfg, state)
    assert len(ensure_flat(model).lazy) == 2
    lr = float(cfg['train']['learning_rate'])
    opt = Adam(model.parameters(), lr=lr)
    catalog, V = _catalog(cfg)
    g = torch.Generator().manual_seed(5)
    b = synth.make_batch(cfg, B, seed=56, edge_cases=True)
    assert b['user_tower']['sequence']['hist_item_ids'].shape[1] == 200
    neg = torch.randint(1, V, (B, N), generator=g)
    got = _c5_step(model, opt, cfg, b, catalog, neg.to(DEV))
    torch.cuda.synchronize()
    cat_sparse = catalog.sparse[neg.to(DEV).reshape(-1)].long().cpu().reshape(B, N, -1)
    cat_seq = {k: v[neg.to(DEV).reshape(-1)].long().cpu().reshape(B, N, -1) for k, v in catalog.sequence.items()}
    sd = {k: v.cpu() for k, v in model.state_dict().items()
          if k in ('user_tower.seq_encoder.feature_embedder.embeddings.hist_item_ids.weight',
                   'item_tower.embeddings.item_id_enc.weight', 'item_tower.mlp.mlp.0.weight')}
    del model, opt, catalog
    ref = OracleTrainer(cfg, state, lr=lr)
    del state
    rb = synth.batch_to_torch(b)
    rb['hard_negatives'] = [{'sparse': cat_sparse[:, n], 'sequence': {k: v[:, n] for k, v in cat_seq.items()}}
                            for n in range(N)]
    want = float(ref.step(rb, maps, temperature=float(cfg['train']['temperature'])))
    assert abs(got - want) < 1e-4, (got, want)
    for k, w in sd.items():
        _assert_adam_close(k, w - ref.S[k].detach(), lr=lr, steps=1)
