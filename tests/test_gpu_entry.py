"""The train_twotower.py entry (recommendsystemproject_amd/train_twotower.py; reference
train_twotower.py:17-218): the same config / metadata_config schema and pickled tables, two
epochs on the device loaders, Recall@K validation, early stopping bookkeeping and the
reference's checkpoint dict (keys, state_dict keys, a torch.optim.Adam-layout optimizer state).
The tables are synthetic DataFrames this test writes itself."""
import os

import numpy as np
import pytest
import torch
import yaml

from test_device_loader import CFG, make_df

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _write_inputs(tmp_path, epochs=2, patience=8, lr=None, n_train=640):
    cfg = yaml.safe_load(yaml.safe_dump(CFG))
    cfg['train'].update({'batch_size': 64, 'epochs': epochs, 'patience': patience})
    if lr is not None:
        cfg['train']['learning_rate'] = lr
    for t in cfg['two_tower'].values():
        t['dropout'] = 0.1
    ut = cfg['two_tower']['user_tower']  # make_df draws histories of up to 25 items
    ut['max_seq_len'] = ut['transformer_parameters']['max_seq_len'] = 32
    meta = {'two_tower': {'user_tower': {'sparse_features': [{'name': 'user_id_enc', 'embedding_dim': 1}],
                                         'metadata_fields': ['user_id_enc']},
                          'item_tower': {'sparse_features': [{'name': 'movie_id_enc', 'embedding_dim': 1}],
                                         'metadata_fields': ['movie_id_enc']}},
            'train': {'batch_size': 64}}
    paths = {k: str(tmp_path / f'{k}.yaml') for k in ('config', 'meta')}
    yaml.safe_dump(cfg, open(paths['config'], 'w'))
    yaml.safe_dump(meta, open(paths['meta'], 'w'))
    train, val = make_df(n_train, seed=1), make_df(192, seed=2)
    # a 60-item catalog (Recall@50 needs >= 50) that every interaction's item belongs to: Recall@10
    # of an untrained model is ~ 10 / 60, so epoch 1 always beats the initial 0 and checkpoints
    rng = np.random.default_rng(4)
    for df in (train, val):
        df['movie_id_enc'] = rng.integers(1, 61, len(df))
    items = make_df(60, seed=3)
    items['movie_id_enc'] = np.arange(1, 61)
    item_cols = ['movie_id_enc', 'genre_ids', 'release_year_enc']
    for name, df in (('train', train), ('val', val), ('items', items[item_cols])):
        paths[name] = str(tmp_path / f'{name}.pkl')
        df.to_pickle(paths[name])  # this test's own files
    return cfg, paths


def test_train_twotower_two_epochs_and_checkpoint(tmp_path):
    from recommendsystemproject_amd.train_twotower import main
    cfg, p = _write_inputs(tmp_path)
    torch.manual_seed(0)
    model, best = main(p['config'], p['train'], p['val'], p['items'], p['meta'],
                       checkpoint_dir=str(tmp_path / 'ckpt'), device=torch.device('cuda:0'))
    # epoch 1's Recall@10 beats the initial 0 (60 items, 192 validation rows: ~0.17 by chance), so
    # at least one checkpoint is always written
    assert 0.0 < best <= 1.0
    ckpts = sorted((tmp_path / 'ckpt').glob('best_model_epoch_*.pt'))
    assert ckpts and ckpts[0].name == 'best_model_epoch_1.pt'
    for c in ckpts:
        ck = torch.load(c, weights_only=True)
        assert set(ck) == {'epoch', 'model_state_dict', 'optimizer_state_dict', 'train_loss', 'val_loss',
                           'metrics', 'user_mapping', 'item_mapping', 'config'}
        assert list(ck['model_state_dict']) == list(model.state_dict())
        assert set(ck['metrics']) == {10, 20, 50}
        assert np.isfinite(ck['train_loss']) and np.isfinite(ck['val_loss'])
        opt = ck['optimizer_state_dict']
        assert set(opt) == {'state', 'param_groups'}
        n_params = len(list(model.parameters()))
        assert len(opt['state']) == n_params
        st = opt['state'][0]
        assert set(st) >= {'step', 'exp_avg', 'exp_avg_sq'}
        assert ck['config']['train']['epochs'] == cfg['train']['epochs']


def test_train_twotower_lazy_tables(tmp_path, monkeypatch):
    """Every lookup table as a lazy-Adam table: the checkpoint holds flushed (current) rows."""
    monkeypatch.setenv('RSYS_LAZY_ROWS', '1')
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.train_twotower import main
    _, p = _write_inputs(tmp_path, epochs=1)
    torch.manual_seed(0)
    model, best = main(p['config'], p['train'], p['val'], p['items'], p['meta'],
                       checkpoint_dir=str(tmp_path / 'ckpt'), device=torch.device('cuda:0'))
    assert best > 0  # validation reads the lazily updated rows (caught up on lookup)
    f = ensure_flat(model)
    assert len(f.lazy) >= 3
    sd = model.state_dict()  # flushes
    for t in f.lazy:
        assert int(t.last.min().item()) == int(t.last.max().item())
    assert all(torch.isfinite(v).all() for v in sd.values() if v.is_floating_point())


def test_optimizer_state_round_trip(tmp_path, monkeypatch):
    """Adam.state_dict -> torch.save -> torch.load -> Adam.load_state_dict resumes exactly: the
    next step from the loaded state equals the next step of the original run (lazy tables
    included)."""
    monkeypatch.setenv('RSYS_LAZY_ROWS', '1')
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.optim import Adam
    from recommendsystemproject_amd.project.utils.training_utils import train_step
    from test_gpu_errors import _batches, _model
    dev = torch.device('cuda:0')
    m1, cfg = _model()
    o1 = Adam(m1.parameters(), lr=1e-3)
    b = _batches(cfg, 4)
    for x in b[:3]:
        train_step(m1, x, o1, 1.0, 0.15)
    torch.save({'m': m1.state_dict(), 'o': o1.state_dict()}, tmp_path / 'ck.pt')
    ck = torch.load(tmp_path / 'ck.pt', weights_only=True)
    m2, _ = _model(seed=5)
    m2.load_state_dict(ck['m'])
    o2 = Adam(m2.parameters(), lr=1e-3)
    ensure_flat(m2)
    o2.load_state_dict(ck['o'])
    l1 = train_step(m1, b[3], o1, 1.0, 0.15).item()
    l2 = train_step(m2, b[3], o2, 1.0, 0.15).item()
    assert l1 == l2
    d = (ensure_flat(m1).data - ensure_flat(m2).data).abs().max().item()
    assert d < 1e-6, d


def test_train_twotower_early_stopping(tmp_path, capsys):
    """Recall@10 early stopping with patience 1 (reference train_twotower.py:174-204): with a zero
    learning rate the model cannot improve on epoch 1, so the loop stops at the first epoch that
    does not beat the best (long before the configured 6 epochs) and the only checkpoint is epoch
    1's."""
    from recommendsystemproject_amd.train_twotower import main
    _, p = _write_inputs(tmp_path, epochs=6, patience=1, lr=0.0)
    torch.manual_seed(0)
    _, best = main(p['config'], p['train'], p['val'], p['items'], p['meta'],
                   checkpoint_dir=str(tmp_path / 'ckpt'), device=torch.device('cuda:0'))
    out = capsys.readouterr().out
    assert best > 0
    assert 'Early stopping triggered after' in out, out[-2000:]
    stopped = int(out.split('Early stopping triggered after ')[1].split()[0])
    assert stopped < 6
    names = [c.name for c in (tmp_path / 'ckpt').glob('best_model_epoch_*.pt')]
    assert 'best_model_epoch_1.pt' in names and len(names) <= stopped - 1


def _entry_worker(rank, world, port, tmp, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK='0', RSYS_DIST_BACKEND='gloo', RSYS_LAZY_ROWS='1')
        from recommendsystemproject_amd.train_twotower import main
        import torch.distributed as dist
        p = {k: os.path.join(tmp, v) for k, v in (('config', 'config.yaml'), ('meta', 'meta.yaml'),
                                                  ('train', 'train.pkl'), ('val', 'val.pkl'),
                                                  ('items', 'items.pkl'))}
        torch.manual_seed(100 + rank)  # different on purpose: main() must agree the ranks itself
        model, best = main(p['config'], p['train'], p['val'], p['items'], p['meta'],
                           checkpoint_dir=os.path.join(tmp, 'ckpt'), device=torch.device('cuda:0'))
        from recommendsystemproject_amd.flat import ensure_flat
        f = ensure_flat(model)
        f.flush()
        w = f.data[:f.replicated_numel].detach().clone()
        ws = [torch.empty_like(w) for _ in range(world)]
        dist.all_gather(ws, w)
        bufs = torch.cat([b.detach().double().reshape(-1) for b in model.buffers() if b.numel()])
        bs = [torch.empty_like(bufs) for _ in range(world)]
        dist.all_gather(bs, bufs)
        q.put((rank, best, bool(torch.equal(ws[0], ws[1])), bool(torch.equal(bs[0], bs[1]))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, 'err', repr(e), traceback.format_exc()[-2000:]))


def test_train_twotower_two_ranks_one_gpu(tmp_path):
    """The epoch loop under data parallelism (2 ranks on cuda:0, gloo; every table lazy): the
    ranks start from different torch seeds, so main() must agree the epoch order and the model
    (sync_seed, broadcast), validate the same model (rank 0's BatchNorm running statistics) and
    take rank 0's early-stopping / checkpoint decisions -- no rank may hang in a collective
    another rank skipped. The dataset size is not a multiple of the global batch (drop_last)."""
    import multiprocessing as mp
    import socket
    _write_inputs(tmp_path, epochs=2, n_train=750)  # 11 full batches of 64 + 46 rows: 12, even
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=280) for _ in range(2)], key=lambda r: r[0])
    for pr in procs:
        pr.join(timeout=60)
    assert all(r[1] != 'err' for r in res), res
    assert res[0][1] == res[1][1] and res[0][1] > 0, res      # one decision, made on rank 0's recall
    assert all(r[2] and r[3] for r in res), res                # same weights and buffers everywhere
    assert list((tmp_path / 'ckpt').glob('best_model_epoch_*.pt'))
