"""GPU parity: the HIP training step against the reference's golden fixtures and the oracle.

Bar (BASELINE.json north_star): loss / embeddings within 1e-4 fp32, index lookup bit-exact.
"""
import glob
import os

import numpy as np
import pytest
import torch
import yaml

import golden_util as gu
from oracle.twotower_oracle import OracleTrainer, model_state_shapes
from recommendsystemproject_amd import synth
from recommendsystemproject_amd.optim import Adam
from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
from recommendsystemproject_amd.project.utils.training_utils import extract_item_id, train_step

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = gu.training_fixtures(os.path.join(ROOT, 'tests', 'golden'))
DEV = torch.device('cuda:0')


def build(cfg, state):
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'), maps['user'], maps['item'])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    return m.to(DEV), maps


def zero_dropout(cfg):
    for t in cfg['two_tower'].values():
        t['dropout'] = 0.0
        if 'transformer_parameters' in t:
            t['transformer_parameters']['dropout'] = 0.0
    return cfg


@pytest.mark.parametrize('lazy', [False, True, 'read'], ids=['dense_adam', 'lazy_adam', 'lazy_read_through'])
@pytest.mark.parametrize('path', GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_training_step_matches_reference_golden(path, lazy, monkeypatch):
    """lazy: every lookup table trained by lazy-exact Adam (flat.py), which must reproduce the
    reference's dense-gradient torch.optim.Adam (trap T16) to the same tolerance; 'read': with the
    forward's catch-up read through inside the gather (rs_gather_fwd_lazy)."""
    if lazy:
        monkeypatch.setenv('RSYS_LAZY_ROWS', '1')
    if lazy == 'read':
        monkeypatch.setenv('RSYS_READ_THROUGH', '1')
    cfg, meta, data = gu.load(path)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=meta['weight_seed'])
    model, _ = build(cfg, state)
    opt = Adam(model.parameters(), lr=meta['lr'])
    if lazy:
        from recommendsystemproject_amd.flat import ensure_flat
        assert len(ensure_flat(model).lazy) >= 3
    T = meta['temperature']
    errs, losses = [], []
    for s, b in enumerate(gu.batches(meta, data)):
        tb = synth.batch_to_torch(b, DEV)
        if s == 0:
            model.train()
            opt.zero_grad()
            U, I, H = model(tb)
            loss = model.compute_loss(U, I, item_ids=extract_item_id(tb['item_tower']), hard_neg_emb=H,
                                      temperature=T)
            loss.backward()
            torch.cuda.synchronize()
            for name, t in (('U', U), ('I', I), ('H', H)):
                if name in data:
                    errs.append(gu.check(name, ('full', data[name]), t.detach().cpu().numpy(), rtol=1e-4, atol=1e-5))
            assert abs(loss.item() - float(data['loss1'])) < 1e-4, (loss.item(), float(data['loss1']))
            for k, p in model.named_parameters():
                errs.append(gu.check(f'grad:{k}', gu.stored(data, 'grad', k), p.grad.cpu().numpy(),
                                     rtol=2e-4, atol=2e-6))
            opt.step(clip_max_norm=1.0)
            tn = opt._clip.norm.item()
            assert abs(tn - float(data['total_norm1'])) < 2e-4 * float(data['total_norm1'])
            losses.append(loss.item())
        else:
            losses.append(train_step(model, tb, opt, 1.0, T).item())
    np.testing.assert_allclose(losses, data['losses'], rtol=0, atol=1e-4)
    for k, v in model.state_dict().items():
        errs.append(gu.check(f'final:{k}', gu.stored(data, 'final', k), v.double().cpu().numpy(), rtol=0,
                             atol=gu.final_atol(k, cfg, meta) * (1 if k in gu.bn_invariant_keys(cfg) else 2)))
    errs = [e for e in errs if e]
    assert not errs, '\n'.join(errs[:25])


@pytest.mark.parametrize('B,L,edge', [(128, 50, True), (37, 7, True), (64, 1, False)])
def test_c2_shape_step_matches_oracle(B, L, edge):
    """C2 structure (seq_len up to 50) on seeded inputs vs the oracle, 2 steps."""
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c2.yaml')))
    cfg = zero_dropout(cfg)
    cfg['two_tower']['user_tower']['transformer_parameters']['max_seq_len'] = max(L, 1)
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=5)
    model, maps = build(cfg, state)
    opt = Adam(model.parameters(), lr=1e-3)
    ref = OracleTrainer(cfg, state, lr=1e-3)
    for step in range(2):
        b = synth.make_batch(cfg, B, seed=50 + step, edge_cases=edge)
        got = train_step(model, synth.batch_to_torch(b, DEV), opt, 1.0, 0.15).item()
        want = float(ref.step(synth.batch_to_torch(b), maps, temperature=0.15))
        assert abs(got - want) < 1e-4, (step, got, want)
    sd = model.state_dict()
    for k in ('user_tower.seq_encoder.transformer_backbone.layers.0.self_attn.in_proj_weight',
              'user_tower.mlp.mlp.0.weight', 'item_tower.mlp.mlp.8.weight',
              'user_tower.seq_encoder.feature_embedder.pos_emb.weight'):
        err = (sd[k].cpu() - ref.S[k].detach()).abs().max().item()
        assert err < 1e-4, (k, err)


def test_hard_negative_and_no_ids_paths():
    cfg = zero_dropout(yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml'))))
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=9)
    model, maps = build(cfg, state)
    ref = OracleTrainer(cfg, state)
    b = synth.make_batch(cfg, 48, seed=3, n_hard=4, edge_cases=True)
    tb = synth.batch_to_torch(b, DEV)
    U, I, H = model(tb)
    from oracle.twotower_oracle import compute_loss, model_forward
    Ur, Ir, Hr = model_forward(cfg, ref.S, synth.batch_to_torch(b), maps, True, 0.0)
    for item_ids in (None, extract_item_id(tb['item_tower'])):
        got = model.compute_loss(U, I, item_ids=item_ids, hard_neg_emb=H, temperature=0.1).item()
        want = compute_loss(Ur, Ir, None if item_ids is None else item_ids.cpu(), Hr, 0.1).item()
        assert abs(got - want) < 1e-4, (got, want)
