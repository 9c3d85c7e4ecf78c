"""The final encoder layer on the selected rows only (functions.layer_fwd_last / layer_bwd_last,
csrc/attn_rows.hip). SequenceEncoder returns context[b, clamp(sum(valid) - 1, 0)]
(SequenceEncoder.py:58-74, T7), so the last layer's other rows are dead: the pruned layer must
give the same encoder output, loss and gradients as the full layer (RSYS_FULL_LAST_LAYER=1).
The golden-fixture parity tests (test_gpu_parity.py) run the pruned path against the reference.
"""
import os

import numpy as np
import pytest
import torch
import yaml

import golden_util as gu
from recommendsystemproject_amd import ops, precision

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).to(DEV)


def _mask(B, L, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    lens[0] = 0  # an all-padding row: T6 unmasks the last key, T7 selects position 0
    if B > 1:
        lens[1] = L
    seq = (torch.arange(L)[None, :] < lens[:, None]).long().to(DEV)
    return ops.seq_mask(seq, 0)


@pytest.mark.parametrize('L,d,H,p', [(50, 64, 4, 0.0), (50, 64, 4, 0.1), (7, 32, 4, 0.0),
                                     (1, 64, 4, 0.0), (200, 64, 4, 0.1), (33, 64, 2, 0.0),
                                     (50, 64, 1, 0.1), (70, 64, 8, 0.1)])
def test_attn_rows_matches_full_fp32(L, d, H, p):
    B = 37
    qkv = rnd(B * L, 3 * d, seed=1)
    key_pad, last = _mask(B, L, 2)
    key = torch.tensor([11, 4], dtype=torch.int64, device=DEV)
    out, lse = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 6)
    outs, lses = ops.attn_rows_fwd(qkv, key_pad, last, B, L, d, H, p, key, 6)
    sel = torch.arange(B, device=DEV) * L + last
    torch.testing.assert_close(outs, out[sel], atol=2e-6, rtol=1e-5)
    lse_full = lse.view(B, H, L)[torch.arange(B, device=DEV), :, last].reshape(B * H)
    torch.testing.assert_close(lses, lse_full, atol=1e-5, rtol=1e-5)
    dsel = rnd(B, d, seed=3)
    dfull = torch.zeros(B * L, d, device=DEV)
    dfull[sel] = dsel
    g_full = ops.attn_bwd(qkv, key_pad, out, dfull, lse, B, L, d, H, p, key, 6)
    g_rows = ops.attn_rows_bwd(qkv, key_pad, last, dsel, lses, B, L, d, H, p, key, 6)
    sc = g_full.abs().max().item()
    assert (g_rows - g_full).abs().max().item() < 2e-5 * sc
    # dQ is exactly zero off the selected rows
    qpart = g_rows.view(B, L, 3, d)[:, :, 0]
    keep = torch.zeros(B, L, dtype=torch.bool, device=DEV)
    keep[torch.arange(B, device=DEV), last] = True
    assert torch.count_nonzero(qpart[~keep]) == 0


@pytest.mark.parametrize('p', [0.0, 0.1])
def test_attn_rows_matches_full_bf16(p):
    B, L, d, H = 64, 50, 64, 4
    precision.set_compute_dtype('bf16')
    try:
        qkv = rnd(B * L, 3 * d, seed=5).to(torch.bfloat16)
        key_pad, last = _mask(B, L, 6)
        key = torch.tensor([3, 8], dtype=torch.int64, device=DEV)
        out, lse = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 6)
        outs, lses = ops.attn_rows_fwd(qkv, key_pad, last, B, L, d, H, p, key, 6)
        sel = torch.arange(B, device=DEV) * L + last
        ref = out[sel]
        sc = ref.abs().max().item()
        assert (outs - ref).abs().max().item() < 5e-3 * sc
        assert (outs - ref).abs().mean().item() < 2e-4 * sc
        dsel = rnd(B, d, seed=7)
        dfull = torch.zeros(B * L, d, device=DEV)
        dfull[sel] = dsel
        g_full = ops.attn_bwd(qkv, key_pad, out, dfull, lse, B, L, d, H, p, key, 6).float()
        g_rows = ops.attn_rows_bwd(qkv, key_pad, last, dsel, lses, B, L, d, H, p, key, 6)
        assert g_rows.dtype == torch.bfloat16
        g_rows = g_rows.float()
        sc = g_full.abs().max().item()
        assert (g_rows - g_full).abs().max().item() < 2e-2 * sc
        assert (g_rows - g_full).abs().mean().item() < 5e-4 * sc
    finally:
        precision.set_compute_dtype('fp32')


def test_attn_rows_bad_args():
    qkv = rnd(3 * 300, 192)
    key_pad = torch.zeros(3, 300, dtype=torch.uint8, device=DEV)
    last = torch.zeros(3, dtype=torch.int64, device=DEV)
    with pytest.raises(RuntimeError):  # L > 256
        ops.attn_rows_fwd(qkv, key_pad, last, 3, 300, 64, 4)


def _step(cfg, state, batch, full_last, monkeypatch, dtype):
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
    from recommendsystemproject_amd.project.utils.training_utils import extract_item_id
    if full_last:
        monkeypatch.setenv('RSYS_FULL_LAST_LAYER', '1')
    else:
        monkeypatch.delenv('RSYS_FULL_LAST_LAYER', raising=False)
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    precision.set_compute_dtype(dtype)
    try:
        m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                          maps['user'], maps['item'])
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
        m = m.to(DEV)
        f = ensure_flat(m)
        f.zero_grad()
        U, I, H = m(batch)
        loss = m.compute_loss(U, I, item_ids=extract_item_id(batch['item_tower']), temperature=0.15)
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), U.detach().clone(), {k: p.grad.clone() for k, p in m.named_parameters()}
    finally:
        precision.set_compute_dtype('fp32')


@pytest.mark.parametrize('dtype,B', [('fp32', 256), ('bf16', 1024), ('fp32', 37)])
def test_pruned_last_layer_step(dtype, B, monkeypatch):
    """A whole training step (forward, loss, backward) with the pruned final layer against the
    full final layer: same user embeddings, loss and every gradient (summation order aside)."""
    from oracle.twotower_oracle import model_state_shapes
    from recommendsystemproject_amd import synth
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c2.yaml')))
    for t in cfg['two_tower'].values():
        t['dropout'] = 0.0
        t.get('transformer_parameters', {})['dropout'] = 0.0
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=3)
    batch = synth.batch_to_torch(synth.make_batch(cfg, B, seed=9, edge_cases=True), DEV)
    l1, U1, g1 = _step(cfg, state, batch, False, monkeypatch, dtype)
    l2, U2, g2 = _step(cfg, state, batch, True, monkeypatch, dtype)
    skip = gu.bn_invariant_keys(cfg)  # exact gradient 0: fp32 noise only, compared elsewhere
    if dtype == 'fp32':
        assert abs(l1 - l2) <= 1e-5 * max(1.0, abs(l2)), (l1, l2)
        assert (U1 - U2).abs().max().item() <= 1e-5
        for k in g1:
            if k in skip:
                continue
            sc = max(g2[k].abs().max().item(), 1e-12)
            err = (g1[k] - g2[k]).abs().max().item()
            assert err <= 2e-4 * sc, (k, err, sc)
    else:
        # bf16 mode: the pruned layer's B-row out-projection has no bf16-MFMA instance and runs in
        # fp32, so the two paths differ at bf16 rounding level (as fused vs unfused FFN do)
        cos = torch.nn.functional.cosine_similarity
        assert abs(l1 - l2) <= 2e-3 * abs(l2), (l1, l2)
        assert cos(U1.flatten(), U2.flatten(), dim=0).item() > 0.9999
        a = torch.cat([g1[k].flatten() for k in g1 if k not in skip])
        b = torch.cat([g2[k].flatten() for k in g2 if k not in skip])
        assert cos(a, b, dim=0).item() > 0.999
        for k in g1:
            if k not in skip and g2[k].norm() > 1e-3 * b.norm():
                cs = cos(g1[k].flatten(), g2[k].flatten(), dim=0).item()
                assert cs > 0.99, (k, cs)


@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
def test_deferred_reductions_bitwise(dtype, monkeypatch):
    """The encoder backward's parameter-gradient reductions queued and run as one launch
    (ops.deferred_reduce, rs_reduce_flush) against the immediate per-call reduce launches, in
    deterministic mode: every gradient bitwise equal (the jobs keep each reduce's order)."""
    from oracle.twotower_oracle import model_state_shapes
    from recommendsystemproject_amd import ops, synth
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c2.yaml')))
    for t in cfg['two_tower'].values():  # the dropout keys advance per step
        t['dropout'] = 0.0
        t.get('transformer_parameters', {})['dropout'] = 0.0
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=5)
    batch = synth.batch_to_torch(synth.make_batch(cfg, 512, seed=11, edge_cases=True), DEV)
    torch.use_deterministic_algorithms(True)
    try:
        monkeypatch.setenv('RSYS_DEFER_REDUCE', '1')
        l1, U1, g1 = _step(cfg, state, batch, False, monkeypatch, dtype)
        monkeypatch.setenv('RSYS_DEFER_REDUCE', '0')
        l2, U2, g2 = _step(cfg, state, batch, False, monkeypatch, dtype)
    finally:
        torch.use_deterministic_algorithms(False)
        ops.sync_deterministic()
    assert l1 == l2 and torch.equal(U1, U2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
