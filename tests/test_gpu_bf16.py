"""bf16 compute mode (precision.py; RS_GEMM_BF16): the encoder's streaming GEMMs round their
operands to bf16 and accumulate in fp32. Checked against torch on the SAME bf16-rounded
operands (products are exact in fp32, so only the summation order differs), and the training
step against the fp32 mode. Parity with the reference is run in fp32; these tests
pin what the bf16 mode computes.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F
import yaml

from recommendsystemproject_amd import ops, precision

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).to(DEV)


def r16(t):
    return t.to(torch.bfloat16).float()


@pytest.fixture
def bf16_mode():
    precision.set_compute_dtype('bf16')
    yield
    precision.set_compute_dtype('fp32')


@pytest.mark.parametrize('N,K,kind', [(256, 64, 'fwd_relu'), (192, 64, 'fwd_bias'), (256, 64, 'fwd_plain'),
                                      (64, 256, 'dgrad_beta'), (64, 192, 'dgrad_beta'),
                                      (256, 64, 'dgrad_mask'), (64, 64, 'dgrad')])
def test_bf16_streaming_gemm(N, K, kind, bf16_mode):
    M = 40960
    x = rnd(M, K, seed=1)
    if kind.startswith('fwd'):
        W, b = rnd(N, K, seed=2) * 0.1, rnd(N, seed=3)
        out = ops.linear_fwd(x, W, b if kind != 'fwd_plain' else None, relu=kind == 'fwd_relu')
        ref = r16(x) @ r16(W).t() + (b if kind != 'fwd_plain' else 0)
        if kind == 'fwd_relu':
            ref = torch.relu(ref)
        exact = x @ W.t() + (b if kind != 'fwd_plain' else 0)
    else:
        W = rnd(K, N, seed=2) * 0.1  # linear_bwd_input: out[M, N] = dy[M, K] @ W[K, N]
        base = rnd(M, N, seed=4)
        mask = rnd(M, N, seed=5)
        out = base.clone() if kind == 'dgrad_beta' else None
        out = ops.linear_bwd_input(x, W, out=out, beta=1.0 if kind == 'dgrad_beta' else 0.0,
                                   relu_mask_of=mask if kind == 'dgrad_mask' else None)
        ref = r16(x) @ r16(W)
        exact = x @ W
        if kind == 'dgrad_mask':
            ref, exact = ref * (mask > 0), exact * (mask > 0)
        if kind == 'dgrad_beta':
            ref, exact = ref + base, exact + base
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err < 2e-5 * scale, (err, scale)
    # and it really ran in bf16: visibly different from the fp32 product
    assert (out - exact).abs().max().item() > 20 * err


@pytest.mark.parametrize('K', [64, 256])
def test_bf16_gemm_add_layernorm(K, bf16_mode):
    M, N = 40960, 64
    x, W, b = rnd(M, K, seed=1), rnd(N, K, seed=2) * 0.2, rnd(N, seed=3)
    res, g, be = rnd(M, N, seed=4), 1 + 0.1 * rnd(N, seed=5), 0.1 * rnd(N, seed=6)
    h, y, mu, rs = ops.linear_add_layernorm(x, W, b, res, g, be, 1e-5, 0.0, None, 0)
    href = r16(x) @ r16(W).t() + b + res
    assert torch.allclose(h, href, atol=2e-5 * href.abs().max().item())
    assert torch.allclose(y, F.layer_norm(href, (N,), g, be, 1e-5), atol=1e-4)


def test_bf16_training_step_close_to_fp32():
    """One C2-structure step (B = 256, L = 50, dropout 0) in both modes: the loss agrees to
    bf16 precision and the weight gradients point the same way."""
    from oracle.twotower_oracle import model_state_shapes
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
    from recommendsystemproject_amd.project.utils.training_utils import extract_item_id
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c2.yaml')))
    for t in cfg['two_tower'].values():
        t['dropout'] = 0.0
        t.get('transformer_parameters', {})['dropout'] = 0.0
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=3)
    b = synth.batch_to_torch(synth.make_batch(cfg, 1024, seed=7), DEV)  # B*L = 51,200 >= 32,768
    res = {}
    for mode in ('fp32', 'bf16'):
        precision.set_compute_dtype(mode)
        try:
            m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                              maps['user'], maps['item'])
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
            m = m.to(DEV)
            f = ensure_flat(m)
            f.zero_grad()
            U, I, H = m(b)
            loss = m.compute_loss(U, I, item_ids=extract_item_id(b['item_tower']), temperature=0.15)
            loss.backward()
            res[mode] = (loss.item(), f.grad.clone())
        finally:
            precision.set_compute_dtype('fp32')
    (l32, g32), (l16, g16) = res['fp32'], res['bf16']
    assert abs(l16 - l32) < 1e-2 * abs(l32), (l16, l32)
    assert l16 != l32  # the bf16 path ran
    cos = F.cosine_similarity(g16, g32, dim=0).item()
    assert cos > 0.99, cos
