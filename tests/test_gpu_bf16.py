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
                                      (256, 64, 'dgrad_mask'), (64, 64, 'dgrad'),
                                      (64, 48, 'fwd_plain'), (48, 64, 'dgrad')])
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


@pytest.mark.parametrize('K', [64, 128, 192, 256, 512])
@pytest.mark.parametrize('M', [4096, 40960])
def test_bf16_gemm_add_layernorm(M, K, bf16_mode):
    """Every FFN width the config may set (FFN_dim, GenericTower.py:90): K in {64, 256} takes the
    fused bf16 LayerNorm instances, other widths the GEMM + rs_add_layernorm_fwd -- never an
    unlaunched kernel (round-5 advisor: K = 128 at M = 4096 returned 0 with h / y unwritten)."""
    N = 64
    x, W, b = rnd(M, K, seed=1), rnd(N, K, seed=2) * 0.2, rnd(N, seed=3)
    res, g, be = rnd(M, N, seed=4), 1 + 0.1 * rnd(N, seed=5), 0.1 * rnd(N, seed=6)
    h, y, mu, rs = ops.linear_add_layernorm(x, W, b, res, g, be, 1e-5, 0.0, None, 0)
    h16 = r16(x) @ r16(W).t() + b + res  # the bf16 instances (K in {64, 256}; large-M streaming GEMMs)
    h32 = x @ W.t() + b + res            # the fp32 kernels (small-M unfused shapes)
    tol = 2e-5 * h16.abs().max().item()
    href = h16 if K in (64, 256) or not torch.allclose(h, h32, atol=tol) else h32
    assert torch.allclose(h, href, atol=tol), (h - h16).abs().max().item()
    assert torch.allclose(y, F.layer_norm(href, (N,), g, be, 1e-5), atol=1e-4)


@pytest.mark.parametrize('ffn', [256, 128, 512])
def test_bf16_training_step_close_to_fp32(ffn):
    """One C2-structure step (B = 1024, L = 50, dropout 0) in both modes: the loss agrees to
    bf16 precision and the weight gradients point the same way -- at the configured FFN width and
    at two others (the pruned last layer's B-row LayerNorm GEMM has bf16 instances for K = 64 / 256
    only; the others must take the unfused path, not skip the launch)."""
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
        t.get('transformer_parameters', {})['FFN_dim'] = ffn
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
    assert np.isfinite(l16) and bool(torch.isfinite(g16).all())
    assert abs(l16 - l32) < 1e-2 * abs(l32), (l16, l32)
    assert l16 != l32  # the bf16 path ran
    cos = F.cosine_similarity(g16, g32, dim=0).item()
    assert cos > 0.99, cos


@pytest.mark.parametrize('Mo,No', [(64, 64), (64, 256), (256, 64), (192, 64), (64, 192), (128, 128),
                                   (128, 64), (64, 128), (32, 64), (64, 32), (128, 256), (256, 128),
                                   (64, 96), (96, 64), (60, 72), (256, 192), (256, 172)])
def test_bf16_wgrad(Mo, No, bf16_mode):
    """dW = dY^T X on bf16 MFMA (operands rounded to bf16, fp32 accumulate); the fused bias
    gradient colsum(dY) stays fp32-exact; beta accumulate; ragged row tail; deterministic."""
    M = 40960 + 37
    dy, x = rnd(M, Mo, seed=21), rnd(M, No, seed=22)
    dW, db = rnd(Mo, No, seed=23), rnd(Mo, seed=24)
    ref = dW.double() + r16(dy).double().t() @ r16(x).double()
    refb = db.double() + dy.double().sum(0)
    exact = dW.double() + dy.double().t() @ x.double()
    ops.linear_bwd_weight(dy, x, dW, beta=1.0, db=db)
    err = (dW.double() - ref).abs().max().item()
    assert err < 5e-3, err  # fp32 accumulation over 41k rows of sum ~ 200
    assert (db.double() - refb).abs().max().item() < 2e-3
    assert (dW.double() - exact).abs().max().item() > 5 * err  # the bf16 path ran
    dW2, dW3 = torch.empty_like(dW), torch.empty_like(dW)
    ops.linear_bwd_weight(dy, x, dW2, beta=0.0)
    ops.linear_bwd_weight(dy, x, dW3, beta=0.0)
    assert torch.equal(dW2, dW3)


def _ffn_weights(seed=0):
    W1, b1 = rnd(256, 64, seed=seed + 1) * 0.15, rnd(256, seed=seed + 2) * 0.1
    W2, b2 = rnd(64, 256, seed=seed + 3) * 0.08, rnd(64, seed=seed + 4) * 0.1
    g, be = 1 + 0.1 * rnd(64, seed=seed + 5), 0.1 * rnd(64, seed=seed + 6)
    return W1, b1, W2, b2, g, be


@pytest.mark.parametrize('p', [0.0, 0.15])
def test_fused_ffn_matches_unfused(p, bf16_mode):
    """csrc/ffn.hip against the unfused bf16 path (linear1 -> linear2 + LayerNorm; the dgrad and
    wgrad GEMMs): f1 and dPre1 bit-exact (same operation order), the rest to fp32 summation-order
    tolerance."""
    M = 40960
    x = rnd(M, 64, seed=7)
    W1, b1, W2, b2, g, be = _ffn_weights()
    key = torch.tensor([1234, 5], dtype=torch.int64, device=DEV)
    # forward
    h, y, mu, rs, mask = ops.ffn_fwd_bf16(x, W1, b1, W2, b2, g, be, 1e-5, p, key, 18, 19)
    f1 = ops.linear_fwd(x, W1, b1, relu=True, drop_p=p, drop_key=key, site_a=18)
    hr, yr, mur, rsr = ops.linear_add_layernorm(f1, W2, b2, x, g, be, 1e-5, p, key, 19)
    assert torch.allclose(h, hr, atol=2e-5, rtol=1e-5)
    assert torch.allclose(y, yr, atol=1e-4, rtol=1e-4)
    assert torch.allclose(mu, mur, atol=1e-5) and torch.allclose(rs, rsr, rtol=1e-4)
    bits = ((mask.view(M, 4, 1) >> torch.arange(64, device=DEV).view(1, 1, 64)) & 1).bool()
    # bit 4h+i of word q <-> column 16h + 4q + i
    cols = (16 * torch.arange(16, device=DEV).view(16, 1) + torch.arange(4, device=DEV).view(1, 4))
    cols = cols.reshape(64).view(1, 1, 64) + 4 * torch.arange(4, device=DEV).view(1, 4, 1)
    ref_bits = torch.gather((f1 > 0).view(M, 1, 256).expand(M, 4, 256), 2, cols.expand(M, 4, 64))
    assert torch.equal(bits, ref_bits)
    # backward
    dff, dres = rnd(M, 64, seed=8), rnd(M, 64, seed=9)
    dx, f1b, dpre = ops.ffn_bwd_bf16(x, W1, b1, W2, mask, dff, dres, p)
    # the fused kernel scales by the forward's fp32 1/(1-p) (rng.h make_key)
    scale = float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
    df1 = ops.linear_bwd_input(dff, W2, relu_mask_of=f1, alpha=scale)
    assert torch.equal(f1b, f1.to(torch.bfloat16))
    assert torch.equal(dpre, df1.to(torch.bfloat16))
    dxr = ops.linear_bwd_input(df1, W1, out=dres.clone(), beta=1.0)
    assert torch.allclose(dx, dxr, atol=1e-4, rtol=1e-4)
    # weight gradients from the bf16 operands vs the fp32-operand bf16 wgrad
    dW2, db2 = torch.zeros_like(W2), torch.zeros_like(b2)
    dW1, db1 = torch.zeros_like(W1), torch.zeros_like(b1)
    ops.wgrad_bf16(dff, f1b, dW2, db=db2)
    ops.wgrad_bf16(dpre, x, dW1, db=db1)
    dW2r, db2r = torch.zeros_like(W2), torch.zeros_like(b2)
    dW1r, db1r = torch.zeros_like(W1), torch.zeros_like(b1)
    ops.linear_bwd_weight(dff, f1, dW2r, db=db2r)
    ops.linear_bwd_weight(df1, x, dW1r, db=db1r)
    for a, b_ in ((dW2, dW2r), (db2, db2r), (dW1, dW1r)):
        assert torch.allclose(a, b_, atol=2e-3 * b_.abs().max().item(), rtol=1e-4)
    # db1 sums bf16-rounded dPre1 (autocast semantics): relative error ~ 2^-9
    assert torch.allclose(db1, db1r, atol=1e-2 * db1r.abs().max().item())


@pytest.mark.parametrize('p,M', [(0.0, 40960), (0.15, 40960), (0.15, 4112), (0.0, 16), (0.1, 204800)])
def test_fused_ffn_wgrad(p, M, bf16_mode):
    """rs_ffn_wgrad_bf16 (f1 / dPre1 recomputed on chip) against the split pair it replaces:
    rs_ffn_bwd_bf16 writing f1 / dPre1, then two rs_wgrad_bf16 passes over them. Same bf16
    operands, so the weight gradients agree to fp32 summation order; db2 is the fp32 colsum of
    dff, db1 the colsum of the bf16 dPre1 in both. The backward without the activations gives
    the same dx bits. Deterministic; accumulates into the gradients."""
    x = rnd(M, 64, seed=7)
    W1, b1, W2, b2, g, be = _ffn_weights()
    key = torch.tensor([99, 3], dtype=torch.int64, device=DEV)
    _, _, _, _, mask = ops.ffn_fwd_bf16(x, W1, b1, W2, b2, g, be, 1e-5, p, key, 18, 19)
    dff, dres = rnd(M, 64, seed=8), rnd(M, 64, seed=9)
    dx, f1b, dpre = ops.ffn_bwd_bf16(x, W1, b1, W2, mask, dff, dres, p)
    dx2, f1n, dpn = ops.ffn_bwd_bf16(x, W1, b1, W2, mask, dff, dres, p, acts=False)
    assert f1n is None and dpn is None and torch.equal(dx, dx2)
    init = [rnd(*t.shape, seed=30 + i) for i, t in enumerate((W1, b1, W2, b2))]
    ref = [t.clone() for t in init]
    ops.wgrad_bf16(dff, f1b, ref[2], db=ref[3])
    ops.wgrad_bf16(dpre, x, ref[0], db=ref[1])
    outs = []
    for _ in range(2):
        got = [t.clone() for t in init]
        ops.ffn_wgrad_bf16(x, W1, b1, W2, mask, dff, p, *got)
        outs.append(got)
    for a, b_ in zip(outs[0], outs[1]):
        assert torch.equal(a, b_)
    for name, a, r, i in zip(('dW1', 'db1', 'dW2', 'db2'), outs[0], ref, init):
        sc = (r - i).abs().max().item()
        assert (a - r).abs().max().item() <= 1e-5 * sc + 1e-6, (name, (a - r).abs().max().item(), sc)


@pytest.mark.parametrize('p,M', [(0.0, 40960), (0.1, 40960), (0.1, 4112)])
def test_fused_ffn_ln_backward(p, M, bf16_mode):
    """rs_ffn_bwd_ln_bf16 (the FFN backward with norm1's backward in its epilogue) against the
    rs_ffn_bwd_bf16 + rs_layernorm_bwd pair it replaces: f1 / dPre1 bit-exact, dh1 and dsa to
    fp32 summation order (the row sums run over the columns in another order), the same dropout
    masks (dsa zero exactly where the pair's is), dgamma / dbeta to fixed-order-sum tolerance."""
    x = rnd(M, 64, seed=7)
    W1, b1, W2, b2, g, be = _ffn_weights()
    key = torch.tensor([4321, 6], dtype=torch.int64, device=DEV)
    _, _, _, _, mask = ops.ffn_fwd_bf16(x, W1, b1, W2, b2, g, be, 1e-5, p, key, 18, 19)
    dff, dres = rnd(M, 64, seed=8), rnd(M, 64, seed=9)
    h1 = rnd(M, 64, seed=10) * 2 + 0.3
    g1 = 1 + 0.1 * rnd(64, seed=11)
    mu1 = h1.mean(1)
    rs1 = 1.0 / torch.sqrt(h1.var(1, unbiased=False) + 1e-5)
    dg0, db0 = rnd(64, seed=12), rnd(64, seed=13)
    # reference pair
    dx, f1r, dpr = ops.ffn_bwd_bf16(x, W1, b1, W2, mask, dff, dres, p)
    dgr, dbr = dg0.clone(), db0.clone()
    dar = torch.empty_like(dx) if p > 0 else None
    dhr = ops.layernorm_bwd(h1, dx, g1, mu1, rs1, dgr, dbr, da=dar, p=p, key=key, site=21)
    # fused
    dgf, dbf = dg0.clone(), db0.clone()
    dh1, dsa, f1b, dpre = ops.ffn_bwd_ln_bf16(x, W1, b1, W2, mask, dff, dres, h1, g1, mu1, rs1, dgf, dbf,
                                              p, key, 21)
    assert torch.equal(f1b, f1r) and torch.equal(dpre, dpr)
    sc = dhr.abs().max().item()
    assert (dh1 - dhr).abs().max().item() < 1e-5 * sc
    if p > 0:
        assert torch.equal(dsa == 0, dar == 0)
        assert (dsa - dar).abs().max().item() < 2e-5 * sc
    else:
        assert dsa is None
    for a, b_ in ((dgf, dgr), (dbf, dbr)):
        assert (a - b_).abs().max().item() < 1e-5 * max(1.0, b_.abs().max().item())


@pytest.mark.parametrize('p,M', [(0.0, 40960), (0.1, 40960), (0.1, 4112), (0.15, 16)])
def test_fused_ffn_ln2_backward(p, M, bf16_mode):
    """rs_ffn_bwd_ln2_bf16 (norm2's backward as the prologue of rs_ffn_bwd_ln_bf16) against the
    rs_layernorm_bwd (norm2, with dropout2's backward) + rs_ffn_bwd_ln_bf16 pair it replaces.
    The row sums of norm2's backward run over the columns in another order, so dff, dh1, dsa and
    the four LayerNorm parameter gradients agree to fp32 summation order; dropout masks are the
    same draws (zeros in the same places); the bf16 operand of dff W2 may round differently where
    dff sits on a bf16 rounding boundary, hence the relative bound on dh1."""
    x = rnd(M, 64, seed=7)
    W1, b1, W2, b2, g, be = _ffn_weights()
    key = torch.tensor([4321, 6], dtype=torch.int64, device=DEV)
    h2, _, mu2, rs2, mask = ops.ffn_fwd_bf16(x, W1, b1, W2, b2, g, be, 1e-5, p, key, 18, 19)
    g2 = 1 + 0.1 * rnd(64, seed=14)
    dy2 = rnd(M, 64, seed=8)
    h1 = rnd(M, 64, seed=10) * 2 + 0.3
    g1 = 1 + 0.1 * rnd(64, seed=11)
    mu1 = h1.mean(1)
    rs1 = 1.0 / torch.sqrt(h1.var(1, unbiased=False) + 1e-5)
    init = [rnd(64, seed=20 + i) for i in range(4)]  # dgamma2, dbeta2, dgamma1, dbeta1
    # reference pair
    r = [t.clone() for t in init]
    dffr = torch.empty_like(dy2) if p > 0 else None
    dh2r = ops.layernorm_bwd(h2, dy2.clone(), g2, mu2, rs2, r[0], r[1], da=dffr, p=p, key=key, site=19)
    dffr = dh2r if dffr is None else dffr
    dh1r, dsar, _, _ = ops.ffn_bwd_ln_bf16(x, W1, b1, W2, mask, dffr, dh2r, h1, g1, mu1, rs1, r[2], r[3],
                                           p, key, 17, acts=False)
    # fused
    outs = []
    for _ in range(2):
        f = [t.clone() for t in init]
        dh1, dsa, dff = ops.ffn_bwd_ln2_bf16(x, W1, b1, W2, mask, dy2, h2, g2, mu2, rs2, f[0], f[1], h1, g1,
                                             mu1, rs1, f[2], f[3], p, key, 17, 19)
        outs.append((dh1, dsa, dff, f))
    (dh1, dsa, dff, f), second = outs[0], outs[1]
    assert torch.equal(dh1, second[0]) and torch.equal(dff, second[2])  # deterministic
    assert all(torch.equal(a, b_) for a, b_ in zip(f, second[3]))
    assert torch.equal(dff == 0, dffr == 0)
    assert (dff - dffr).abs().max().item() < 1e-5 * dffr.abs().max().item()
    sc = dh1r.abs().max().item()
    assert (dh1 - dh1r).abs().max().item() < 2e-3 * sc
    assert (dh1 - dh1r).abs().mean().item() < 1e-5 * sc
    if p > 0:
        assert torch.equal(dsa == 0, dsar == 0)
        assert (dsa - dsar).abs().max().item() < 3e-3 * sc
    else:
        assert dsa is None
    for a, b_ in zip(f, r):
        assert (a - b_).abs().max().item() < 2e-3 * max(1.0, b_.abs().max().item())


def test_fused_ffn_bad_args(bf16_mode):
    x = rnd(40, 64)  # M % 16 != 0
    W1, b1, W2, b2, g, be = _ffn_weights()
    with pytest.raises(RuntimeError):
        ops.ffn_fwd_bf16(x, W1, b1, W2, b2, g, be, 1e-5, 0.0, None, 18, 19)


def test_bf16_step_fused_ffn_vs_unfused(monkeypatch):
    """A whole bf16 training step with the fused FFN against the unfused bf16 path."""
    from oracle.twotower_oracle import model_state_shapes
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
    from recommendsystemproject_amd.project.utils.training_utils import extract_item_id
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c2.yaml')))
    for t in cfg['two_tower'].values():  # dropout keys differ per model instance (rng.py)
        t['dropout'] = 0.0
        t.get('transformer_parameters', {})['dropout'] = 0.0
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=3)
    b = synth.batch_to_torch(synth.make_batch(cfg, 1024, seed=7), DEV)
    res = {}
    # the full final layer: both FFN paths then run at B*L rows, where each has its bf16 instance
    # (the pruned layer's B-row unfused FFN would run on the fp32 kernels)
    monkeypatch.setenv('RSYS_FULL_LAST_LAYER', '1')
    precision.set_compute_dtype('bf16')
    try:
        for mode in ('fused', 'unfused'):
            if mode == 'unfused':
                monkeypatch.setenv('RSYS_UNFUSED_FFN', '1')
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
    (l1, g1), (l2, g2) = res['fused'], res['unfused']
    assert abs(l1 - l2) < 1e-4 * abs(l2), (l1, l2)
    assert F.cosine_similarity(g1, g2, dim=0).item() > 0.9999


def _bf16_attention_ref(qkv, key_pad, dout, B, L, d, H):
    """The bf16 MFMA attention's arithmetic in float64: Q, K, V, dO rounded to bf16; the
    unnormalised probabilities and dS rounded to bf16 where they enter a product; softmax,
    dropout-free dS and the scale in full precision. D = sum_j P_ij dP_ij for L <= 64 (the
    per-wave kernels form it from their register tiles); for L > 64 the key-parallel kernels take
    D = dO_i . O_i from the fp32 dO and the forward output, which carries the bf16 rounding of P."""
    hd = d // H
    q, k, v = (r16(t).double() for t in qkv.view(B, L, 3, H, hd).permute(2, 0, 3, 1, 4))
    g = r16(dout).double().view(B, L, H, hd).transpose(1, 2)
    sc = hd ** -0.5
    s = q @ k.transpose(-1, -2)
    mask = key_pad.bool()[:, None, None, :]
    s = s.masked_fill(mask, float('-inf'))
    m = (s * sc).amax(-1, keepdim=True)
    e = torch.exp(s * sc - m).masked_fill(mask, 0.0)
    l = e.sum(-1, keepdim=True)
    out = (r16(e.float()).double() @ v) / l
    P = e / l
    dp = g @ v.transpose(-1, -2)
    o32 = out.transpose(1, 2).reshape(B * L, d).float()
    # D_i = sum_j P_ij dP_ij (== dO_i . O_i in exact arithmetic): the kernel forms it from its
    # register tiles, with dP from the bf16-rounded dO and V
    D = (P * dp).sum(-1, keepdim=True)
    if L > 64:
        D = (dout.double().view(B, L, H, hd).transpose(1, 2) * out).sum(-1, keepdim=True)
    ds = P * (dp - D)
    dsb, Pb = r16(ds.float()).double(), r16(P.float()).double()
    dq = dsb @ k * sc
    dk = dsb.transpose(-1, -2) @ q * sc
    dv = Pb.transpose(-1, -2) @ g
    dqkv = torch.stack([dq, dk, dv], 0).permute(1, 3, 0, 2, 4).reshape(B * L, 3 * d)
    return o32, dqkv.float()


# L > 64: the long-history kernels (one workgroup per (b, h), FlashAttention-2 backward split)
@pytest.mark.parametrize('B,L', [(3, 50), (5, 16), (4, 33), (2, 64), (3, 1), (3, 65), (2, 100), (2, 200),
                                 (2, 256)])
def test_bf16_attention(B, L, bf16_mode):
    d, H = 64, 4
    qkv = rnd(B * L, 3 * d, seed=11)
    lens = torch.randint(1, L + 1, (B,), generator=torch.Generator().manual_seed(L))  # fixed padding
    seq = (torch.arange(L)[None, :] < lens[:, None]).long().to(DEV)
    key_pad, _ = ops.seq_mask(seq, 0)
    dout = rnd(B * L, d, seed=12)
    out, lse = ops.attn_fwd(qkv, key_pad, B, L, d, H)
    dqkv = ops.attn_bwd(qkv, key_pad, out, dout, lse, B, L, d, H)
    ro, rd = _bf16_attention_ref(qkv, key_pad, dout, B, L, d, H)
    # an fp32 value next to a bf16 rounding boundary may round the other way than in float64:
    # single-ulp (2^-8) flips of a probability bound the worst element; the mean stays tight
    # (1.5e-4: with unseeded padding a draw at L = 100 measured 1.04e-4; a wrong product is ~1e-2)
    for a, b_ in ((out, ro), (dqkv, rd)):
        sc = b_.abs().max().item()
        err = (a - b_).abs()
        assert err.max().item() < 5e-3 * sc, (err.max().item(), sc)
        assert err.mean().item() < 1.5e-4 * sc, (err.mean().item(), sc)
    # and it is not the fp32 kernel
    precision.set_compute_dtype('fp32')
    out32, _ = ops.attn_fwd(qkv, key_pad, B, L, d, H)
    precision.set_compute_dtype('bf16')
    if L > 1:
        assert not torch.equal(out, out32)


@pytest.mark.parametrize('L', [50, 120, 201])
def test_bf16_attention_dropout_matches_fp32_masks(L, bf16_mode):
    """Same dropout masks as the fp32 kernels (the draw is per element): results agree to
    bf16 precision, and differ clearly from the no-dropout output."""
    B, d, H, p = 6, 64, 4, 0.2
    qkv = rnd(B * L, 3 * d, seed=13)
    key_pad = torch.zeros(B, L, dtype=torch.uint8, device=DEV)
    key = torch.tensor([77, 3], dtype=torch.int64, device=DEV)
    dout = rnd(B * L, d, seed=14)
    o16, l16 = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 5)
    g16 = ops.attn_bwd(qkv, key_pad, o16, dout, l16, B, L, d, H, p, key, 5)
    precision.set_compute_dtype('fp32')
    o32, l32 = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 5)
    g32 = ops.attn_bwd(qkv, key_pad, o32, dout, l32, B, L, d, H, p, key, 5)
    o0, _ = ops.attn_fwd(qkv, key_pad, B, L, d, H, 0.0)
    precision.set_compute_dtype('bf16')
    scale = o32.abs().max().item()
    assert (o16 - o32).abs().max().item() < 2e-2 * scale
    assert (o0 - o32).abs().max().item() > 0.2 * scale
    assert (g16 - g32).abs().max().item() < 3e-2 * g32.abs().max().item()


@pytest.mark.parametrize('L', [50, 33, 64, 7])
def test_bf16_attention_saved_keep_bits(L, bf16_mode):
    """L <= 64: the forward saves its dropout keep bits in lse's storage tail (ops.attn_fwd) and
    the backward reads them instead of hashing again -- the same draws, so dqkv is bitwise the
    one an lse without the tail (re-drawn) gives; fp32 and bf16 qkv storage, odd and even L."""
    B, d, H, p = 5, 64, 4, 0.3
    lens = torch.randint(1, L + 1, (B,))
    seq = (torch.arange(L)[None, :] < lens[:, None]).long().to(DEV)
    key_pad, _ = ops.seq_mask(seq, 0)
    key = torch.tensor([123, 4], dtype=torch.int64, device=DEV)
    dout = rnd(B * L, d, seed=16)
    q32 = rnd(B * L, 3 * d, seed=15)
    for q in (q32, q32.to(torch.bfloat16)):
        assert ops._zbits_words(B, L, d, H, p, ops._attn_flags(q)) > 0
        o, lse = ops.attn_fwd(q, key_pad, B, L, d, H, p, key, 7)
        assert lse.numel() == B * H * L and lse.untyped_storage().nbytes() > 4 * lse.numel()
        g_bits = ops.attn_bwd(q, key_pad, o, dout, lse, B, L, d, H, p, key, 7)
        g_hash = ops.attn_bwd(q, key_pad, o, dout, lse.clone(), B, L, d, H, p, key, 7)
        assert torch.equal(g_bits, g_hash)
        o2, _ = ops.attn_fwd(q, key_pad, B, L, d, H, p, key, 8)  # another site: other draws
        assert not torch.equal(o, o2)


def _ce_ref(U, I, ids, H, T, gout=1.0):
    """compute_loss (TwoTowerModel.py:81-140) in float64 on bf16-rounded U, I (the fused kernel's
    products); hard-negative logits from the fp32 embeddings as in the kernel."""
    Ud = r16(U).double().requires_grad_(True)
    Id = r16(I).double().requires_grad_(True)
    logits = Ud @ Id.t() / T
    if ids is not None:
        coll = (ids[:, None] == ids[None, :]) & ~torch.eye(len(ids), dtype=torch.bool, device=U.device)
        logits = logits.masked_fill(coll, -1e9)
    Uh = U.double().requires_grad_(True)
    if H is not None:
        Hd = H.double().requires_grad_(True)
        hl = torch.einsum('bd,bnd->bn', Uh, Hd) / T
        logits = torch.cat([logits, hl], 1)
    loss = F.cross_entropy(logits, torch.arange(len(U), device=U.device))
    (loss * gout).backward()
    dU = Ud.grad + (Uh.grad if H is not None else 0)
    return loss.item(), dU.float(), Id.grad.float(), (Hd.grad.float() if H is not None else None)


@pytest.mark.parametrize('B,D,N,coll', [(4096, 128, 0, True), (1000, 128, 3, True), (300, 64, 0, False),
                                        (33, 128, 2, True)])
def test_fused_inbatch_ce(B, D, N, coll, bf16_mode):
    from recommendsystemproject_amd.functions import InBatchLossFn
    U = F.normalize(rnd(B, D, seed=21), dim=1).requires_grad_(True)
    I = F.normalize(rnd(B, D, seed=22), dim=1).requires_grad_(True)
    ids = torch.randint(0, B // 2 if coll else 10 ** 9, (B,), device=DEV) if True else None
    H = F.normalize(rnd(B, N, D, seed=23), dim=2).requires_grad_(True) if N else None
    T = 0.15
    loss = InBatchLossFn.apply(U, I, ids, H, T)
    loss.backward(torch.tensor(0.7, device=DEV))
    l_ref, dU, dI, dH = _ce_ref(U.detach(), I.detach(), ids, H.detach() if N else None, T, 0.7)
    assert abs(loss.item() - l_ref) < 2e-4 * max(1.0, abs(l_ref)), (loss.item(), l_ref)
    for a, b_ in ((U.grad, dU), (I.grad, dI)) + (((H.grad, dH),) if N else ()):
        sc = b_.abs().max().item()
        assert (a - b_).abs().max().item() < 2e-2 * sc, ((a - b_).abs().max().item(), sc)


@pytest.mark.parametrize('B,splits', [(4096, 3), (4096, 5), (2000, 2), (777, 1)])
def test_fused_inbatch_ce_ragged_batches(B, splits, bf16_mode, monkeypatch):
    """Column splits whose tile count is not a multiple of the staged batch (4 tiles forward, 2
    backward), odd batch counts, and a last split shorter than the others."""
    monkeypatch.setenv('RSYS_CE_SPLITS', str(splits))
    test_fused_inbatch_ce(B, 128, 0, True, bf16_mode)


@pytest.mark.parametrize('B,D,splits', [(4096, 128, 0), (4096, 128, 3), (777, 128, 0), (33, 64, 0),
                                        (300, 64, 2)])
def test_fused_ce_forward_rounded_copies(B, D, splits, bf16_mode, monkeypatch):
    """rs_inbatch_ce_fused_fwd_uib's copies of U and I (written by the forward's finish kernel)
    are U, I rounded to bf16, and the backward that streams them gives the bits of the one that
    rounds U, I in its own launch."""
    from recommendsystemproject_amd import _hip
    from recommendsystemproject_amd.functions import InBatchLossFn
    if splits:
        monkeypatch.setenv('RSYS_CE_SPLITS', str(splits))
    U = F.normalize(rnd(B, D, seed=41), dim=1).requires_grad_(True)
    I = F.normalize(rnd(B, D, seed=42), dim=1).requires_grad_(True)
    ids = torch.randint(0, max(B // 2, 1), (B,), device=DEV)
    uib = torch.full((2, B, D), float('nan'), device=DEV, dtype=torch.bfloat16)
    lse, rl = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    loss = torch.empty((), device=DEV)
    w = torch.empty(_hip.lib().rs_inbatch_ce_fused_ws_bytes(B, D) // 4, device=DEV)
    _hip.call('rs_inbatch_ce_fused_fwd_uib', U.data_ptr(), I.data_ptr(), None, 0, 0, ids.data_ptr(), 1, B, 0, D,
              0.15, lse.data_ptr(), rl.data_ptr(), loss.data_ptr(), w.data_ptr(), uib.data_ptr(), None)
    torch.cuda.synchronize()
    assert torch.equal(uib[0], U.detach().bfloat16()) and torch.equal(uib[1], I.detach().bfloat16())
    res = []
    for flag in ('1', '0'):
        monkeypatch.setenv('RSYS_CE_UIB', flag)
        U.grad = I.grad = None
        l_ = InBatchLossFn.apply(U, I, ids, None, 0.15)
        l_.backward()
        res.append((l_.item(), U.grad.clone(), I.grad.clone()))
    assert res[0][0] == res[1][0] == loss.item()
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


def test_fused_ce_deterministic(bf16_mode):
    from recommendsystemproject_amd.functions import InBatchLossFn
    B, D = 4096, 128
    U = F.normalize(rnd(B, D, seed=31), dim=1).requires_grad_(True)
    I = F.normalize(rnd(B, D, seed=32), dim=1).requires_grad_(True)
    ids = torch.randint(0, 3000, (B,), device=DEV)
    res = []
    for _ in range(2):
        U.grad = I.grad = None
        loss = InBatchLossFn.apply(U, I, ids, None, 0.1)
        loss.backward()
        res.append((loss.item(), U.grad.clone(), I.grad.clone()))
    assert res[0][0] == res[1][0] and torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


# ------------------------------------------------------------ bf16 storage of qkv / dqkv
@pytest.mark.parametrize('B,L,p', [(3, 50, 0.0), (4, 33, 0.1), (3, 1, 0.0), (2, 64, 0.0)])
def test_qkv_bf16_storage_is_lossless(B, L, p, bf16_mode):
    """RS_ATTN_QKV_BF16: Q, K, V enter the bf16 attention only as MFMA operands, so bf16 storage
    gives bit-identical out / lse, and dqkv stored as bf16 is the fp32 dqkv rounded (RNE)."""
    d, H = 64, 4
    qkv = rnd(B * L, 3 * d, seed=21)
    lens = torch.randint(1, L + 1, (B,))
    seq = (torch.arange(L)[None, :] < lens[:, None]).long().to(DEV)
    key_pad, _ = ops.seq_mask(seq, 0)
    key = torch.tensor([5, 9], dtype=torch.int64, device=DEV)
    dout = rnd(B * L, d, seed=22)
    q16 = qkv.to(torch.bfloat16)
    o32, l32 = ops.attn_fwd(q16.float(), key_pad, B, L, d, H, p, key, 3)
    o16, l16 = ops.attn_fwd(q16, key_pad, B, L, d, H, p, key, 3)
    assert torch.equal(o32, o16) and torch.equal(l32, l16)
    g32 = ops.attn_bwd(q16.float(), key_pad, o32, dout, l32, B, L, d, H, p, key, 3)
    g16 = ops.attn_bwd(q16, key_pad, o16, dout, l16, B, L, d, H, p, key, 3)
    assert g16.dtype == torch.bfloat16
    assert torch.equal(g16, g32.to(torch.bfloat16))


def test_qkv_bf16_storage_gemms(bf16_mode):
    """The streaming GEMM's bf16-storage instances: bf16 C == fp32 C rounded; bf16 A == fp32 A
    (the kernel rounds fp32 A rows to bf16 in registers); the in_proj weight gradient from bf16
    dqkv == from fp32 dqkv (dW bit-exact, db sums the bf16 values)."""
    M, d = 40960, 64
    x = rnd(M, d, seed=31)
    W, b = rnd(3 * d, d, seed=32) * 0.1, rnd(3 * d, seed=33)
    c32 = ops.linear_fwd(x, W, b)
    c16 = ops.linear_fwd(x, W, b, out_dtype=torch.bfloat16)
    assert c16.dtype == torch.bfloat16 and torch.equal(c16, c32.to(torch.bfloat16))
    dq = rnd(M, 3 * d, seed=34).to(torch.bfloat16)
    base = rnd(M, d, seed=35)
    r32 = ops.linear_bwd_input(dq.float(), W, out=base.clone(), beta=1.0)
    r16_ = ops.linear_bwd_input(dq, W, out=base.clone(), beta=1.0)
    assert torch.equal(r32, r16_)
    dW32, db32 = torch.zeros_like(W), torch.zeros_like(b)
    dW16, db16 = torch.zeros_like(W), torch.zeros_like(b)
    ops.wgrad_bf16(dq.float(), x, dW32, db=db32)
    ops.wgrad_bf16(dq, x, dW16, db=db16)
    assert torch.equal(dW32, dW16)
    assert torch.allclose(db16, db32, atol=1e-3 * db32.abs().max().item())


def test_qkv_bf16_storage_rejected_off_path():
    """bf16 storage outside the bf16 MFMA path fails loudly (no silent conversion)."""
    precision.set_compute_dtype('fp32')
    x = rnd(4096, 64, seed=1)
    W = rnd(192, 64, seed=2)
    with pytest.raises(RuntimeError):
        ops.linear_fwd(x, W, out_dtype=torch.bfloat16)


def test_bf16_step_qkv_storage(monkeypatch):
    """A whole bf16 step with bf16 qkv / dqkv storage against fp32 storage: identical loss and
    gradients except the in_proj bias gradients (column sums of the bf16-rounded dqkv)."""
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
    b = synth.batch_to_torch(synth.make_batch(cfg, 1024, seed=7), DEV)
    res = {}
    precision.set_compute_dtype('bf16')
    try:
        for mode in ('bf16', 'fp32'):
            if mode == 'fp32':
                monkeypatch.setenv('RSYS_QKV_FP32', '1')
            m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'),
                              maps['user'], maps['item'])
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
            m = m.to(DEV)
            f = ensure_flat(m)
            f.zero_grad()
            U, I, H = m(b)
            loss = m.compute_loss(U, I, item_ids=extract_item_id(b['item_tower']), temperature=0.15)
            loss.backward()
            res[mode] = (loss.item(), {k: p.grad.clone() for k, p in m.named_parameters()})
    finally:
        precision.set_compute_dtype('fp32')
    (l1, g1), (l2, g2) = res['bf16'], res['fp32']
    assert l1 == l2
    for k in g1:
        if k.endswith('in_proj_bias'):
            assert torch.allclose(g1[k], g2[k], atol=1e-2 * g2[k].abs().max().item()), k
        elif 'in_proj_bias' not in k:
            # everything upstream of the first layer's in_proj bias sees the same dqkv rounding
            sc = g2[k].abs().max().item()
            assert (g1[k] - g2[k]).abs().max().item() <= 1e-5 * max(sc, 1e-30), k
