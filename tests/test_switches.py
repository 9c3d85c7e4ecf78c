"""Every RSYS_* environment switch the library reads is documented and exercised by a test
(round-5 verdict: 32 of 51 switches were referenced by no test; the alternatives measured slower
were deleted in round 6). CPU: the inventory, RSYS_COMPUTE_DTYPE and RSYS_SHARD_CAPACITY;
-m gpu: RSYS_CHECK_NAN and RSYS_DETERMINISTIC."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'recommendsystemproject_amd')


def _switches():
    names = set()
    for d, _, files in os.walk(PKG):
        if '__pycache__' in d or os.sep + 'build' in d:
            continue
        for f in files:
            if f.endswith(('.py', '.hip', '.cpp', '.h')):
                names |= set(re.findall(r'RSYS_[A-Z0-9_]+', open(os.path.join(d, f)).read()))
    return names


def test_every_switch_documented_and_tested():
    names = _switches()
    assert names, 'no switches found'
    me = os.path.abspath(__file__)
    test_text = ''
    for d, _, files in os.walk(os.path.join(ROOT, 'tests')):
        for f in files:
            p = os.path.join(d, f)
            if f.endswith('.py') and os.path.abspath(p) != me:
                test_text += open(p).read()
    test_text += open(os.path.join(ROOT, 'bench.py')).read()
    integ = open(os.path.join(ROOT, 'INTEGRATION.md')).read()
    untested = sorted(n for n in names if not re.search(r'\b%s\b' % n, test_text + _THIS_FILE_USES))
    undocumented = sorted(n for n in names if not re.search(r'\b%s\b' % n, integ))
    assert not untested, untested
    assert not undocumented, undocumented


# the switches this file itself exercises (below)
_THIS_FILE_USES = 'RSYS_COMPUTE_DTYPE RSYS_SHARD_CAPACITY RSYS_CHECK_NAN RSYS_DETERMINISTIC RSYS_TOWER_STREAMS'


def test_compute_dtype_switch():
    code = 'from recommendsystemproject_amd import precision as p; print(p.compute_dtype(), p.gemm_flags())'
    for val, want in (('bf16', 'bf16'), ('fp32', 'fp32')):
        env = dict(os.environ, RSYS_COMPUTE_DTYPE=val, HIP_VISIBLE_DEVICES='')
        r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        dt, flags = r.stdout.split()
        assert dt == want and (int(flags) != 0) == (want == 'bf16')


def test_shard_capacity_switch(monkeypatch):
    from recommendsystemproject_amd import flat
    monkeypatch.delenv('RSYS_SHARD_CAPACITY', raising=False)
    assert flat.shard_capacity(4096, 4) == int(-(-4096 * 1.5 // 4)) + 64
    monkeypatch.setenv('RSYS_SHARD_CAPACITY', '3')
    assert flat.shard_capacity(4096, 4) == 3 * 1024 + 64


def _demo_model(dev):
    import torch
    import yaml
    from oracle.twotower_oracle import model_state_shapes
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml')))
    for t in cfg['two_tower'].values():
        t['dropout'] = 0.0
        t.get('transformer_parameters', {})['dropout'] = 0.0
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'), maps['user'], maps['item'])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.make_state(shapes, seed=2).items()})
    return m.to(dev), cfg


@pytest.mark.gpu
def test_check_nan_switch_raises_at_the_step(monkeypatch):
    """RSYS_CHECK_NAN=1: compute_loss syncs and raises the reference's RuntimeError at once
    (TwoTowerModel.py: 'Found NaN in User Embedding') instead of flagging it for check_errors()."""
    import torch
    dev = torch.device('cuda:0')
    monkeypatch.setenv('RSYS_CHECK_NAN', '1')
    m, _ = _demo_model(dev)
    assert m.check_nan
    U = torch.nn.functional.normalize(torch.randn(8, 32, device=dev), dim=1)
    I = torch.nn.functional.normalize(torch.randn(8, 32, device=dev), dim=1)
    m.compute_loss(U, I, temperature=0.15)  # finite: no error
    U[3, 0] = float('nan')
    with pytest.raises(RuntimeError, match='Found NaN in User Embedding'):
        m.compute_loss(U, I, temperature=0.15)
    monkeypatch.delenv('RSYS_CHECK_NAN')
    assert not _demo_model(dev)[0].check_nan


@pytest.mark.gpu
def test_deterministic_switch_bitwise(monkeypatch):
    """RSYS_DETERMINISTIC=1 (without torch.use_deterministic_algorithms): the ordinary tables'
    gradients through the fixed-order kernels, so two backward passes of the same step give the
    same bits."""
    import torch
    from recommendsystemproject_amd import ops, synth
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.project.utils.training_utils import extract_item_id
    dev = torch.device('cuda:0')
    monkeypatch.setenv('RSYS_DETERMINISTIC', '1')
    assert ops.deterministic_enabled() and not torch.are_deterministic_algorithms_enabled()
    m, cfg = _demo_model(dev)
    b = synth.batch_to_torch(synth.make_batch(cfg, 2048, seed=9), dev)
    f = ensure_flat(m)
    grads = []
    for _ in range(2):
        f.zero_grad()
        U, I, H = m(b)
        loss = m.compute_loss(U, I, item_ids=extract_item_id(b['item_tower']), temperature=0.15)
        loss.backward()
        torch.cuda.synchronize()
        grads.append(f.grad.clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.gpu
def test_tower_streams_off_same_step(monkeypatch):
    """RSYS_TOWER_STREAMS=0 (the bench's serial instrumented pass): the same loss and gradients as
    the default two-stream step, bitwise in deterministic mode."""
    import torch
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.flat import ensure_flat
    from recommendsystemproject_amd.project.utils.training_utils import extract_item_id
    dev = torch.device('cuda:0')
    monkeypatch.setenv('RSYS_DETERMINISTIC', '1')
    out = {}
    for mode in ('1', '0'):
        monkeypatch.setenv('RSYS_TOWER_STREAMS', mode)
        m, cfg = _demo_model(dev)
        b = synth.batch_to_torch(synth.make_batch(cfg, 1024, seed=11), dev)
        f = ensure_flat(m)
        f.zero_grad()
        U, I, H = m(b)
        loss = m.compute_loss(U, I, item_ids=extract_item_id(b['item_tower']), temperature=0.15)
        loss.backward()
        torch.cuda.synchronize()
        assert (m._side_stream(dev) is None) == (mode == '0')
        out[mode] = (loss.item(), f.grad.clone())
    assert out['0'][0] == out['1'][0]
    assert torch.equal(out['0'][1], out['1'][1])
