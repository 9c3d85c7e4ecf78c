"""CPU-only tests: C-ABI library loads and exports every declared symbol, the drop-in modules
keep the reference's state_dict layout, host-side planning logic, synthetic data contract."""
import os
import re

import numpy as np
import pytest
import torch
import yaml

from oracle.twotower_oracle import model_state_shapes
from recommendsystemproject_amd import _hip, synth
from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'rsys_hip.h')
CONFIGS = ['demo', 'c1', 'c2', 'root', 'c3']


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(rs_[a-z0-9_]+)\s*\(', src)))


def test_header_and_binding_agree():
    syms = header_symbols()
    assert len(syms) > 20
    assert sorted(_hip.SIGNATURES) == syms


def test_library_loads_and_exports_everything():
    L = _hip.lib()  # no GPU needed to load
    for s in header_symbols():
        assert hasattr(L, s), s
    assert L.rs_version() >= 1
    # host-only queries work without a device
    assert L.rs_gemm_auto_split(192, 64, 204800) > 1
    assert L.rs_gemm_auto_split(204800, 192, 64) == 1
    assert L.rs_colsum_ws_bytes(4096, 64) > 0


def test_bad_arguments_report_errors_without_gpu():
    with pytest.raises(_hip.HipError, match='negative size'):
        _hip.call('rs_gemm_f32', 0, 0, -1, 4, 4, 1.0, None, 4, None, 4, 0.0, None, 4, 0, None, None,
                  0, 0, 0.0, None, 0, 0, None, 1, None, None)
    with pytest.raises(_hip.HipError, match='head_dim'):
        _hip.call('rs_attn_fwd', 1, 1, 1, 1, 2, 5, 60, 4, 1.0, 0.0, None, 0, 0, None, None)


@pytest.mark.parametrize('name', CONFIGS)
def test_state_dict_layout_matches_reference_layout(name):
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', f'{name}.yaml')))
    if name == 'c3':  # 10M-row tables: layout only, keep it cheap
        for t in cfg['two_tower'].values():
            for f in t.get('sparse_features', []):
                f['vocab_size'] = min(f['vocab_size'], 1000)
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'))
    got = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    want = [(k, tuple(s)) for k, s, _ in model_state_shapes(cfg)]
    assert got == want


def test_param_count_demo_schema():
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml')))
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'))
    assert sum(p.numel() for p in m.parameters()) == 886540  # SURVEY §8b (measured on the reference)


@pytest.mark.skipif(not os.path.isdir('/root/reference'), reason='reference only in the build container')
def test_initial_weights_identical_to_reference_under_same_seed():
    import sys
    sys.path.insert(0, '/root/reference')
    from project.models.TwoTower.GenericTower import GenericTower as RG
    from project.models.TwoTower.TwoTowerModel import TwoTowerModel as RM
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml')))
    torch.manual_seed(11)
    ref = RM(RG(cfg, 'user_tower'), RG(cfg, 'item_tower')).state_dict()
    torch.manual_seed(11)
    ours = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower')).state_dict()
    for k in ref:
        assert torch.equal(ref[k], ours[k]), k


def test_cpu_tensors_fail_loudly():
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c1.yaml')))
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'))
    b = synth.batch_to_torch(synth.make_batch(cfg, 8, seed=0))
    with pytest.raises(_hip.HipError, match='MI355X only'):
        m(b)


def test_synthetic_batch_contract():
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml')))
    b = synth.make_batch(cfg, 64, seed=3, edge_cases=True, n_hard=2)
    u, it = b['user_tower'], b['item_tower']
    assert u['sparse'].shape == (64, 5) and u['sparse'].dtype == np.int64
    assert u['dense'].shape == (64, 1) and u['dense'].dtype == np.float32
    assert u['sequence']['hist_movie_ids'].shape == (64, 20)
    assert u['sequence']['hist_genre_ids'].shape == (64, 20, 3)
    assert (u['sequence']['hist_movie_ids'][0] == 0).all()           # all-padding history row (T6/T7)
    assert it['sparse'][1, 0] == it['sparse'][2, 0] == it['sparse'][3, 0]   # collisions (T12)
    assert it['sequence']['genre_ids'].shape == (64, 3)
    assert len(b['hard_negatives']) == 2
    hist = u['sequence']['hist_movie_ids']
    valid = hist != 0   # right-padded: valid prefix
    assert (np.sort(~valid, axis=1) == ~valid).all()
    maps = synth.tower_layout(cfg['two_tower']['item_tower'])
    assert maps == {'sparse': {'movie_id_enc': 0, 'release_year_enc': 1}, 'dense': {},
                    'sequence': {'genre_ids': 'genre_ids'}}


def test_history_csr_filters_like_reference():
    """validate()'s history mask input (training_utils.py:238-252): per user the catalog
    columns of their items; ids above the catalog's max id or not in it are dropped."""
    from recommendsystemproject_amd.project.utils.training_utils import _history_csr
    item_ids = np.array([10, 11, 13, 20])  # column = position
    hist = {0: {10, 13, 99}, 2: {12, 20, 11}, 3: set()}
    off, idx, U = _history_csr(hist, item_ids, 'cpu')
    assert U == 4
    off, idx = off.numpy(), idx.numpy()
    rows = [sorted(idx[off[u]:off[u + 1]].tolist()) for u in range(U)]
    assert rows == [[0, 2], [], [1, 3], []]


def test_host_code_under_asan():
    """The host side of the C-ABI (argument checks, launch planning, workspace sizing, job tables)
    under AddressSanitizer: tests/asan_harness.py in a subprocess against librsys_hip_asan.so
    (csrc/Makefile target `asan`, host-only ASan build), with the clang ASan runtime preloaded."""
    import glob
    import subprocess
    import sys
    lib = os.path.join(ROOT, 'recommendsystemproject_amd', '_lib', 'librsys_hip_asan.so')
    if not os.path.exists(lib):
        subprocess.run(['make', '-C', os.path.join(ROOT, 'recommendsystemproject_amd', 'csrc'), 'asan', '-j8'],
                       check=True, capture_output=True)
    rt = sorted(glob.glob('/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so'))
    if not rt:
        pytest.skip('clang ASan runtime not found')
    env = dict(os.environ, RSYS_LIB_PATH=lib, LD_PRELOAD=rt[-1], HIP_VISIBLE_DEVICES='',
               ASAN_OPTIONS='detect_leaks=0:abort_on_error=1:verify_asan_link_order=0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'asan_harness.py')], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and 'asan harness ok' in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert 'ERROR: AddressSanitizer' not in r.stderr


def test_custom_ops_registered_with_fake_impls():
    """library.py registers the two-tower step as torch custom ops (namespace rsys), each with a
    backward op; the loss op's fake implementation gives its shapes without a device."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    from recommendsystemproject_amd import library  # noqa: F401  (registers torch.ops.rsys.*)
    for n in ('seq_encoder', 'seq_features', 'tower_features', 'tower_chain', 'batch_norm', 'mlp_tower',
              'inbatch_softmax_loss'):
        assert hasattr(torch.ops.rsys, n) and hasattr(torch.ops.rsys, n + '_backward'), n
    with FakeTensorMode():
        U, I = torch.empty(64, 128), torch.empty(64, 128)
        loss, ticket = torch.ops.rsys.inbatch_softmax_loss(U, I, torch.empty(64, dtype=torch.int64), None, 0.15,
                                                          True)
        assert loss.shape == () and ticket.dtype == torch.int64


def test_catchup_batch_grouping(monkeypatch):
    """flat.catchup_batch: up to 8 calls a launch, one row-width class and one flat buffer per
    launch, and never two calls of one table in a launch (their catch-ups touch the same rows: the
    later call goes in a later launch, in order)."""
    import torch
    from recommendsystemproject_amd import _hip, flat

    class FakeFlat:
        def __init__(self):
            z = torch.zeros(4)
            self.data = z
            self.lazy_opt = {'m': z, 'v': z, 'step_dev': z, 'consts': z, 'hyper': (0.9, 0.999, 1e-8, 0.0)}

    class FakeTable:
        def __init__(self, D, fl):
            self.D, self.flat, self.last = D, fl, torch.zeros(2, dtype=torch.int32)

        def ptr(self, t):
            return t.data_ptr()

    class FakeCall:
        def __init__(self):
            self.keys, self.n, self.catchup_due = torch.zeros(3, dtype=torch.int32), 3, True

    f1, f2 = FakeFlat(), FakeFlat()
    a, b, c, d = FakeTable(128, f1), FakeTable(100, f1), FakeTable(16, f1), FakeTable(128, f2)
    items = [(a, FakeCall()), (b, FakeCall()), (a, FakeCall()), (c, FakeCall()), (d, FakeCall()), (b, FakeCall())]
    launched = []

    def fake_call(name, arr_ptr, n, *rest):
        arr = (_hip.SortedCall * n).from_address(arr_ptr)
        launched.append([next(t for t, cl in items if cl.keys.data_ptr() == arr[j].keys) for j in range(n)])
        return 0
    monkeypatch.setattr(_hip, 'call', fake_call)
    monkeypatch.setattr(flat, '_stream', lambda: None)
    flat.catchup_batch(items)
    assert all(not cl.catchup_due for _, cl in items)
    names = {id(a): 'a', id(b): 'b', id(c): 'c', id(d): 'd'}
    got = [[names[id(t)] for t in g] for g in launched]
    assert got == [['a', 'b'], ['a', 'b'], ['c'], ['d']], got
