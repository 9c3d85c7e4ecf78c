"""Recall@K on the device (reference validate(), training_utils.py:121-275):
rs_topk_rows against a numpy restatement of torch.topk (value descending; ties -> lower column,
which torch leaves unspecified), rs_mask_history against the reference's per-user masking loop
(:238-252), the chunked catalog path against one chunk, and validate() end to end against a
torch restatement of the reference's loop. Integer-valued embeddings make every score exact in
fp32 whatever the GEMM's summation order, so index sets and orders compare bit-exactly."""
import os

import numpy as np
import pytest
import torch
import yaml

from recommendsystemproject_amd import _hip, ops
from recommendsystemproject_amd.project.utils.training_utils import (_history_csr, retrieval_topk,
                                                                      to_device, validate)

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def np_topk(S, K):
    """Per row: the K largest, descending, ties by lower column (stable argsort of -S)."""
    order = np.argsort(-S, axis=1, kind='stable')[:, :K]
    return order, np.take_along_axis(S, order, axis=1)


def dev_topk(S, K, col_offset=0):
    B, N = S.shape
    idx = torch.empty(B, K, dtype=torch.int32, device=DEV)
    val = torch.empty(B, K, dtype=torch.float32, device=DEV)
    _hip.call('rs_topk_rows', S.data_ptr(), int(S.stride(0)), B, N, K, None, 0, col_offset, idx.data_ptr(),
              val.data_ptr(), K, ops.stream())
    return idx.cpu().numpy(), val.cpu().numpy()


@pytest.mark.parametrize('N,K', [(1, 1), (7, 7), (100, 10), (1000, 20), (1000, 256), (70001, 50),
                                 (300, 256)])
def test_topk_distinct(N, K):
    rng = np.random.default_rng(N + K)
    B = 37
    S = rng.standard_normal((B, N)).astype(np.float32)
    S[0] = -np.abs(S[0])  # all-negative row
    idx, val = dev_topk(torch.from_numpy(S).to(DEV), K)
    ri, rv = np_topk(S, K)
    assert np.array_equal(idx, ri)
    assert np.array_equal(val, rv)


@pytest.mark.parametrize('N,K', [(500, 20), (4096, 256), (64, 64)])
def test_topk_ties_and_inf(N, K):
    rng = np.random.default_rng(N)
    B = 19
    S = rng.integers(-3, 4, (B, N)).astype(np.float32)  # heavy ties
    S[1] = 0.0  # one value everywhere: the first K columns
    S[2, ::2] = -np.inf
    S[3] = -np.inf  # fully masked row still yields K columns (lowest indices)
    S[4, 5] = np.inf
    S[5, :] = -0.0
    S[5, 7] = 0.0  # +0 ranks above -0 in the key order (torch treats them equal; one column)
    idx, val = dev_topk(torch.from_numpy(S).to(DEV), K)
    ri, rv = np_topk(S, K)
    rows = [r for r in range(B) if r != 5]
    assert np.array_equal(idx[rows], ri[rows])
    assert np.array_equal(val[rows], rv[rows])
    assert idx[5, 0] == 7 and np.array_equal(idx[5, 1:], [c for c in range(N) if c != 7][:K - 1])


def test_topk_col_offset_and_idx_in():
    rng = np.random.default_rng(3)
    B, N, K = 8, 600, 30
    S = torch.from_numpy(rng.standard_normal((B, N)).astype(np.float32)).to(DEV)
    idx, _ = dev_topk(S, K, col_offset=1000)
    ri, _ = np_topk(S.cpu().numpy(), K)
    assert np.array_equal(idx, ri + 1000)
    mapping = torch.from_numpy(rng.permutation(10 ** 6)[:B * N].reshape(B, N).astype(np.int32)).to(DEV)
    out = torch.empty(B, K, dtype=torch.int32, device=DEV)
    _hip.call('rs_topk_rows', S.data_ptr(), N, B, N, K, mapping.data_ptr(), N, 0, out.data_ptr(), None, K,
              ops.stream())
    assert np.array_equal(out.cpu().numpy(), np.take_along_axis(mapping.cpu().numpy(), ri, axis=1))


def test_topk_bad_args():
    S = torch.zeros(2, 10, device=DEV)
    out = torch.empty(2, 300, dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError):
        _hip.call('rs_topk_rows', S.data_ptr(), 10, 2, 10, 11, None, 0, 0, out.data_ptr(), None, 11, ops.stream())
    with pytest.raises(RuntimeError):
        _hip.call('rs_topk_rows', S.data_ptr(), 10, 2, 10, 257, None, 0, 0, out.data_ptr(), None, 300,
                  ops.stream())


def _history(rng, U, N, max_len=40):
    """user -> catalog item ids (= column + 100), with the reference's filters exercised:
    ids above the catalog's max id and ids not in the catalog are skipped."""
    hist = {}
    for u in range(U):
        if rng.random() < 0.2:
            continue  # user without history
        h = list(rng.integers(100, 100 + N, rng.integers(0, max_len)))
        h += [10 ** 7, 5]  # > max id; not in the catalog
        hist[u] = set(int(x) for x in h)
    return hist


def _mask_reference(S, users, hist, item_ids):
    """training_utils.py:238-252 restated with numpy (scores[i, indices[valid]] = -inf)."""
    S = S.copy()
    max_id = int(item_ids.max())
    id_to_index = np.full(max_id + 1, -1)
    id_to_index[item_ids] = np.arange(len(item_ids))
    for i, u in enumerate(users):
        if u in hist:
            valid = [x for x in hist[u] if x <= max_id]
            if valid:
                ind = id_to_index[np.asarray(valid)]
                S[i, ind[ind >= 0]] = -np.inf
    return S


def test_mask_history_matches_reference_loop():
    rng = np.random.default_rng(5)
    B, N, U = 64, 3000, 50
    item_ids = np.arange(100, 100 + N)
    hist = _history(rng, U, N)
    users = rng.integers(0, U + 5, B)  # some users beyond the history table
    S = rng.standard_normal((B, N)).astype(np.float32)
    ref = _mask_reference(S, users, hist, item_ids)
    off, idx, nu = _history_csr(hist, item_ids, DEV)
    u_dev = torch.from_numpy(users).to(DEV)
    for c0, n in ((0, N), (0, 1024), (1024, 1024), (2048, N - 2048)):  # whole row and column chunks
        St = torch.from_numpy(np.ascontiguousarray(S[:, c0:c0 + n])).to(DEV)
        _hip.call('rs_mask_history', St.data_ptr(), n, B, c0, n, u_dev.data_ptr(), 1, off.data_ptr(),
                  idx.data_ptr(), nu, ops.stream())
        assert np.array_equal(St.cpu().numpy(), ref[:, c0:c0 + n])


@pytest.mark.parametrize('chunk', [100000, 1000, 999])
def test_retrieval_topk_chunked(chunk):
    rng = np.random.default_rng(7)
    B, N, D, K = 48, 5000, 64, 20
    Ue = rng.integers(-3, 4, (B, D)).astype(np.float32)
    Ie = rng.integers(-3, 4, (N, D)).astype(np.float32)
    item_ids = np.arange(100, 100 + N)
    hist = _history(rng, 40, N, max_len=300)
    users = rng.integers(0, 40, B)
    S = _mask_reference(Ue @ Ie.T, users, hist, item_ids)  # exact integers
    ri, _ = np_topk(S, K)
    out = retrieval_topk(torch.from_numpy(Ue).to(DEV), torch.from_numpy(Ie).to(DEV), K,
                         torch.from_numpy(users).to(DEV), _history_csr(hist, item_ids, DEV), chunk=chunk)
    assert np.array_equal(out.cpu().numpy(), ri)


def test_host_tensors_fail_loudly():
    """ids handed to the towers by pointer must be on the device (no illegal access)."""
    from oracle.twotower_oracle import model_state_shapes  # noqa: F401
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml')))
    tower = GenericTower(cfg, 'item_tower').to(DEV)
    rng = np.random.default_rng(0)
    tb = synth.batch_to_torch(synth.make_tower_batch(cfg['two_tower']['item_tower'], 8, rng))
    with pytest.raises(_hip.HipError):
        tower(tb, synth.tower_layout(cfg['two_tower']['item_tower']))


def test_validate_matches_reference_loop():
    """validate() on a small model: loss and Recall@{1,10,50} against the reference's loop
    restated in torch on the same embeddings."""
    from oracle.twotower_oracle import model_state_shapes
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'demo.yaml')))
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
    state = synth.make_state(shapes, seed=2)
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'), maps['user'], maps['item'])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    m = m.to(DEV)
    it = cfg['two_tower']['item_tower']
    V = int(it['sparse_features'][0]['vocab_size'])
    rng = np.random.default_rng(9)
    # item index: every item once, in batches of 256 (catalog column = item id - 1)
    item_loader = []
    for s in range(1, V, 256):
        ids = np.arange(s, min(V, s + 256))
        tb = synth.make_tower_batch(it, len(ids), rng, ids_override={it['sparse_features'][0]['name']: ids})
        item_loader.append(synth.batch_to_torch(tb))  # host tensors: validate() moves them
    loader, meta = [], []
    for i in range(3):
        b = synth.make_batch(cfg, 128, seed=20 + i)
        loader.append(synth.batch_to_torch(b))
        meta.append({'user_tower': {'sparse': torch.from_numpy(rng.integers(0, 60, (128, 1)))}})
    hist = {u: set(int(x) for x in rng.integers(1, V, 30)) for u in range(50)}
    loss, acc = validate(m, loader, item_loader, DEV, epoch=None, k_list=[1, 10, 50], meta_data_loader=meta,
                         log_embeddings=False, user_history=hist)
    # the reference's loop (training_utils.py:150-275) in torch, same model and batches
    m.eval()
    with torch.no_grad():
        embs = torch.cat([m.get_item_embeddings(to_device(b, DEV)) for b in item_loader])
        all_ids = torch.cat([b['sparse'][:, 0] for b in item_loader]).to(DEV)
        tot, hits, n = 0.0, {k: 0 for k in (1, 10, 50)}, 0
        for b, mb in zip(loader, meta):
            bd = to_device(b, DEV)
            U, I, H = m(bd)
            tg = bd['item_tower']['sparse'][:, 0]
            tot += m.compute_loss(U, I, hard_neg_emb=H, item_ids=tg).item()
            S = (U.double() @ embs.double().t()).cpu().numpy()
            S = _mask_reference(S, mb['user_tower']['sparse'][:, 0].numpy(), hist, all_ids.cpu().numpy())
            S = torch.from_numpy(S)
            for k in hits:
                top = torch.topk(S, k, dim=1).indices
                hits[k] += (all_ids.cpu()[top] == tg.cpu().view(-1, 1)).any(dim=1).sum().item()
            n += len(tg)
    assert abs(loss - tot / len(loader)) < 1e-5
    # fp64 scores vs the device's fp32: a near-tie at the k-th place could move one hit
    for k in hits:
        assert abs(acc[k] - hits[k] / n) <= 1.0 / n, (k, acc[k], hits[k] / n)
    assert acc[50] >= acc[10] >= acc[1]


def test_validate_matches_reference_fixture():
    """validate() against the reference's OWN validate() (tests/golden/validate_demo.npz, made by
    make_validate_golden.py): same weights (synth seed 3 + the fixture's running statistics), same
    item index, batches, metadata loader and user history; loss to 1e-4, Recall@{1,5,10} to one
    hit (a near-tie at the k-th place between the CPU and the device scores could move one)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    import golden_util as gu
    from recommendsystemproject_amd import synth
    from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower
    from recommendsystemproject_amd.project.models.TwoTower.TwoTowerModel import TwoTowerModel
    cfg, meta, data = gu.load(os.path.join(ROOT, 'tests', 'golden', 'validate_demo.npz'))
    bn = dict(np.load(os.path.join(ROOT, 'tests', 'golden', 'validate_demo_bn.npz')))
    maps = {'user': synth.tower_layout(cfg['two_tower']['user_tower']),
            'item': synth.tower_layout(cfg['two_tower']['item_tower'])}
    m = TwoTowerModel(GenericTower(cfg, 'user_tower'), GenericTower(cfg, 'item_tower'), maps['user'], maps['item'])
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}  # the reference's key order
    state = synth.make_state(shapes, seed=int(meta['weight_seed']))
    state.update(bn)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    m = m.to(DEV)
    item_loader = [synth.batch_to_torch(gu.unflatten_batch(data, f'items/{j}')) for j in range(meta['item_batches'])]
    loader = [synth.batch_to_torch(gu.unflatten_batch(data, f'val/{i}')) for i in range(meta['val_batches'])]
    meta_loader = [{'user_tower': {'sparse': torch.from_numpy(data[f'uid/{i}'])}} for i in range(meta['val_batches'])]
    users, offs, items = data['hist/users'], data['hist/offs'], data['hist/items']
    hist = {int(u): set(int(x) for x in items[offs[i]:offs[i + 1]]) for i, u in enumerate(users)}
    k_list = list(meta['k_list'])
    loss, acc = validate(m, loader, item_loader, DEV, epoch=None, k_list=k_list, meta_data_loader=meta_loader,
                         log_embeddings=False, user_history=hist)
    n = sum(int(b['item_tower']['sparse'].shape[0]) for b in loader)
    assert abs(loss - float(data['loss'])) < 1e-4, (loss, float(data['loss']))
    for k, want in zip(k_list, data['recall']):
        assert abs(acc[k] - float(want)) <= 1.0 / n + 1e-12, (k, acc[k], float(want))
